#!/usr/bin/env python3
"""HBM bytes of the split-row packet path's two kernels (tools/prof_path.py SPLIT=1) from a
gpu_session.sh run with the `pathtrace:SPLIT=1` and `pathpmc:SPLIT=1` stages, against their
algorithmic bytes: the one-launch worker pack (8 workers' fp32 + the shared base read; header
rows, payload rows and descriptors written) and the fused switch + PS pass (header rows of
acks + packets, payload rows, the PS's local parameters read).  gfx950 corrections of
MI355X_MICROARCH.md: counters in KiB, FETCH_SIZE doubled.

usage: path_traffic.py <session dir> <out.json> [session tag]
"""
import csv
import json
import statistics
import sys


def med(path, sub):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    return statistics.median(v), len(v)


def main():
    sess, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else sess.rstrip("/").split("/")[-1]
    us = {r["Name"]: float(r["AverageNs"]) / 1e3
          for r in csv.DictReader(open(f"{sess}/pathtrace_SPLIT_1_TRACE/run_kernel_stats.csv"))}
    W, n, V = 8, 26_214_400, 256
    npk = n // V
    doc = {"workload": ("tools/prof_path.py SPLIT=1: the steady-state INA step in split rows (8 workers x "
                        f"26,214,400 fp32, acks in front, PS fused), session {tag}"),
           "correction": ("read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16B/lane streams); "
                          "write = WRITE_SIZE x 1024"),
           "kernels": {}}
    for sub, algo_r, algo_w in (("k_qpack_nga_multi_split<8>", W * 4 * n + 4 * n, W * npk * (16 + 4 * V) + W * npk * 8),
                                ("k_switch_run2<true, false, true>", (W + 1) * npk * 16 + W * npk * 4 * V + 4 * n,
                                 None)):
        f, nf = med(f"{sess}/pathpmc_SPLIT_1_FETCH_SIZE/run_counter_collection.csv", sub)
        w, nw = med(f"{sess}/pathpmc_SPLIT_1_WRITE_SIZE/run_counter_collection.csv", sub)
        t = [v for k, v in us.items() if sub in k]
        d = {"dispatches": [nf, nw], "hbm_read_bytes": int(2 * f * 1024), "hbm_write_bytes": int(w * 1024),
             "avg_us": round(t[0], 1) if t else None,
             "algorithmic_read_bytes": algo_r, "read_over_algorithmic": round(2 * f * 1024 / algo_r, 4)}
        if algo_w:
            d["algorithmic_write_bytes"] = algo_w
            d["write_over_algorithmic"] = round(w * 1024 / algo_w, 4)
        doc["kernels"][sub] = d
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
