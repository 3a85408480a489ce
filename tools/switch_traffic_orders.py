#!/usr/bin/env python3
"""HBM traffic of the device switch per arrival order, for bench.py's switch legs
(profiles/traffic_switch_v<V>.json, read by bench._switch_traffic): from gpu_session.sh's
`swtrace:<env>` (kernel trace) and `swpmc:<env>` (FETCH_SIZE and WRITE_SIZE, separate passes)
stages over tools/prof_switch.py, with the gfx950 corrections of MI355X_MICROARCH.md (counters
in KiB; FETCH_SIZE doubled -- half-count of 16 B/lane streams).  Per order: every switch
kernel's bytes, the run kernel's, and the call's measured bytes / its algorithmic bytes.

usage: switch_traffic_orders.py <session dir> <out.json> <V> <algorithmic bytes> ORDER=VARIANT ...
  e.g. shuffled_split=V_32_SLOTS_1048576_ORDER_random_SPLIT_1"""
import csv
import json
import statistics
import sys

from switch_traffic import counters, short


def main():
    sess, out, V, algo = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    doc = {"source": (f"tools/gpu_session.sh session {sess.rstrip('/').split('/')[-1]}: swtrace + swpmc "
                      "(FETCH_SIZE, WRITE_SIZE: separate rocprofv3 --pmc passes) over tools/prof_switch.py"),
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16B/lane streams); write = WRITE_SIZE x 1024",
           "V": V, "orders": {}}
    for spec in sys.argv[5:]:
        order, var = spec.split("=", 1)
        us = {short(r["Name"]): float(r["AverageNs"]) / 1e3
              for r in csv.DictReader(open(f"{sess}/swtrace_{var}/run_kernel_stats.csv"))}
        fetch = counters(f"{sess}/swpmc_{var}_FETCH_SIZE/run_counter_collection.csv")
        write = counters(f"{sess}/swpmc_{var}_WRITE_SIZE/run_counter_collection.csv")
        kernels = {}
        for k in fetch:
            if k not in write or "pack_nga" in k:
                continue
            kernels[k] = {"avg_us": round(us.get(k, 0.0), 1), "hbm_read_bytes": int(2 * fetch[k] * 1024),
                          "hbm_write_bytes": int(write[k] * 1024)}
        run = max((k for k in kernels if "k_switch_run" in k), key=lambda k: kernels[k]["avg_us"])
        total = sum(v["hbm_read_bytes"] + v["hbm_write_bytes"] for v in kernels.values())
        r = kernels[run]
        doc["orders"][order] = {
            "kernel": run, "avg_us": r["avg_us"], "hbm_read_bytes": r["hbm_read_bytes"],
            "hbm_write_bytes": r["hbm_write_bytes"], "algorithmic_bytes": algo,
            "traffic_ratio": round(total / algo, 3),
            "switch_kernels": kernels, "variant": var,
            "note": ("traffic_ratio = every switch kernel's measured HBM bytes (sort passes included) / "
                     "the call's algorithmic bytes (bench.py measure_switch)")}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({k: {"run_us": v["avg_us"], "traffic_ratio": v["traffic_ratio"]} for k, v in doc["orders"].items()}))


if __name__ == "__main__":
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    main()
