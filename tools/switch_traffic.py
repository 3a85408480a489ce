#!/usr/bin/env python3
"""Per-kernel HBM bytes and rates of the device switch program (tools/prof_switch.py)
from one gpu_session.sh `swprof` stage: the kernel-trace stats plus the two --pmc
passes (FETCH_SIZE, WRITE_SIZE), with the gfx950 corrections of MI355X_MICROARCH.md
(counters in KiB; FETCH_SIZE doubled -- half-count of 16 B/lane streams).

usage: switch_traffic.py <session dir> <out.json> [session tag] [variant]
  variant (e.g. SPLIT_1): read the `swtrace:<env>` / `swpmc:<env>` stages' directories
  (swtrace_<variant>, swpmc_<variant>_FETCH_SIZE, swpmc_<variant>_WRITE_SIZE) instead of swprof's
"""
import csv
import json
import re
import statistics
import sys


def short(name: str) -> str:
    """'void ina::k_rs_scatter<true>(unsigned int const*, ...)' -> 'ina::k_rs_scatter<true>'."""
    name = re.sub(r"^void ", "", name)
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def counters(path):
    per = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k.startswith("ina::"):
            per.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in per.items()}


def main():
    sess, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else sess.rstrip("/").split("/")[-1]
    var = sys.argv[4] if len(sys.argv) > 4 else ""
    tr, pm = (f"swtrace_{var}", f"swpmc_{var}_") if var else ("swprof", "swpmc_")
    us = {short(r["Name"]): float(r["AverageNs"]) / 1e3
          for r in csv.DictReader(open(f"{sess}/{tr}/run_kernel_stats.csv"))}
    fetch = counters(f"{sess}/{pm}FETCH_SIZE/run_counter_collection.csv")
    write = counters(f"{sess}/{pm}WRITE_SIZE/run_counter_collection.csv")
    kernels = {}
    for k in sorted(fetch, key=lambda k: -us.get(k, 0.0)):
        if k not in us or k not in write:
            continue
        rd, wr = int(2 * fetch[k] * 1024), int(write[k] * 1024)
        kernels[k] = {"avg_us": round(us[k], 1), "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                      "TB_per_s": round((rd + wr) / (us[k] * 1e-6) / 1e12, 2)}
    doc = {
        "workload": ("tools/prof_switch.py: 819,200 NGA-256 packets (8 workers x 102,400 slots, "
                     f"2^17-slot pool), session {tag}" + (f", env {var}" if var else "")),
        "correction": ("read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16B/lane streams); "
                       "write = WRITE_SIZE x 1024"),
        "kernels": kernels,
    }
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
