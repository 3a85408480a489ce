#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM
bytes for one kernel, with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
counters are in KiB; FETCH_SIZE reports exactly half of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores.

usage: pmc_traffic.py <session dir> <kernel substring> <out.json> [workers values]
"""
import csv
import json
import statistics
import sys


def per_launch(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no dispatch of {kernel!r} in {path}")
    return statistics.median(float(r["Counter_Value"]) for r in rows), len(rows), rows[0]["Kernel_Name"]


def main():
    sess, kernel, out = sys.argv[1], sys.argv[2], sys.argv[3]
    W = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 26_214_400
    fetch_kib, nf, name = per_launch(f"{sess}/pmc_FETCH_SIZE/run_counter_collection.csv", kernel)
    write_kib, nw, _ = per_launch(f"{sess}/pmc_WRITE_SIZE/run_counter_collection.csv", kernel)
    read_b = 2 * fetch_kib * 1024
    write_b = write_kib * 1024
    algo = (W + 1) * n * 4
    res = {"kernel": name, "session": sess.rstrip("/").split("/")[-1] if "/" in sess else sess,
           "workers": W, "values": n, "dispatches": [nf, nw],
           "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
           "hbm_read_bytes": int(read_b), "hbm_write_bytes": int(write_b),
           "hbm_bytes_per_launch": int(read_b + write_b), "algorithmic_bytes": algo,
           "traffic_over_algorithmic": round((read_b + write_b) / algo, 5),
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16B/lane streams); "
                         "write = WRITE_SIZE x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
