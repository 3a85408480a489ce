#!/usr/bin/env python3
"""Median duration (µs) per (kernel, grid size) of a rocprofv3 --kernel-trace CSV, for the
kernels whose name contains any filter.  usage: trace_by_grid.py <run_kernel_trace.csv> [filter ...]"""
import collections
import csv
import statistics
import sys


def main():
    path, filt = sys.argv[1], sys.argv[2:]
    groups = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        if filt and not any(f in name for f in filt):
            continue
        grid = int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0)
        groups[(name.split("(")[0][-60:], grid)].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    for (name, grid), ds in sorted(groups.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        print(f"{name:60s} grid={grid:9d} blocks={grid // 1024:6d} n={len(ds):4d} median_us={statistics.median(ds):8.2f}")


if __name__ == "__main__":
    main()
