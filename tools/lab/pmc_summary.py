#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
for d in sorted(glob.glob(f"{root}/*_p*")):
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            if pat and pat not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"][:40], r["Dispatch_Id"])
            acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
        for k, cs in acc.items():
            out = []
            for c, vals in sorted(cs.items()):
                per = defaultdict(float)
                for di, v in vals:
                    per[di] += v
                out.append(f"{c}={sum(per.values()) / len(per):.4g}")
            print(d.split('/')[-1], k, " ".join(out))
