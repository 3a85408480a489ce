#!/usr/bin/env python3
"""Lab: does the distance between the W workers' packet regions matter to the switch?
Worker-major batches put a slot's W packets exactly N x 1040 bytes apart (N = 102,400
packets per worker: a multiple of 64 KiB), so if HBM channels interleave below that
distance all W rows of a segment may sit in one channel.  Here `gap` foreign packets
(another switch's id: forwarded untouched, FWD_OTHER) are inserted between the workers'
regions, shifting region w by w x gap rows; the same 819,200 data packets go through
ina_switch_process (descriptor keys) for each gap.  Interleaved, HIP events, median.

  python tools/lab/region_gap_lab.py
"""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
n, W, V, slots = 26_214_400, 8, 256, 1 << 17
GAPS = [int(x) for x in os.environ.get("GAPS", "0,1,3,4,17,64").split(",")]
g = torch.Generator(device=dev).manual_seed(1)
packed = []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    packed.append(ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True))
    del b
npk_w, stride = packed[0][0].shape
foreign = ops.pack_nga(torch.zeros(V * max(GAPS) + V, dtype=torch.int32, device=dev), V, 1, W, 2, 1,
                       num_slots=slots, desc=True)
cases = {}
for gap in GAPS:
    parts, dparts = [], []
    for w in range(W):
        if w and gap:
            parts.append(foreign[0][:gap])
            dparts.append(foreign[1][:gap])
        parts.append(packed[w][0])
        dparts.append(packed[w][1])
    cases[gap] = (torch.cat(parts), torch.cat(dparts))
del packed
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
times = {gap: [] for gap in GAPS}
done = {}
for _ in range(int(os.environ.get("ROUNDS", 6))):
    for gap, (st, ds) in cases.items():
        acts = torch.empty(st.shape[0], dtype=torch.uint8, device=dev)
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            sw.process(st, acts, desc=ds)
            e1.record()
            torch.cuda.synchronize()
            times[gap].append(e0.elapsed_time(e1) * 1e3)
        done[gap] = int((acts == 1).sum())
print(json.dumps({f"gap {gap} rows": {"median_us": round(statistics.median(t), 1),
                                      "completed": done[gap]} for gap, t in times.items()}, indent=1))
