#!/usr/bin/env python3
"""Lab: does the physical placement of the packet buffer move the switch?  The same
819,200-packet config-3 batch (worker-major) copied into K separately allocated buffers
(with spacer allocations between them), each run through ina_switch_process
interleaved, one event pair around 5 back-to-back calls; median per buffer.

  python tools/lab/placement_lab.py
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
K = int(os.environ.get("K", 5))
g = torch.Generator(device=dev).manual_seed(1)
packed = []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    packed.append(ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True))
    del b
src = torch.cat([p for p, _ in packed])
ds = torch.cat([d for _, d in packed])
del packed
bufs, spacers = [], []
for k in range(K):
    spacers.append(torch.empty((k + 1) * (37 << 20), dtype=torch.uint8, device=dev))
    bufs.append(src.clone())
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(src.shape[0], dtype=torch.uint8, device=dev)
times = {k: [] for k in range(K)}
for _ in range(int(os.environ.get("ROUNDS", 6))):
    for k, b in enumerate(bufs):
        sw.process(b, acts, desc=ds)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            sw.process(b, acts, desc=ds)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e3 / 5)
print(json.dumps({f"buffer {k} @0x{bufs[k].data_ptr():x}": round(statistics.median(t), 1)
                  for k, t in times.items()}, indent=1))
