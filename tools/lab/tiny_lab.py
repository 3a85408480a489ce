#!/usr/bin/env python3
"""Lab: small switch batches (NGA-32, 16,384-slot pool, 8 workers per slot) per batch size
through the one-launch path (k_switch_tiny: sort + run in one workgroup), the two-launch
one-workgroup sort + run kernel, and the multi-launch bucket sort + run kernel;
interleaved, HIP events, median.

  python tools/lab/tiny_lab.py
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
V, W, slots = 32, 8, 16384
g = torch.Generator(device=dev).manual_seed(5)
sizes = [16, 64, 128, 256, 512, 1024, 2048, 4096]
streams = {}
for n in sizes:
    per = max(1, n // W)
    vals = [torch.randint(-(1 << 20), 1 << 20, (per * V,), dtype=torch.int32, device=dev, generator=g)
            for _ in range(W)]
    streams[n] = torch.cat([ops.pack_nga(v, V, w + 1, W, 1, 1, num_slots=slots) for w, v in enumerate(vals)])
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(max(s.shape[0] for s in streams.values()), dtype=torch.uint8, device=dev)
MODES = {"one launch": dict(switch_small_sort=2048, switch_tiny_max=2048),
         "two launches": dict(switch_small_sort=2048, switch_tiny_max=0),
         "bucket sort": dict(switch_small_sort=False, switch_tiny_max=0)}
times = {(n, t): [] for n in sizes for t in MODES}
ref = {}
for _ in range(int(os.environ.get("ROUNDS", 8))):
    for n in sizes:
        for t, kw in MODES.items():
            ops.set_tuning(**kw)
            st = streams[n]
            a = acts[: st.shape[0]]
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                sw.process(st, a)
                e1.record()
                torch.cuda.synchronize()
                times[(n, t)].append(e0.elapsed_time(e1) * 1e3)
            if (n, t) not in ref:
                ref[(n, t)] = a.clone()
ops.set_tuning(switch_small_sort=True, switch_tiny_max=128)
for n in sizes:
    assert all(torch.equal(ref[(n, "one launch")], ref[(n, t)]) for t in MODES), n
print(json.dumps({f"{n} packets": {t: round(statistics.median(times[(n, t)]), 1) for t in MODES}
                  for n in sizes}, indent=1))
