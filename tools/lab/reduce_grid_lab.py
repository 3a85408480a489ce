#!/usr/bin/env python3
"""Lab: the headline W = 8 reduce (config 3) against grids up to one 16-byte chunk per
worker per thread (no grid-stride loop: 25,600 workgroups), next to the r01 rule (512
workgroups x 4 chunks per stream).  Back-to-back launches over two alternating input
sets (the bench's timing), HIP events around 20 launches, interleaved rounds, median.
(experiment only: ops.set_tuning(reduce_blocks, unroll))"""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
n, W = 26_214_400, 8
sets = [[torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev) for _ in range(W)]
        for _ in range(2)]
outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
ref = ops.sum_reduce(sets[0])
VARIANTS = [(0, 0)] + [(u, b) for u in (1, 2, 4) for b in (512, 1024, 4096, 8192, 25600, 51200)]
res = {}
s = torch.cuda.current_stream()
for rnd in range(int(os.environ.get("ROUNDS", 4))):
    for u, b in VARIANTS:
        ops.set_tuning(unroll=u, reduce_blocks=b)
        for i in range(4):
            ops.sum_reduce(sets[i % 2], out=outs[i % 2])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(20):
            ops.sum_reduce(sets[i % 2], out=outs[i % 2])
        e1.record(s)
        torch.cuda.synchronize()
        res.setdefault(f"U{u}/{b or 'rule'}", []).append(e0.elapsed_time(e1) * 1e3 / 20)
        assert torch.equal(outs[0], ref)
ops.set_tuning(unroll=0, reduce_blocks=0)
out = {k: {"us": round(statistics.median(v), 1), "frac": round((W + 1) * n * 4 / (statistics.median(v) * 1e-6) / 8e12, 4)}
       for k, v in res.items()}
print(json.dumps(dict(sorted(out.items(), key=lambda kv: kv[1]["us"])), indent=1))
