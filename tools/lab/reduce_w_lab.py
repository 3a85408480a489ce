#!/usr/bin/env python3
"""Interleaved grid sweep of the product sum-reduce for several W (experiment only)."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

n = 26_214_400
g = torch.Generator(device="cuda").manual_seed(5)
pool = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
        for _ in range(17)]
out = torch.empty(n, dtype=torch.int32, device="cuda")
cfgs = [(W, G) for W in (2, 4, 8, 16) for G in (256, 512, 1024, 2048, 4096, 8192)]
times = {c: [] for c in cfgs}
for r in range(int(os.environ.get("ROUNDS", 6))):
    for W, G in cfgs:
        ops.set_tuning(reduce_blocks=G)
        bufs = pool[:W] if r % 2 == 0 else pool[17 - W:]
        ev = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ops.sum_reduce(bufs, out=out)
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        times[(W, G)] += [a.elapsed_time(b) / 1e3 for a, b in ev[1:]]
ops.set_tuning(reduce_blocks=0)
for W in (2, 4, 8, 16):
    rows = []
    for G in (256, 512, 1024, 2048, 4096, 8192):
        m = statistics.median(times[(W, G)])
        rows.append((round((W + 1) * n * 4 / m / 1e9, 1), G, round(m * 1e6, 1)))
    print(W, sorted(rows, reverse=True))
