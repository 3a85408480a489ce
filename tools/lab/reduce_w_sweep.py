#!/usr/bin/env python3
"""Grid x chunks sweep of the W-way int32 reduce for W = 2, 4, 16 (experiment only):
in-tree library, ops.set_tuning(reduce_blocks, unroll), cold caches."""
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
n = 26_214_400
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
for W in (2, 4, 16):
    bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev) for _ in range(W)]
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ref = ops.sum_reduce(bufs)
    res = []
    for u in (1, 2, 4):
        for blocks in (0, 256, 512, 768, 1024, 2048):
            ops.set_tuning(unroll=u, reduce_blocks=blocks)
            ts = []
            for _ in range(12):
                ops.checksum(flush)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ops.sum_reduce(bufs, out=out)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            assert torch.equal(out, ref)
            us = statistics.median(ts[2:])
            res.append((us, u, blocks))
    ops.set_tuning(unroll=0, reduce_blocks=0)
    res.sort()
    print(f"W={W}: " + "  ".join(f"U{u}/{b or 'rule'} {us:.1f}" for us, u, b in res[:6]),
          f"| default rule U4: {[us for us, u, b in res if u == 4 and b == 0][0]:.1f} us", flush=True)
    del bufs, out, ref
