#!/usr/bin/env python3
"""Quick median timings of selected product ops (experiment helper)."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402


def t(fn, reps=30):
    for _ in range(3):
        fn()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3


n, V = 26_214_400, 256
x = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device="cuda")
pk = ops.pack_nga(x, V, 1, 8, 1, 1)
npk, stride = pk.shape
which = sys.argv[1:] or ["unpack", "unpack_vals", "pack"]
for w in which:
    if w == "unpack":
        us = t(lambda: ops.unpack_nga(pk, V))
        nb = npk * stride + 4 * n + 15 * npk
    elif w == "unpack_vals":
        us = t(lambda: ops.unpack_nga(pk, V, with_values=True))
        nb = npk * stride + 4 * n + 15 * npk
    elif w == "pack":
        us = t(lambda: ops.pack_nga(x, V, 1, 8, 1, 1, out=pk))
        nb = 4 * n + npk * stride
    print(f"{w}: {us:.1f} us  {nb / us / 1e3:.1f} GB/s  {nb / us / 1e3 / 8000:.3f}")
