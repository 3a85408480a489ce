#!/usr/bin/env python3
"""Packet-kernel grid lab (experiment only): the flat NGA pack / fused quantise + pack /
unpack kernels at grid caps up to a covering grid (one 16-byte chunk per thread), product
library, interleaved over rounds, HIP events around 20 back-to-back launches on two
rotating inputs.  Outputs are compared with the default setting's."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(4)
ROUNDS, K, V = int(os.environ.get("ROUNDS", 8)), 20, 256
GRIDS = [int(x) for x in os.environ.get("GRIDS", "8192,16384,32768").split(",")]
n3, nr = 26_214_400, 25_557_032
stride = ops.nga_stride(V)
npk3, npkr = (n3 + V - 1) // V, (nr + V - 1) // V
vi = [torch.randint(-(1 << 20), 1 << 20, (n3,), dtype=torch.int32, device=dev, generator=g) for _ in range(2)]
pk = [torch.empty((npk3, stride), dtype=torch.uint8, device=dev) for _ in range(2)]
xs = [torch.randn(nr, device=dev, generator=g) * 1e-2 for _ in range(2)]
base = torch.randn(nr, device=dev, generator=g) * 1e-2
pr = [torch.empty((npkr, stride), dtype=torch.uint8, device=dev) for _ in range(2)]
cases = [
    ("pack_nga C3 (102,400 pkts)", lambda r: ops.pack_nga(vi[r], V, 1, 8, 1, 1, out=pk[r]), lambda: pk[0],
     4 * n3 + npk3 * stride),
    ("quantize_pack_nga ResNet-50 delta", lambda r: ops.quantize_pack_nga(xs[r], 16, V, 1, 8, 1, 1, base=base,
                                                                          out=pr[r]), lambda: pr[0],
     8 * nr + npkr * stride),
    ("unpack_nga C3", lambda r: ops.unpack_nga(pk[r], V), None, npk3 * stride + 4 * n3 + 15 * npk3),
]


def timed(fn):
    for i in range(6):
        fn(i % 2)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(K):
        fn(i % 2)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / K


for name, fn, res, nbytes in cases:
    ref = None
    for v in GRIDS:
        ops.set_tuning(stream_blocks=v)
        fn(0)
        torch.cuda.synchronize()
        if res is not None:
            if ref is None:
                ref = res().clone()
            assert torch.equal(res(), ref), (name, v)
    t = {v: [] for v in GRIDS}
    for _ in range(ROUNDS):
        for v in GRIDS:
            ops.set_tuning(stream_blocks=v)
            t[v].append(timed(fn))
    ops.set_tuning(stream_blocks=16384)
    for v in GRIDS:
        m = statistics.median(t[v])
        print(f"{name:36s} stream_blocks={v:<6d} {m:7.2f} us  frac {nbytes / m / 1e3 / 8000:.4f}", flush=True)
