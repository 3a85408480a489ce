#!/usr/bin/env python3
"""Grid lab after the write-through store change (experiment only): the grid caps were
tuned with nt stores; re-sweep them with the product library as it is now, interleaved
over rounds, HIP events around 20 back-to-back launches on two rotating input sets (the
bench's method).  Outputs are compared with the default setting's."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
ROUNDS, K = int(os.environ.get("ROUNDS", 6)), 20
RN = 25_557_032


def f32(n):
    return torch.randn(n, device=dev, generator=g) * 1e-2


def i32(n):
    return torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)


cases = []
# headline C3 reduce: reduce_blocks (0 = 64 W = 512)
c3 = [[i32(26_214_400) for _ in range(8)] for _ in range(2)]
c3o = [torch.empty(26_214_400, dtype=torch.int32, device=dev) for _ in range(2)]
cases.append(("C3 reduce W=8", "reduce_blocks", [0, 768, 1024, 2048],
              lambda r: ops.sum_reduce(c3[r], out=c3o[r]), lambda r: c3o[r], 9 * 26_214_400 * 4))
# C2 fused quantise + reduce W=4: ew_blocks (default 2^24 = covering grid)
c2 = [[f32(RN) for _ in range(4)] for _ in range(2)]
c2o = [torch.empty(RN, dtype=torch.int32, device=dev) for _ in range(2)]
cases.append(("C2 quant+reduce W=4", "ew_blocks", [1 << 24, 4096, 2048, 1024],
              lambda r: ops.quantize_reduce(c2[r], 16, out=c2o[r]), lambda r: c2o[r], 20 * RN))
# C4 int16 W=16: max_blocks (default 16384)
c4 = [[f32(RN) for _ in range(16)] for _ in range(2)]
c4o = [torch.empty(RN, dtype=torch.int16, device=dev) for _ in range(2)]
c4f = [torch.empty((RN + 255) // 256, dtype=torch.uint8, device=dev) for _ in range(2)]
cases.append(("C4 quant+reduce i16 W=16", "max_blocks", [16384, 8192, 4096, 2048, 1024],
              lambda r: ops.quantize_reduce_i16(c4[r], 13, 256, out=c4o[r], overflow=c4f[r]),
              lambda r: c4o[r], 66 * RN + RN // 256))
# C5 quantise / dequantise, 1 GiB: ew_blocks
N5 = 1 << 28
c5 = [f32(N5) for _ in range(2)]
c5q = [torch.empty(N5, dtype=torch.int32, device=dev) for _ in range(2)]
cases.append(("C5 quantize 1 GiB", "ew_blocks", [1 << 24, 16384, 8192, 4096],
              lambda r: ops.quantize(c5[r], 16, out=c5q[r]), lambda r: c5q[r], 8 * N5))
c5d = [torch.empty(N5, dtype=torch.float32, device=dev) for _ in range(2)]
cases.append(("C5 dequantize 1 GiB", "ew_blocks", [1 << 24, 16384, 8192, 4096],
              lambda r: ops.dequantize(c5q[r], 16, out=c5d[r]), lambda r: c5d[r], 8 * N5))


def setk(knob, v):
    ops.set_tuning(**{knob: v})


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


for name, knob, vals, fn, res, nbytes in cases:
    ref = None
    for v in vals:
        setk(knob, v)
        fn(0)
        torch.cuda.synchronize()
        if ref is None:
            ref = res(0).clone()
        assert torch.equal(res(0), ref), (name, v)
    t = {v: [] for v in vals}
    for _ in range(ROUNDS):
        for v in vals:
            setk(knob, v)
            t[v].append(timed(fn))
    setk(knob, vals[0])
    for v in vals:
        m = statistics.median(t[v])
        print(f"{name:26s} {knob}={v:<9d} {m:8.2f} us  frac {nbytes / m / 1e3 / 8000:.4f}", flush=True)
