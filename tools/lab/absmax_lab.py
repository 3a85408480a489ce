#!/usr/bin/env python3
"""Interleaved A/B of ina_absmax_f32 across libina builds (experiment only): ResNet-50
delta (x - base, 25,557,032 fp32), cold caches; results must agree bit for bit."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
n = 25_557_032
g = torch.Generator(device=dev).manual_seed(4)
x = torch.randn(n, device=dev, generator=g) * 1e-2
b = torch.randn(n, device=dev, generator=g) * 1e-2
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
libs = []
for p in sys.argv[1:]:
    lib = C.CDLL(p)
    lib.ina_absmax_f32.argtypes = _lib.SIGNATURES["ina_absmax_f32"]
    libs.append((os.path.basename(p), lib, torch.zeros(1, device=dev), []))
for nm, lib, out, _ in libs:
    assert lib.ina_absmax_f32(x.data_ptr(), b.data_ptr(), n, out.data_ptr(), st) == 0
torch.cuda.synchronize()
assert all(torch.equal(libs[0][2], o) for _, _, o, _ in libs), [float(o) for _, _, o, _ in libs]
assert float(libs[0][2]) == float((x - b).abs().max())
for r in range(int(os.environ.get("ROUNDS", 6))):
    for nm, lib, out, ts in libs:
        evs = []
        for _ in range(4):
            ops.checksum(flush)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lib.ina_absmax_f32(x.data_ptr(), b.data_ptr(), n, out.data_ptr(), st)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        ts += [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs[1:]]
for nm, _, _, ts in libs:
    us = statistics.median(ts)
    print(f"{nm:20s} absmax {us:6.1f} us  {8 * n / us / 1e3:7.1f} GB/s")
