#!/usr/bin/env python3
"""Interleaved A/B of ina_pack_c128 across libina builds (experiment only): ResNet-50 in
C-128 packets (199,665, communicator.py:10), cold caches, outputs must agree."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
npk = 199_665
g = torch.randint(-(1 << 31), (1 << 31) - 1, (npk * 128,), dtype=torch.int32, device=dev)
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
libs, ts = [], []
out = torch.empty(npk * 524, dtype=torch.uint8, device=dev)     # one buffer for every variant
for path in sys.argv[1:]:
    lib = C.CDLL(path)
    lib.ina_pack_c128.argtypes = _lib.SIGNATURES["ina_pack_c128"]
    libs.append(lib)
    ts.append([])
for n_small in (1, 2, 3, 5, 1000):                      # ragged tails agree too
    o = [torch.zeros(n_small * 524, dtype=torch.uint8, device=dev) for _ in libs]
    for lib, oo in zip(libs, o):
        assert lib.ina_pack_c128(g.data_ptr(), n_small, 3, 7, 10, oo.data_ptr(), st) == 0
    assert all(torch.equal(o[0], x) for x in o[1:]), n_small
ref = None
for lib in libs:
    assert lib.ina_pack_c128(g.data_ptr(), npk, 3, 7, 10, out.data_ptr(), st) == 0
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(ref, out)
del ref
for r in range(int(os.environ.get("ROUNDS", 8))):
    for i, lib in enumerate(libs):
        evs = []
        for _ in range(4):
            ops.checksum(flush)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            lib.ina_pack_c128(g.data_ptr(), npk, 3, 7, 10, out.data_ptr(), st)
            b.record()
            evs.append((a, b))
        torch.cuda.synchronize()
        ts[i] += [a.elapsed_time(b) * 1e3 for a, b in evs[1:]]
for path, t in zip(sys.argv[1:], ts):
    us = statistics.median(t)
    print(f"{os.path.basename(path):18s} pack_c128 {us:6.1f} us  {npk * 1036 / us / 1e3:7.1f} GB/s")
