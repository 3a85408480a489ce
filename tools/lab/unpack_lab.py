#!/usr/bin/env python3
"""Unpack variants (experiment): with / without the SoA header fields, cold caches."""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
n, V = 26_214_400, 256
x = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev)
pk = ops.pack_nga(x, V, 1, 8, 1, 1)
npk, stride = pk.shape
vals = torch.empty(npk * V, dtype=torch.int32, device=dev)
f = {k: torch.empty(npk, dtype=torch.int32, device=dev) for k in ("bitmap", "index", "frag_id")}
f.update({k: torch.empty(npk, dtype=torch.uint8, device=dev) for k in ("count", "flags", "switch_id")})
fs = _lib.NgaFields(*[f[k].data_ptr() for k in ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream


def run(with_fields):
    return lib.ina_unpack_nga(pk.data_ptr(), npk, V, stride, C.byref(fs) if with_fields else None,
                              vals.data_ptr(), st)


for name, wf in (("fields+values", True), ("values only", False)):
    ts = []
    for _ in range(3):
        run(wf)
    for _ in range(20):
        ops.checksum(flush)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        assert run(wf) == 0
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    us = statistics.median(a.elapsed_time(b) for a, b in ts) * 1e3
    print(f"{name:16s} {us:6.1f} us  {(npk * stride + 4 * n) / us / 1e3:7.1f} GB/s")
