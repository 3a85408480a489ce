#!/usr/bin/env python3
"""Interleaved A/B of the flat NGA pack / unpack kernels across libina builds (experiment
only): config 3's bucket at V = 256 (102,400 packets), one output buffer per kernel shared
by every variant, cold caches (512 MiB read between launches), outputs must agree."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
n, V = 26_214_400, 256
x = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev)
pk = ops.pack_nga(x, V, 1, 8, 1, 1)
npk, stride = pk.shape
out_pk = torch.empty_like(pk)
vals = torch.empty(n, dtype=torch.int32, device=dev)
f = {k: torch.empty(npk, dtype=torch.int32, device=dev) for k in ("bitmap", "index", "frag_id")}
f.update({k: torch.empty(npk, dtype=torch.uint8, device=dev) for k in ("count", "flags", "switch_id")})
fs = _lib.NgaFields(*[f[k].data_ptr() for k in ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
prm = _lib.NgaParams(1, 8, 0, 1, 0, 1, 16384, V)
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
libs = []
for p in sys.argv[1:]:
    lib = C.CDLL(p)
    for nm in ("ina_unpack_nga", "ina_pack_nga", "ina_pack_nga_desc"):
        getattr(lib, nm).argtypes = _lib.SIGNATURES[nm]
    libs.append((os.path.basename(p), lib, {"pack": [], "pack_desc": [], "unpack": []}))


desc = torch.empty(npk, dtype=torch.int64, device=dev)


def run(lib, which):
    if which == "pack_desc":
        return lib.ina_pack_nga_desc(x.data_ptr(), n, C.byref(prm), None, out_pk.data_ptr(), stride,
                                     desc.data_ptr(), st)
    if which == "pack":
        return lib.ina_pack_nga(x.data_ptr(), n, C.byref(prm), None, out_pk.data_ptr(), stride, st)
    return lib.ina_unpack_nga(pk.data_ptr(), npk, V, stride, C.byref(fs), vals.data_ptr(), st)


ref = None
for nm, lib, _ in libs:
    assert run(lib, "pack_desc") == 0
    torch.cuda.synchronize()
    got_d = (out_pk.clone(), desc.clone())
    desc.fill_(0)
    assert run(lib, "pack") == 0 and run(lib, "unpack") == 0
    torch.cuda.synchronize()
    got = (out_pk.clone(), vals.clone()) + tuple(f[k].clone() for k in sorted(f)) + got_d
    for t in f.values():
        t.fill_(0x5A)                            # the next variant must write every field
    if ref is None:
        ref = got
    assert all(torch.equal(a, b) for a, b in zip(ref, got)), nm
del ref
for _ in range(int(os.environ.get("ROUNDS", 8))):
    for nm, lib, ts in libs:
        for which in ("pack", "pack_desc", "unpack"):
            evs = []
            for _ in range(4):
                ops.checksum(flush)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(lib, which)
                b.record()
                evs.append((a, b))
            torch.cuda.synchronize()
            ts[which] += [a.elapsed_time(b) * 1e3 for a, b in evs[1:]]
for nm, _, ts in libs:
    print(f"{nm:22s} " + "   ".join(f"{k} {statistics.median(v):6.1f} us" for k, v in ts.items()))
