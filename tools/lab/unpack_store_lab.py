#!/usr/bin/env python3
"""Unpack store-policy lab (experiment only): ina_unpack_nga (config 3 as 102,400 NGA-256
packets -> header fields + 26,214,400 int32 values) from each library on the command line
(builds that differ in the cache policy of the value stores), interleaved over rounds, HIP
events around 20 back-to-back launches on two rotating packet sets.  Outputs must agree."""
import ctypes as C
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(6)
V, n = 256, 26_214_400
stride = ops.nga_stride(V)
npk = n // V
pk = [ops.pack_nga(torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g),
                   V, 1, 8, 1, 1, out=torch.empty((npk, stride), dtype=torch.uint8, device=dev)) for _ in range(2)]
F = [{k: torch.empty(npk, dtype=dt, device=dev) for k, dt in
      (("bitmap", torch.int32), ("count", torch.uint8), ("flags", torch.uint8), ("index", torch.int32),
       ("switch_id", torch.uint8), ("frag_id", torch.int32))} for _ in range(2)]
FS = [_lib.NgaFields(*[f[k].data_ptr() for k in ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
      for f in F]
vals = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
st = torch.cuda.current_stream().cuda_stream
libs = []
for p in sys.argv[1:]:
    lib = C.CDLL(p)
    lib.ina_unpack_nga.argtypes = _lib.SIGNATURES["ina_unpack_nga"]
    libs.append((os.path.basename(p), lib))


def call(lib, r):
    assert lib.ina_unpack_nga(pk[r].data_ptr(), npk, V, stride, C.byref(FS[r]), vals[r].data_ptr(), st) == 0


ref = None
for name, lib in libs:
    call(lib, 0)
    torch.cuda.synchronize()
    got = (vals[0].clone(), F[0]["frag_id"].clone())
    if ref is None:
        ref = got
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), name
ROUNDS, K = int(os.environ.get("ROUNDS", 10)), 20
t = {name: [] for name, _ in libs}
for _ in range(ROUNDS):
    for name, lib in libs:
        for i in range(6):
            call(lib, i % 2)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(K):
            call(lib, i % 2)
        b.record()
        torch.cuda.synchronize()
        t[name].append(a.elapsed_time(b) * 1e3 / K)
algo = npk * stride + 4 * n + 15 * npk
for name, _ in libs:
    m = statistics.median(t[name])
    print(f"{name:22s} median {m:7.2f} us  min {min(t[name]):7.2f}  frac {algo / m / 1e3 / 8000:.4f}", flush=True)
