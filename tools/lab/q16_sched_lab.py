#!/usr/bin/env python3
"""C4 kernel-schedule lab (experiment only): ina_quantize_reduce_f32_i16_sat (16 workers x
25,557,032 fp32, V = 256 slot flags) from each library given on the command line -- builds
of k_quant_reduce_i16 that differ only in how the worker loads are scheduled -- interleaved
over rounds, HIP events around 20 back-to-back launches on two rotating input sets (the
bench's method).  Values and flags must be identical across libraries."""
import ctypes as C
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
W, n, k, V = 16, 25_557_032, 13, 256
sets = [[torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)] for _ in range(2)]
for b in sets[0][:3]:
    b[::4999] = 9.0                          # some saturation
ptrs = [(C.c_void_p * W)(*[t.data_ptr() for t in s]) for s in sets]
outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
flags = [torch.empty((n + V - 1) // V, dtype=torch.uint8, device=dev) for _ in range(2)]
st = torch.cuda.current_stream().cuda_stream
libs = []
for p in sys.argv[1:]:
    lib = C.CDLL(p)
    lib.ina_quantize_reduce_f32_i16_sat.argtypes = _lib.SIGNATURES["ina_quantize_reduce_f32_i16_sat"]
    libs.append((os.path.basename(p), lib))


def call(lib, r):
    rc = lib.ina_quantize_reduce_f32_i16_sat(ptrs[r], W, outs[r].data_ptr(), n, k, V, flags[r].data_ptr(), st)
    assert rc == 0, rc


ref = None
for name, lib in libs:
    call(lib, 0)
    torch.cuda.synchronize()
    got = (outs[0].clone(), flags[0].clone())
    if ref is None:
        ref = got
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), name
print("outputs identical; flags set:", int(ref[1].sum()), flush=True)
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
algo = (4 * W + 2) * n + (n + V - 1) // V
for name, _ in libs:
    m = statistics.median(t[name])
    print(f"{name:22s} median {m:7.2f} us  min {min(t[name]):7.2f}  frac {algo / m / 1e3 / 8000:.4f}", flush=True)
