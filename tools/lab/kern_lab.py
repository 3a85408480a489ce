#!/usr/bin/env python3
"""Interleaved A/B of product-kernel variants and grids (experiment only)."""
import ctypes as C
import json
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
lab = C.CDLL(os.path.join(HERE, "kern_lab.so"))
lab.lab_kern.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_int,
                         C.c_void_p, C.c_void_p]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
n = 25_557_032
bufs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(16)]
arr16 = (C.c_void_p * 16)(*[b.data_ptr() for b in bufs])
o16 = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
f16 = [torch.empty((n + 255) // 256, dtype=torch.uint8, device=dev) for _ in range(2)]
o32 = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream

# (round 1 also compared a coalesced 512-value "tile" form of the int16 kernel: equal
#  results, equal speed within noise -- not kept)

cfgs = []
for G in (256, 512, 1024, 2048, 4096, 8192):
    cfgs += [("C4 row", 0, G, (16 * 4 + 2) * n),
             ("C2", 2, G, (4 * 4 + 4) * n), ("quantize", 3, G, 8 * n)]


def run(c):
    name, which, G, _ = c
    if which == 0:
        return lab.lab_kern(which, G, arr16, 16, o16[0].data_ptr(), n, 256, f16[0].data_ptr(), st)
    if which == 2:
        return lab.lab_kern(2, G, arr16, 4, o32.data_ptr(), n, 256, None, st)
    return lab.lab_kern(3, G, arr16, 1, o32.data_ptr(), n, 256, None, st)


times = {c: [] for c in cfgs}
for r in range(int(os.environ.get("ROUNDS", 6))):
    for c in cfgs:
        ev = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert run(c) == 0
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        times[c] += [a.elapsed_time(b) / 1e3 for a, b in ev[1:]]
rows = []
for c, ts in times.items():
    m = statistics.median(ts)
    rows.append({"kernel": c[0], "grid": c[2], "us": round(m * 1e6, 1),
                 "GBps": round(c[3] / m / 1e9, 1)})
for k in ("C4 row", "C2", "quantize"):
    for r in sorted([r for r in rows if r["kernel"] == k], key=lambda r: -r["GBps"]):
        print(r)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(REPO, "gpurun_out", "kern_lab.json"), "w"), indent=1)
