#!/usr/bin/env python3
"""Interleaved A/B timing of the reduce variants in reduce_lab.so (experiment only).

Every configuration is checked bit-exact against the product kernel once, then all
configurations are timed round-robin (R rounds x L launches each, HIP events), and
the median per configuration is reported (cdna_hip_programming.md 5.4 rule 24).
"""
import ctypes as C
import itertools
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

lab = C.CDLL(os.path.join(HERE, "reduce_lab.so"))
lab.lab_launch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                           C.c_size_t, C.c_void_p]

N = 26_214_400
W = 8
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
sets = []
for r in range(2):
    g.manual_seed(1000 + r)
    sets.append([torch.randint(-(1 << 20), 1 << 20, (N,), dtype=torch.int32, device=dev, generator=g)
                 for _ in range(W)])
outs = [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(2)]
arrs = [(C.c_void_p * W)(*[b.data_ptr() for b in s]) for s in sets]
ref = ops.sum_reduce(sets[0])
stream = torch.cuda.current_stream().cuda_stream

configs = []
FOCUS = os.environ.get("FOCUS", "")
if FOCUS == "sched":
    for U, B, G in itertools.product((2, 4), (256, 512), (256, 512, 1024)):
        configs.append(("gridstride", 1, U, B, G))
        configs.append(("loads_first", 8, U, B, G))
        configs.append(("loads_first_schedbarrier", 9, U, B, G))
    for G in (1024, 2048):
        configs.append(("readonly8", 6, 1, 256, G))
elif FOCUS == "copy":
    # U field of variant 12: load/store policy (0 plain/plain, 1 plain/nt, 2 nt/plain, 3 nt/nt)
    for pol in (0, 1, 2, 3):
        for G in (512, 1024, 2048, 4096, 8192):
            configs.append((f"copy_pol{pol}", 12, pol, 256, G))
    for G in (4096, 16384):
        configs.append(("copy", 7, 1, 256, G))
elif FOCUS == "store":
    # U field: variant 11 packs the cache-policy pair: 2 = nt/nt, 4 = nt/default,
    # 5 = nt/sc0, 6 = default/nt
    for B, G in ((256, 512), (512, 256), (256, 1024), (512, 512)):
        configs.append(("gridstride", 1, 4, B, G))
        configs.append(("plainstore", 10, 4, B, G))
        for aux in (2, 4, 5, 6):
            configs.append((f"buf{aux}", 11, aux, B, G))
    for G in (1024, 2048):
        configs.append(("readonly8", 6, 1, 256, G))
elif FOCUS == "grid":
    for U, B, G in itertools.product((2, 4, 6, 8), (128, 256, 512, 768, 1024), (128, 192, 256, 320, 384, 512, 768)):
        configs.append(("gridstride", 1, U, B, G))
    for G in (1024, 2048):
        configs.append(("readonly8", 6, 1, 256, G))
else:
    for U, B, G in itertools.product((1, 2, 4), (256, 512, 1024), (256, 512, 1024, 2048, 4096, 16384)):
        configs.append(("gridstride", 1, U, B, G))
    for U, B, G in itertools.product((1, 2, 4), (256, 512), (512, 1024, 2048, 4096)):
        configs.append(("tile", 2, U, B, G))
    for U, B, G in itertools.product((1, 2, 4), (256, 512), (256, 512, 1024, 2048)):
        configs.append(("span", 3, U, B, G))
    for A, B, G in itertools.product((1, 2), (256, 512, 1024), (512, 1024, 2048, 4096, 8192)):
        configs.append(("ldsdma" + ("_nt" if A == 2 else ""), 4, A, B, G))
    for A, B, G in itertools.product((1, 2), (256, 512), (512, 1024, 2048, 4096)):
        configs.append(("ldsdma2" + ("_nt" if A == 2 else ""), 5, A, B, G))
    for G in (1024, 2048, 4096, 16384):
        configs.append(("readonly8", 6, 1, 256, G))
        configs.append(("copy", 7, 1, 256, G))


def nbytes(v):
    return {6: W * N * 4, 7: 2 * N * 4, 12: 2 * N * 4}.get(v, (W + 1) * N * 4)


# copy variants read buffer k % 16 (1.7 GB rotation, never resident in the 256 MB MALL)
flat = [b for st in sets for b in st]
carrs = [(C.c_void_p * W)(*([flat[j].data_ptr()] * W)) for j in range(len(flat))]


def launch(cfg, k):
    name, v, U, B, G = cfg
    arr = carrs[k % len(carrs)] if v in (7, 12) else arrs[k % 2]
    rc = lab.lab_launch(v, W, U, B, G, arr, outs[k % 2].data_ptr(), N // 4, stream)
    assert rc == 0, (cfg, rc)


bad = []
for cfg in configs:
    if cfg[1] in (6, 7, 12):
        continue
    outs[0].zero_()
    launch(cfg, 0)
    torch.cuda.synchronize()
    if not torch.equal(outs[0], ref):
        bad.append(cfg)
print("mismatching configs:", bad, flush=True)

R, L = int(os.environ.get("ROUNDS", "5")), int(os.environ.get("LAUNCHES", "8"))
times = {cfg: [] for cfg in configs}
for r in range(R):
    for cfg in configs:
        evs = []
        for k in range(L):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(cfg, k)
            b.record()
            evs.append((a, b))
        torch.cuda.synchronize()
        times[cfg] += [a.elapsed_time(b) / 1e3 for a, b in evs[1:]]
rows = []
for cfg, ts in times.items():
    med = statistics.median(ts)
    rows.append({"variant": cfg[0], "U_or_aux": cfg[2], "B": cfg[3], "grid": cfg[4],
                 "us": round(med * 1e6, 2), "min_us": round(min(ts) * 1e6, 2),
                 "GBps": round(nbytes(cfg[1]) / med / 1e9, 1)})
rows.sort(key=lambda r: -r["GBps"])
for r in rows[:40]:
    print(r)
print("...")
best = {}
for r in rows:
    best.setdefault(r["variant"], r)
for v, r in best.items():
    print("best", v, r)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump({"rows": rows, "bad": [list(b) for b in bad]},
          open(os.path.join(REPO, "gpurun_out", "reduce_lab.json"), "w"), indent=1)
