#!/usr/bin/env python3
"""Store-policy lab (experiment only): the headline W = 8 reduce with different cache-policy
bits on its 16-byte stores (tools/lab/store_policy_lab.hip), timed back to back (20 launches,
two alternating input sets, HIP events -- bench.py's method) and as single launches after a
512 MiB read, interleaved over rounds.  If the nt-stored lines left dirty in the caches cost
the next dependent launch, a write-through policy shows a smaller back-to-back time.
  build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -shared tools/lab/store_policy_lab.hip \
         -o tools/lab/store_policy_lab.so"""
import ctypes as C
import json
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
lab = C.CDLL(os.path.join(HERE, "store_policy_lab.so"))
lab.lab_reduce8.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(11)
n, W = 26_214_400, 8
sets = [[torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
        for _ in range(2)]
outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
arrs = [(C.c_void_p * W)(*[t.data_ptr() for t in s]) for s in sets]
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
NAMES = {0: "nt (product)", 1: "sc0 sc1", 2: "sc1 nt", 3: "sc0 sc1 nt", 4: "default", 5: "sc1"}
K, ROUNDS, GRID = int(os.environ.get("K", 20)), int(os.environ.get("ROUNDS", 8)), 512


def launch(v, s):
    assert lab.lab_reduce8(v, GRID, arrs[s], outs[s].data_ptr(), n // 4, st) == 0


ref = None
for v in NAMES:
    launch(v, 0)
    torch.cuda.synchronize()
    if ref is None:
        ref = outs[0].clone()
    assert torch.equal(outs[0], ref), NAMES[v]
b2b = {v: [] for v in NAMES}
cold = {v: [] for v in NAMES}
for _ in range(ROUNDS):
    for v in NAMES:
        for i in range(6):
            launch(v, i % 2)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(K):
            launch(v, i % 2)
        b.record()
        torch.cuda.synchronize()
        b2b[v].append(a.elapsed_time(b) * 1e3 / K)
        flush.sum()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        launch(v, 0)
        b.record()
        torch.cuda.synchronize()
        cold[v].append(a.elapsed_time(b) * 1e3)
algo = (W + 1) * n * 4
rows = []
for v, name in NAMES.items():
    bb, cc = statistics.median(b2b[v]), statistics.median(cold[v])
    rows.append({"variant": name, "back_to_back_us": round(bb, 2), "cold_single_us": round(cc, 2),
                 "frac_b2b": round(algo / bb / 1e3 / 8000, 4), "frac_cold": round(algo / cc / 1e3 / 8000, 4)})
    print(f"{name:14s} back-to-back {bb:7.2f} us ({algo / bb / 1e3 / 8000:.3f})   single {cc:7.2f} us "
          f"({algo / cc / 1e3 / 8000:.3f})")
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(REPO, "gpurun_out", "store_policy_lab.json"), "w"), indent=1)
