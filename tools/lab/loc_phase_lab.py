#!/usr/bin/env python3
"""Phase timing of the near-sorted path's list build (experiment only): a lab build of libina
with -DINA_LOC_TIMING=1 (tools/lab/libina_loctime.so) stamps each unit's wall clock (100 MHz) in
k_local_lists: entry, counts done, scan done, lists done (one pass units).  Config 3 as NGA-32
(8 x 819,200 packets, 2^20 slots), round-robin with jitter J (env J, default 64), split rows.
  build: make -C distributed-training-ina_amd/csrc OUT=../../tools/lab/libina_loctime.so \\
         BUILD=build_loctime EXTRA=-DINA_LOC_TIMING=1"""
import ctypes as C
import os
import statistics
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

_lib._lib = _lib.open_library(os.path.join(HERE, os.environ.get("LOCLIB", "libina_loctime.so")))
lab = _lib._lib
lab.ina_lab_loc_times.argtypes = [C.c_void_p]
n, W, V, slots = 26_214_400, 8, 32, 1 << 20
npk = n // V
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
hs, ps, ds = [], [], []
for w in range(W):
    p, d = ops.pack_nga(torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g),
                        V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    h = torch.zeros((npk, 16), dtype=torch.uint8, device=dev)
    h[:, :15] = p[:, :15]
    hs.append(h)
    ps.append(p[:, 15:15 + 4 * V].contiguous())
    ds.append(d)
    del p
N = W * npk
rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)
for J in [int(x) for x in os.environ.get("J", "64,4096").split(",")]:
    key = torch.arange(N, device=dev) + torch.randint(0, J, (N,), device=dev, generator=g)
    perm = rr[torch.sort(key, stable=True).indices]
    hdr, pay, desc = torch.cat(hs)[perm], torch.cat(ps)[perm], torch.cat(ds)[perm]
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    buf = np.zeros((8192, 4), np.uint64)
    res = {k: [] for k in ("count", "scan", "place", "block", "start_spread", "span", "units")}
    for rep in range(6):
        sw.process_split(hdr, pay, desc=desc)
        torch.cuda.synchronize()
        assert lab.ina_lab_loc_times(buf.ctypes.data) == 0
        b = buf.astype(np.int64)
        d0, dl = b[8191], b[8190]           # the decision pass: block 0 and the last block
        if rep >= 2:
            res.setdefault("dec_breaks", []).append(float(d0[1] - d0[0]) / 100)
            res.setdefault("dec_decide", []).append(float(d0[2] - d0[1]) / 100)
            dsub = b[8189]                   # inside the decision: PM/SM, units, reduction
            res.setdefault("dec_pmsm", []).append(float(dsub[0] - d0[1]) / 100)
            res.setdefault("dec_units", []).append(float(dsub[1] - dsub[0]) / 100)
            res.setdefault("dec_reduce", []).append(float(dsub[2] - dsub[1]) / 100)
            res.setdefault("dec_write", []).append(float(d0[2] - dsub[2]) / 100)
            res.setdefault("dec_last_entry", []).append(float(dl[0] - d0[0]) / 100)
            res.setdefault("dec_last_seen", []).append(float(dl[1] - d0[0]) / 100)
            res.setdefault("dec_to_lists", []).append(float(b[:8189, 0][b[:8189, 0] > 0].min() - d0[2]) / 100)
        b = b[:8189]
        b = b[(b[:, 0] > 0) & (b[:, 3] >= b[:, 0])]
        if rep < 2:
            continue
        res["count"].append(float(np.mean(b[:, 1] - b[:, 0])) / 100)
        res["scan"].append(float(np.mean(b[:, 2] - b[:, 1])) / 100)
        res["place"].append(float(np.mean(b[:, 3] - b[:, 2])) / 100)
        res["block"].append(float(np.mean(b[:, 3] - b[:, 0])) / 100)
        res["start_spread"].append(float(b[:, 0].max() - b[:, 0].min()) / 100)
        res["span"].append(float(b[:, 3].max() - b[:, 0].min()) / 100)
        res["units"].append(len(b))
        ev = sorted([(int(x), 1) for x in b[:, 0]] + [(int(x), -1) for x in b[:, 3]])
        cur = best = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
        res.setdefault("max_in_flight", []).append(best)
        st = np.sort(b[:, 0] - b[:, 0].min()) / 100
        res.setdefault("start_p10_p50_p90", []).append(0)
        if rep == 5:
            print("  start quantiles (us):", [round(float(np.quantile(st, q)), 1) for q in (0.1, 0.25, 0.5, 0.75, 0.9, 1.0)])
            qs = (0.1, 0.5, 0.9, 0.99, 1.0)
            for nm, x in (("block", b[:, 3] - b[:, 0]), ("count", b[:, 1] - b[:, 0]), ("place", b[:, 3] - b[:, 2]),
                          ("end", b[:, 3] - b[:, 0].min())):
                print(f"  {nm} quantiles (us) {qs}:", [round(float(np.quantile(x, q)) / 100, 1) for q in qs])
            slow = np.argsort(b[:, 3] - b[:, 0])[-8:]
            print("  slowest blocks' row index / start (us) / time (us):",
                  [(int(i), round(float(b[i, 0] - b[:, 0].min()) / 100, 1), round(float(b[i, 3] - b[i, 0]) / 100, 1)) for i in slow])
    print(f"J={J} path={sw.batch_path(N)} (us, means over blocks):",
          {k: round(statistics.median(v), 2) for k, v in res.items()}, flush=True)
    del hdr, pay, desc, sw
