#!/usr/bin/env python3
"""Phase timing of the switch sort's bucket kernel (experiment only): a lab build of libina
with -DINA_BK_TIMING=1 (tools/lab/libina_bktime.so) stamps each k_sort_buckets block's wall
clock (s_memrealtime, 100 MHz) at: start, row read + scans done, gather + tile counts done,
digit scan done, scatter done.  Runs ina_switch_process on config 3 as 8 x 102,400 NGA-256
packets (descriptor keys) and prints the block start spread and the mean / max of each phase.
Env V=32 SLOTS=1048576 ORDERS=shuffled: the NGA-32 batch (6,553,600 packets) shuffled.
  build: make -C distributed-training-ina_amd/csrc OUT=../../tools/lab/libina_bktime.so \
         BUILD=build_bktime EXTRA=-DINA_BK_TIMING=1"""
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

lab = C.CDLL(os.path.join(HERE, "libina_bktime.so"))
for nm in ("ina_switch", "ina_switch_scratch_bytes"):
    getattr(lab, nm).argtypes = _lib.SIGNATURES[nm]
lab.ina_switch_scratch_bytes.restype = C.c_size_t
lab.ina_lab_bk_times.argtypes = [C.c_void_p]

n, W = 26_214_400, 8
V, slots = int(os.environ.get("V", 256)), int(os.environ.get("SLOTS", 1 << 17))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
packed = [ops.pack_nga(torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g),
                       V, w + 1, W, 1, 1, num_slots=slots, desc=True) for w in range(W)]
src = torch.cat([p for p, _ in packed])
desc = torch.cat([d for _, d in packed])
del packed
orders = {"worker_major": (src, desc)}
perm = torch.arange(src.shape[0], device=dev).view(W, -1).t().reshape(-1)
orders["round_robin"] = (src[perm].contiguous(), desc[perm].contiguous())
perm = torch.randperm(src.shape[0], device=dev, generator=g)
orders["shuffled"] = (src[perm].contiguous(), desc[perm].contiguous())
del perm
keep = os.environ.get("ORDERS", "worker_major,round_robin").split(",")
orders = {k: v for k, v in orders.items() if k in keep}
npk, stride = src.shape
count = torch.zeros(slots, dtype=torch.uint8, device=dev)
frag = torch.zeros(slots, dtype=torch.int32, device=dev)
regs = torch.zeros((slots, V), dtype=torch.int32, device=dev)
acts = torch.empty(npk, dtype=torch.uint8, device=dev)
st = _lib.SwitchState(slots, V, 1, 0, count.data_ptr(), frag.data_ptr(), regs.data_ptr())
scratch = torch.empty(lab.ina_switch_scratch_bytes(npk, slots), dtype=torch.uint8, device=dev)
buf = np.zeros((2048, 6), np.uint64)
names = ["rows+scans", "gather+counts", "digit scan", "scatter"]
for oname, (pk, ds) in orders.items():
    work = pk.clone()
    res = {k: [] for k in names}
    buf[:] = 0
    spread, span = [], []
    for rep in range(6):
        work.copy_(pk)
        count.zero_()
        frag.zero_()
        b = _lib.SwitchBatch(work.data_ptr(), None, npk, stride, ds.data_ptr(), acts.data_ptr(),
                             scratch.data_ptr())
        assert lab.ina_switch(C.byref(st), C.byref(b), None, _lib.INA_SWITCH_ALL,
                              torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        assert lab.ina_lab_bk_times(buf.ctypes.data) == 0
        if rep < 2:
            continue
        t = buf.astype(np.int64)
        t0 = t[:, 0]
        launched = t0 >= t0.max() - 10_000_000                  # this launch's blocks (< 100 ms)
        t0 = t0[launched]
        spread.append((t0.max() - t0.min()) * 10 / 1000)          # us (100 MHz ticks)
        full = launched & np.all(np.diff(t[:, :5], axis=1) >= 0, axis=1) & (t[:, 4] >= t[:, 0])
        full &= t[:, 0] >= t0.min()
        tf = t[full]
        span.append((tf[:, 4].max() - t0.min()) * 10 / 1000)
        for q, nm in enumerate(names):
            d = (tf[:, q + 1] - tf[:, q]) * 10 / 1000
            res[nm].append((d.mean(), d.max()))
        res.setdefault("blocks", []).append((int(launched.sum()), int(full.sum())))
        ev = np.concatenate([np.stack([tf[:, 0], np.ones(len(tf), np.int64)], 1),
                             np.stack([tf[:, 4], -np.ones(len(tf), np.int64)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        res.setdefault("conc", []).append(int(np.cumsum(ev[:, 1]).max()))
        life = (tf[:, 4] - tf[:, 0]) * 10 / 1000
        res.setdefault("life", []).append((float(life.mean()), float(np.percentile(life, 90))))
    print(f"{oname}: block start spread {statistics.median(spread):.2f} us, first start -> last "
          f"scatter done {statistics.median(span):.2f} us")
    print(f"   blocks launched / with a full tile pass: {res['blocks'][-1]}; most full blocks in "
          f"flight at once {max(res['conc'])}; block life mean / p90 {res['life'][-1][0]:.2f} / "
          f"{res['life'][-1][1]:.2f} us")
    nf = ~np.all(np.diff(t[:, :5], axis=1) >= 0, axis=1) & launched
    print("   a block without a full pass (stamps - its start, us):", ((t[nf][:2] - t[nf][:2, :1]) * 10 / 1000).tolist())
    for nm in names:
        print(f"   {nm:14s} mean {statistics.median(m for m, _ in res[nm]):6.2f} us  "
              f"max {statistics.median(x for _, x in res[nm]):6.2f} us")
