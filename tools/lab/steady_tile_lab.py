#!/usr/bin/env python3
"""Bucket-tile lab (experiment only): the switch on the packet path's steady-state batch
(step t's 102,400 PS acks in front of step t+1's 8 x 102,400 worker packets, as
bench_extra's steady-state rows) and on the plain 8-worker batch, with the slot sort's
bucket tile forced to 4 or 8 rounds per wave or left to the auto rule (ina_set_tuning key
17), interleaved over rounds, HIP events around back-to-back calls.  Actions must agree."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(8)
W, V, n = 8, 256, 26_214_400
npk, stride = n // V, ops.nga_stride(V)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
glob_p = torch.randn(n, device=dev, generator=g) * 1e-2
upd = torch.empty_like(glob_p)
big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=dev)
ack_rows, rows_w = big[:npk], big[npk:].view(W, npk, stride)
desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
desc_ack, desc_w = desc[:npk], desc[npk:].view(W, npk)
acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
sw = ops.Switch(V, num_slots=1 << 17, switch_id=1, device=dev)
for _ in range(2):                              # two steps: the ack rows are then real PS acks
    for w in range(W):
        ops.quantize_pack_nga(xs[w], 16, V, w + 1, W, 1, 1, base=glob_p, num_slots=1 << 17,
                              out=rows_w[w], desc=desc_w[w])
    ops.nga_descriptors(ack_rows, out=desc_ack)
    sw.process(big, acts, desc=desc)
    ops.apply_completed(big, acts, V, 1, glob_p, 16, 1.0 / (W + 1), out=upd, acks=ack_rows)
ops.nga_descriptors(ack_rows, out=desc_ack)
torch.cuda.synchronize()
batches = {"steady (acks + 8 workers)": (big, desc, acts),
           "plain (8 workers)": (big[npk:], desc[npk:], acts[npk:])}
SETTINGS = [0, 4, 8]
ROUNDS, K = int(os.environ.get("ROUNDS", 8)), 5
for name, (b, d, a_) in batches.items():
    ref = None
    for t in SETTINGS:
        ops.set_tuning(switch_bucket_tile=t)
        sw.process(b, a_, desc=d)
        sw.process(b, a_, desc=d)
        torch.cuda.synchronize()
        if ref is None:
            ref = a_.clone()
        assert torch.equal(a_, ref), (name, t)
    res = {t: [] for t in SETTINGS}
    for _ in range(ROUNDS):
        for t in SETTINGS:
            ops.set_tuning(switch_bucket_tile=t)
            sw.process(b, a_, desc=d)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                sw.process(b, a_, desc=d)
            e1.record()
            torch.cuda.synchronize()
            res[t].append(e0.elapsed_time(e1) * 1e3 / K)
    for t in SETTINGS:
        print(f"{name:28s} tile {'auto' if t == 0 else t:>4}  median {statistics.median(res[t]):7.1f} us  "
              f"min {min(res[t]):7.1f} us", flush=True)
ops.set_tuning(switch_bucket_tile=0)
