#!/usr/bin/env python3
"""Switch lab (experiment only): the slot sort's first pass whole (tuning key 19 = 0: keys of
<= 18 bits run k_sort_chunks once) or split into detection + one-block decision + digits
(key 19 = 1), and the packed against the split rows, on config 3 as NGA-256 packets (8 x
102,400, 2^17-slot pool, descriptors): worker-major (run table), round-robin (in order),
shuffled (sorted).  HIP events around 20 back-to-back process() calls, interleaved over
rounds; medians in us.  Also the steady-state packet path step (packs + switch + PS) in both
row layouts."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
W, n, V, slots = 8, 26_214_400, 256, 1 << 17
npk = n // V
g = torch.Generator(device=dev).manual_seed(3)
rows, descs = [], []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    rows.append(p)
    descs.append(d)
    del b
stream, desc = torch.cat(rows), torch.cat(descs)
del rows, descs
hdr = torch.zeros((W * npk, 16), dtype=torch.uint8, device=dev)
hdr[:, :15] = stream[:, :15]
pay = stream[:, 15:15 + 4 * V].contiguous()
perms = {"worker_major": None,
         "round_robin": torch.arange(W * npk, device=dev).view(W, npk).t().reshape(-1),
         "shuffled": torch.randperm(W * npk, device=dev, generator=g)}
batches = {}
for name, perm in perms.items():
    if perm is None:
        batches[name] = (stream, hdr, pay, desc)
    else:
        batches[name] = (stream[perm], hdr[perm], pay[perm], desc[perm])
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(W * npk, dtype=torch.uint8, device=dev)
K, ROUNDS = 20, int(os.environ.get("ROUNDS", 5))


def timed(fn):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(K):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / K


res = {}
for r in range(ROUNDS):
    for name, (st, h, p, d) in batches.items():
        for pre in (0, 1):
            for rows_kind in ("packed", "split"):
                ops.set_tuning(switch_pre_all=bool(pre))
                if rows_kind == "packed":
                    us = timed(lambda: sw.process(st, acts, desc=d))
                else:
                    us = timed(lambda: sw.process_split(h, p, acts, desc=d))
                res.setdefault(f"{name}/{rows_kind}/pre{pre}", []).append(us)
                path = sw.batch_path(W * npk)
                res.setdefault(f"{name}/{rows_kind}/pre{pre}/path", path)
ops.set_tuning(switch_pre_all=False)
out = {k: (round(statistics.median(v), 2) if isinstance(v, list) else v) for k, v in res.items()}
print(json.dumps(out, indent=1))
