#!/usr/bin/env python3
"""Arrival-order lab (experiment only): the device switch over config 3 as NGA-V packets (V
env, default 32: 8 workers x 819,200 packets, 2^20-slot pool, descriptors) in round-robin
arrival with local jitter -- every packet of the round-robin order displaced by less than J
positions (sort key = position + U[0, J)), the arrival of W sequence-ordered senders
(DataManager.py:116-134) interleaved by a NIC with local disorder -- next to plain
round-robin, worker-major and a shuffled batch.  Packed rows and split rows; HIP events
around K back-to-back process() calls; the path each call took.  ORDERS env: comma list."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
V = int(os.environ.get("V", 32))
W, n = 8, 26_214_400
slots = (1 << 17) if V == 256 else (1 << 20)
npk = n // V
N = W * npk
g = torch.Generator(device=dev).manual_seed(21)
rows, descs = [], []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    rows.append(p)
    descs.append(d)
    del b
base, base_desc = torch.cat(rows), torch.cat(descs)
del rows, descs
acts = torch.empty(N, dtype=torch.uint8, device=dev)
K = int(os.environ.get("K", 10))
rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)


def jitter(J, seed):
    gj = torch.Generator(device=dev).manual_seed(seed)
    key = torch.arange(N, device=dev) + torch.randint(0, J, (N,), device=dev, generator=gj)
    return rr[torch.sort(key, stable=True).indices]


perms = {"worker_major": None, "round_robin": rr}
for J in (8, 64, 512, 4096, 16384):
    perms[f"jitter{J}"] = jitter(J, 100 + J)
perms["shuffled"] = torch.randperm(N, device=dev, generator=g)
want = [o for o in os.environ.get("ORDERS", ",".join(perms)).split(",") if o]


def timed(fn):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(3):
        a.record()
        for _ in range(K):
            fn()
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / K)
    return round(statistics.median(res), 2)


out = {"V": V, "npk": N, "slots": slots}
for order in want:
    perm = perms[order]
    stream, desc = (base, base_desc) if perm is None else (base[perm], base_desc[perm])
    hdr = torch.zeros((N, 16), dtype=torch.uint8, device=dev)
    hdr[:, :15] = stream[:, :15]
    pay = stream[:, 15:15 + 4 * V].contiguous()
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    r = {"packed_us": timed(lambda: sw.process(stream, acts, desc=desc))}
    r["packed_path"] = sw.batch_path(N)
    r["split_us"] = timed(lambda: sw.process_split(hdr, pay, acts, desc=desc))
    r["split_path"] = sw.batch_path(N)
    r["completed"] = int((acts == 1).sum())
    out[order] = r
    print(order, json.dumps(r), flush=True)
    del stream, desc, hdr, pay, sw
    torch.cuda.empty_cache()
print(json.dumps(out))
