#!/usr/bin/env python3
"""Switch tuning-key A/B lab (experiment only): one library, a switch tuning key set to each of
VALUES in turn (env KEY=name of the ops.set_tuning argument, VALUES=comma list, e.g.
KEY=switch_strided VALUES=1,0), on config 3 as NGA-V packets (V env, default 32: 8 x 819,200
packets, 2^20 slots; descriptors) in the orders of ORDERS, split rows (ROWS=packed for packed
rows).  Per order: the settings' actions, payload rows and registers compared byte for byte on
fresh switches and the path each took, then HIP events around K back-to-back calls, the settings
interleaved over ROUNDS rounds; medians in us."""
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
KEY = os.environ.get("KEY", "switch_strided")
VALUES = [int(v) for v in os.environ.get("VALUES", "1,0").split(",")]
V = int(os.environ.get("V", 32))
W, n = 8, 26_214_400
slots = (1 << 17) if V == 256 else (1 << 20)
npk = n // V
N = W * npk
packed = os.environ.get("ROWS", "split") == "packed"
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
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 3))
rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)


def order_perm(name):
    if name == "worker_major":
        return None
    if name == "round_robin":
        return rr
    if name == "shuffled":
        return torch.randperm(N, device=dev, generator=g)
    J = int(name[len("jitter"):])
    key = torch.arange(N, device=dev) + torch.randint(0, J, (N,), device=dev, generator=g)
    return rr[torch.sort(key, stable=True).indices]


def setting(v):
    ops.set_tuning(**{KEY: v})


def timed(fn):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(K):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / K


out = {"V": V, "rows": "packed" if packed else "split", "key": KEY, "values": VALUES}
try:
    for order in os.environ.get("ORDERS", "round_robin,worker_major").split(","):
        perm = order_perm(order)
        stream, desc = (base, base_desc) if perm is None else (base[perm], base_desc[perm])
        hdr = torch.zeros((N, 16), dtype=torch.uint8, device=dev)
        hdr[:, :15] = stream[:, :15]
        pay = stream[:, 15:15 + 4 * V].contiguous()

        def call(sw):
            return sw.process(stream, acts, desc=desc) if packed else sw.process_split(hdr, pay, acts, desc=desc)

        state, paths = {}, {}
        for v in VALUES:
            setting(v)
            sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
            st, h, p = stream.clone(), hdr.clone(), pay.clone()
            a = sw.process(st, desc=desc) if packed else sw.process_split(h, p, desc=desc)
            state[v] = [x.cpu() for x in (a, st if packed else p, sw.count, sw.frag, sw.regs)]
            paths[v] = sw.batch_path(N)
            del sw, st, h, p
            torch.cuda.empty_cache()
        ref = state[VALUES[0]]
        out[f"{order}/bytes_equal"] = {v: all(torch.equal(x, y) for x, y in zip(ref, s)) for v, s in state.items()}
        out[f"{order}/path"] = paths
        del state
        sws = {v: ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for v in VALUES}
        res = {}
        for _ in range(ROUNDS):
            for v in VALUES:
                setting(v)
                res.setdefault(v, []).append(timed(lambda: call(sws[v])))
        out[f"{order}/us"] = {v: round(statistics.median(x), 2) for v, x in res.items()}
        print(order, json.dumps({k: v for k, v in out.items() if k.startswith(order)}), flush=True)
        del sws, stream, desc, hdr, pay
        torch.cuda.empty_cache()
finally:
    ops.set_tuning(**{KEY: VALUES[0]})
print(json.dumps(out))
