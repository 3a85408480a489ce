#!/usr/bin/env python3
"""Switch A/B/... lab (experiment only): the in-tree libina.so ("A") against other builds of it
(env LIBS=name:path,name:path; e.g. make -C distributed-training-ina_amd/csrc
OUT=../../tools/lab/libina_x.so BUILD=build_x EXTRA=-D...) on config 3 as NGA-V packets (V env,
default 32: 8 x 819,200 packets, 2^20 slots; descriptors) in the orders of ORDERS (worker_major,
round_robin, jitterJ -- round-robin with every packet displaced by < J positions --, shuffled),
split rows (ROWS=packed for packed rows).  Per order: the libraries' actions, payload rows and
registers compared byte for byte on fresh switches, then HIP events around K back-to-back
calls, interleaved over ROUNDS rounds; medians in us."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

libs = {"A": _lib.load()}
for spec in filter(None, os.environ.get("LIBS", "").split(",")):
    name, path = spec.split(":")
    libs[name] = _lib.open_library(os.path.join(REPO, path))
dev = torch.device("cuda")
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


def use(name):
    _lib._lib = libs[name]


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


out = {"V": V, "rows": "packed" if packed else "split", "libs": {k: os.environ.get("LIBS", "") for k in libs}}
for order in os.environ.get("ORDERS", "round_robin,jitter64,jitter4096,shuffled").split(","):
    perm = order_perm(order)
    stream, desc = (base, base_desc) if perm is None else (base[perm], base_desc[perm])
    hdr = torch.zeros((N, 16), dtype=torch.uint8, device=dev)
    hdr[:, :15] = stream[:, :15]
    pay = stream[:, 15:15 + 4 * V].contiguous()

    def call(sw):
        return sw.process(stream, acts, desc=desc) if packed else sw.process_split(hdr, pay, acts, desc=desc)

    state, paths = {}, {}
    for name in libs:
        use(name)
        sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        st, h, p = stream.clone(), hdr.clone(), pay.clone()
        a = sw.process(st, desc=desc) if packed else sw.process_split(h, p, desc=desc)
        state[name] = [x.cpu() for x in (a, st if packed else p, sw.count, sw.frag, sw.regs)]
        paths[name] = sw.batch_path(N)
        del sw, st, h, p
        torch.cuda.empty_cache()
    ref = state["A"]
    out[f"{order}/bytes_equal"] = {k: all(torch.equal(x, y) for x, y in zip(ref, v)) for k, v in state.items()}
    out[f"{order}/path"] = paths
    del state
    sws = {name: ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for name in libs}
    res = {}
    for _ in range(ROUNDS):
        for name in libs:
            use(name)
            res.setdefault(name, []).append(timed(lambda: call(sws[name])))
    out[f"{order}/us"] = {k: round(statistics.median(v), 2) for k, v in res.items()}
    print(order, json.dumps({k: v for k, v in out.items() if k.startswith(order)}), flush=True)
    del sws, stream, desc, hdr, pay
    torch.cuda.empty_cache()
use("A")
print(json.dumps(out))
