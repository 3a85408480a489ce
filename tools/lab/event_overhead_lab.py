#!/usr/bin/env python3
"""Lab: how much of a per-call HIP-event pair is measurement overhead for the switch?
The same 819,200-packet config-3 batch through ina_switch_process timed (a) one event
pair per call (median), (b) one event pair around K back-to-back calls (/K), and
(c) the headline reduce the same two ways, for comparison.

  python tools/lab/event_overhead_lab.py
"""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
n, W, V, slots = 26_214_400, 8, 256, 1 << 17
g = torch.Generator(device=dev).manual_seed(1)
bufs, packed = [], []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    bufs.append(b)
    packed.append(ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True))
st = torch.cat([p for p, _ in packed])
ds = torch.cat([d for _, d in packed])
del packed
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(st.shape[0], dtype=torch.uint8, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
K = int(os.environ.get("K", 10))


def per_call(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def batched(fn, rounds=5):
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / K)
    return statistics.median(ts)


def switch():
    sw.process(st, acts, desc=ds)


def reduce():
    ops.sum_reduce(bufs, out=out)


for f in (switch, reduce):
    f()
torch.cuda.synchronize()
res = {}
for name, f in (("switch", switch), ("reduce", reduce)):
    res[name] = {"per_call_pair_us": round(per_call(f), 1), f"one_pair_per_{K}_calls_us": round(batched(f), 1)}
print(json.dumps(res, indent=1))
