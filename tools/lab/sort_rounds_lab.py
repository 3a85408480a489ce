#!/usr/bin/env python3
"""Sort-chunk lab (experiment only): the product switch on config 3's 819,200 NGA-256
packets (descriptor keys, worker-major and round-robin arrival) with the slot sort's chunk
set by ina_set_tuning key 13 (64-item rounds per wave: 16 = 4,096-packet chunks, 200 A
blocks; 8 = 2,048, 400 blocks; 4 = 1,024, 800 blocks), interleaved per round, HIP events
around each call.  Actions must agree across settings."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

n, W, V = 26_214_400, 8, 256
slots = 1 << 17
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
        for _ in range(W)]
packed = [ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True) for w, b in enumerate(bufs)]
del bufs
wm = torch.cat([p for p, _ in packed])
wm_d = torch.cat([d for _, d in packed])
del packed
npw = wm.shape[0] // W
perm = torch.arange(W * npw, device=dev).view(W, npw).t().reshape(-1)
streams = {"wm": (wm, wm_d), "rr": (wm[perm].contiguous(), wm_d[perm].contiguous())}
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(wm.shape[0], dtype=torch.uint8, device=dev)
SETTINGS = [int(x) for x in os.environ.get("SETTINGS", "16,8,4").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", 12))


def call(pk, d):
    sw.count.zero_()
    sw.frag.zero_()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    sw.process(pk, acts, desc=d)
    b.record()
    return a, b


for name, (pk, d) in streams.items():
    ref = None
    for s in SETTINGS:
        ops.set_tuning(switch_sort_rounds=s)
        call(pk, d)
        torch.cuda.synchronize()
        if ref is None:
            ref = acts.clone()
        assert torch.equal(acts, ref), (name, s)
    t = {s: [] for s in SETTINGS}
    for _ in range(ROUNDS):
        for s in SETTINGS:
            ops.set_tuning(switch_sort_rounds=s)
            for _ in range(2):
                call(pk, d)
            ev = [call(pk, d) for _ in range(3)]
            torch.cuda.synchronize()
            t[s].extend(a.elapsed_time(b) * 1e3 for a, b in ev)
    for s in SETTINGS:
        print(f"{name} rounds {s:2d} (chunk {s * 256:5d})  median {statistics.median(t[s]):7.1f} us  "
              f"min {min(t[s]):7.1f} us", flush=True)
ops.set_tuning(switch_sort_rounds=0)
