#!/usr/bin/env python3
"""Narrow-run lab (experiment only): the NGA-32 run over a run table slot-parallel (8 slots per
wave, the runs walked in order: INA_SWITCH_NARROW_SLOTS=1, the in-tree libina.so) against one
slot's 8 packets side by side (tools/lab/libina_noslots.so: make -C
distributed-training-ina_amd/csrc OUT=../../tools/lab/libina_noslots.so BUILD=build_noslots
EXTRA=-DINA_SWITCH_NARROW_SLOTS=0).  (Round 4's first try, slot s+1's loads issued before slot
s runs, measured 541.8 vs 547.8 us packed, 488.2 vs 491.3 split: profiles/r04/lab/narrow_pre_lab.log.)
Config 3 as NGA-32 packets (8 workers x 819,200, 2^20-slot pool, descriptors) in worker-major
arrival, packed and split rows, and the same batch with the previous step's PS acks in front;
HIP events around K back-to-back process() calls, interleaved over rounds, medians in us.
Every library's actions, registers, count/frag and rewritten rows are compared byte for byte."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

libs = {"slots": _lib.load(), "segments": _lib.open_library(os.path.join(HERE, "libina_noslots.so"))}
dev = torch.device("cuda")
W, n, V, slots = 8, 26_214_400, 32, 1 << 20
npk = n // V
g = torch.Generator(device=dev).manual_seed(11)
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
acts = torch.empty(W * npk, dtype=torch.uint8, device=dev)
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 5))


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


# parity: a fresh switch per library over pristine copies, two batches (the second finds the
# first's count/frag/registers), everything compared
state, paths = {}, {}
for name in libs:
    use(name)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    out = []
    for rep in range(2):
        st, h, p = stream.clone(), hdr.clone(), pay.clone()
        a1 = sw.process(st, desc=desc)
        a2 = ops.Switch(V, num_slots=slots, switch_id=1, device=dev).process_split(h, p, desc=desc)
        out += [a1, st, a2, h, p]
    out += [sw.count.clone(), sw.frag.clone(), sw.regs.clone()]
    paths[name] = sw.batch_path(W * npk)
    state[name] = out
    del sw
same = all(torch.equal(x, y) for x, y in zip(state["slots"], state["segments"]))
del state

# one switch (and sort scratch) per library: each library keeps its own call epochs
sws = {name: ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for name in libs}
res = {}
for r in range(ROUNDS):
    for name in libs:
        use(name)
        sw = sws[name]
        res.setdefault(f"packed/{name}", []).append(timed(lambda: sw.process(stream, acts, desc=desc)))
        res.setdefault(f"split/{name}", []).append(timed(lambda: sw.process_split(hdr, pay, acts, desc=desc)))
use("slots")
sw = sws["slots"]
out = {k: round(statistics.median(v), 2) for k, v in res.items()}
out["bytes_equal"] = same
out["parity_batch_path"] = paths
out["batch_path"] = sw.batch_path(W * npk)
print(json.dumps(out, indent=1))
