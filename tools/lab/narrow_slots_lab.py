#!/usr/bin/env python3
"""Narrow-run lab (experiment only): the NGA-32 run kernel with lane groups taking 8 slots /
segments side by side (INA_SWITCH_NARROW_SLOTS=1, the in-tree libina.so: the run table walked
run by run, sorted windows segment by segment) against one slot's 8 packets side by side
(tools/lab/libina_noslots.so: make -C distributed-training-ina_amd/csrc
OUT=../../tools/lab/libina_noslots.so BUILD=build_noslots EXTRA=-DINA_SWITCH_NARROW_SLOTS=0).
(Round 4's first try, slot s+1's loads issued before slot s runs, measured 541.8 vs 547.8 us
packed, 488.2 vs 491.3 split: profiles/r04/lab/narrow_pre_lab.log.)
Config 3 as NGA-32 packets (8 workers x 819,200, 2^20-slot pool, descriptors) in worker-major
(run table), round-robin (in slot order) and shuffled (bucket sort) arrival, packed and split
rows; HIP events around K back-to-back process() calls, interleaved over rounds, medians in
us.  Each library's actions, registers, count/frag and rewritten rows are compared byte for
byte (two batches on a fresh switch, the second finding the first's state)."""
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
base, base_desc = torch.cat(rows), torch.cat(descs)
del rows, descs
acts = torch.empty(W * npk, dtype=torch.uint8, device=dev)
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 4))
perms = {"worker_major": None,
         "round_robin": torch.arange(W * npk, device=dev).view(W, npk).t().reshape(-1),
         "shuffled": torch.randperm(W * npk, device=dev, generator=g)}


def use(name):
    _lib._lib = libs[name]


def split_rows(st):
    h = torch.zeros((st.shape[0], 16), dtype=torch.uint8, device=dev)
    h[:, :15] = st[:, :15]
    return h, st[:, 15:15 + 4 * V].contiguous()


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


out = {}
for order, perm in perms.items():
    stream, desc = (base, base_desc) if perm is None else (base[perm], base_desc[perm])
    hdr, pay = split_rows(stream)
    # parity: per library a fresh switch, two batches, packed and split rows
    state, paths = {}, {}
    for name in libs:
        use(name)
        sw, sws = (ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for _ in range(2))
        res = []
        for rep in range(2):
            st = stream.clone()
            h, p = hdr.clone(), pay.clone()
            res += [sw.process(st, desc=desc), st, sws.process_split(h, p, desc=desc), h, p]
            del st, h, p
        res += [sw.count.clone(), sw.frag.clone(), sw.regs.clone(), sws.regs.clone()]
        paths[name] = sw.batch_path(W * npk)
        state[name] = [x.cpu() for x in res]
        del sw, sws, res
        torch.cuda.empty_cache()
    out[f"{order}/bytes_equal"] = all(torch.equal(x, y) for x, y in zip(state["slots"], state["segments"]))
    out[f"{order}/batch_path"] = paths
    del state
    # timing: one switch (and sort scratch) per library, interleaved rounds
    sws = {name: ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for name in libs}
    res = {}
    for r in range(ROUNDS):
        for name in libs:
            use(name)
            sw = sws[name]
            res.setdefault(f"{order}/packed/{name}", []).append(timed(lambda: sw.process(stream, acts, desc=desc)))
            res.setdefault(f"{order}/split/{name}", []).append(
                timed(lambda: sw.process_split(hdr, pay, acts, desc=desc)))
    out.update({k: round(statistics.median(v), 2) for k, v in res.items()})
    del sws, stream, desc, hdr, pay
    torch.cuda.empty_cache()
use("slots")
print(json.dumps(out, indent=1))
