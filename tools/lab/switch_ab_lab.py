#!/usr/bin/env python3
"""Switch A/B lab (experiment only): the in-tree libina.so against another build of it
(LIB_B: e.g. make -C distributed-training-ina_amd/csrc OUT=../../tools/lab/libina_b.so
BUILD=build_b EXTRA=-D...) on config 3
as NGA-V packets (V env, 256 or 32; 8 workers; 2^17 / 2^20-slot pool; descriptors) in
worker-major, round-robin and shuffled arrival, packed rows and split rows.  Per order: the
two libraries' actions, rewritten rows and registers compared byte for byte on fresh
switches, then HIP events around K back-to-back process() calls, interleaved over rounds
(one switch and sort scratch per library: each keeps its own call epochs); medians in us."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

if "LIB_B" not in os.environ:
    raise SystemExit("set LIB_B to the library build to compare against")
libs = {"A": _lib.load(), "B": _lib.open_library(os.environ["LIB_B"])}
dev = torch.device("cuda")
V = int(os.environ.get("V", 256))
W, n = 8, 26_214_400
slots = (1 << 17) if V == 256 else (1 << 20)
npk = n // V
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


out = {"V": V, "lib_B": os.path.basename(os.environ["LIB_B"])}
for order, perm in perms.items():
    stream, desc = (base, base_desc) if perm is None else (base[perm], base_desc[perm])
    hdr, pay = split_rows(stream)
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
    out[f"{order}/bytes_equal"] = all(torch.equal(x, y) for x, y in zip(state["A"], state["B"]))
    out[f"{order}/batch_path"] = paths
    del state
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
use("A")
print(json.dumps(out, indent=1))
