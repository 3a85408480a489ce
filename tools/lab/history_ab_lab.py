#!/usr/bin/env python3
"""History A/B (experiment only): the NGA-256 config-3 switch batch (bench.py's switch_c3: 8
workers x 102,400 packed NGA-256 packets, 2^17-slot pool, descriptor keys) in worker-major and
round-robin arrival, through libina.so builds of earlier commits on ONE box -- so a change
between the driver's rounds is told apart from box-to-box spread.  Each build is called
through the entry point it exports (ina_switch, or the older ina_switch_process_desc); HIP
events around K back-to-back calls, the builds interleaved over ROUNDS rounds; medians in us.
  env LIBS=name:path,...  (e.g. r03:tools/lab/libina_r03.so); ORDERS; K; ROUNDS;
  PROFILE=name (one build only, for a rocprofv3 kernel trace of it)."""
import ctypes as C
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

specs = [("head", _lib.LIB_PATH)] + [tuple(x.split(":")) for x in filter(None, os.environ.get("LIBS", "").split(","))]
if os.environ.get("PROFILE"):
    specs = [x for x in specs if x[0] == os.environ["PROFILE"]]
libs = {}
for name, path in specs:
    lib = C.CDLL(os.path.join(REPO, path) if not os.path.isabs(path) else path)
    lib.ina_switch_scratch_bytes.restype = C.c_size_t
    lib.ina_switch_scratch_bytes.argtypes = [C.c_size_t, C.c_uint32]
    if hasattr(lib, "ina_switch"):
        lib.ina_switch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    else:
        lib.ina_switch_process_desc.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_void_p]
    libs[name] = lib

dev = torch.device("cuda")
V, W, n, slots = 256, 8, 26_214_400, 1 << 17
npk = n // V
N = W * npk
g = torch.Generator(device=dev).manual_seed(4242)
rows, descs = [], []
for w in range(W):
    b = torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=dev, generator=g)
    p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    rows.append(p)
    descs.append(d)
    del b
base, base_desc = torch.cat(rows), torch.cat(descs)
del rows, descs
stride = base.shape[1]
acts = torch.empty(N, dtype=torch.uint8, device=dev)
rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 5))
strm = torch.cuda.current_stream().cuda_stream


class State:
    def __init__(self, lib):
        self.count = torch.zeros(slots, dtype=torch.uint8, device=dev)
        self.frag = torch.zeros(slots, dtype=torch.int32, device=dev)
        self.regs = torch.zeros((slots, V), dtype=torch.int32, device=dev)
        self.st = _lib.SwitchState(slots, V, 1, 0, self.count.data_ptr(), self.frag.data_ptr(), self.regs.data_ptr())
        self.scratch = torch.empty(lib.ina_switch_scratch_bytes(N, slots), dtype=torch.uint8, device=dev)


def call(lib, s, pk, ds):
    if hasattr(lib, "ina_switch"):
        b = _lib.SwitchBatch(pk.data_ptr(), None, N, stride, ds.data_ptr(), acts.data_ptr(), s.scratch.data_ptr())
        rc = lib.ina_switch(C.byref(s.st), C.byref(b), None, 0, strm)
    else:
        rc = lib.ina_switch_process_desc(C.byref(s.st), pk.data_ptr(), N, stride, ds.data_ptr(), acts.data_ptr(),
                                         s.scratch.data_ptr(), strm)
    assert rc == 0, rc


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


out = {"workload": "NGA-256 C3, packed rows, descriptor keys", "libs": dict(specs)}
for order in os.environ.get("ORDERS", "worker_major,round_robin").split(","):
    perm = None if order == "worker_major" else rr
    pk, ds = (base.clone(), base_desc) if perm is None else (base[perm].contiguous(), base_desc[perm].contiguous())
    sts = {name: State(lib) for name, lib in libs.items()}
    res = {}
    for _ in range(ROUNDS):
        for name, lib in libs.items():
            res.setdefault(name, []).append(timed(lambda: call(lib, sts[name], pk, ds)))
    done = int((acts == 1).sum())
    out[order] = {k: round(statistics.median(v), 2) for k, v in res.items()}
    out[order]["completed_last"] = done
    print(order, json.dumps(out[order]), flush=True)
    del pk, sts
    torch.cuda.empty_cache()
print(json.dumps(out))
