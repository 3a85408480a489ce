#!/usr/bin/env python3
"""Placement lab (experiment only): the NGA-32 C3 round-robin split-row switch call with its
header rows, payload rows and slot registers in torch's default allocations, against the same
arrays in physically contiguous allocations (hipExtMallocWithFlags(hipDeviceMallocContiguous)),
wrapped as torch tensors through __cuda_array_interface__ (KINDS: torch, contiguous = all three,
rows = header + payload rows only, regs = slot registers only).  Each kind is allocated afresh REPS
times, alternating, with a large allocation freed in between to change the allocator's history;
HIP events around K back-to-back calls, median of ROUNDS.  Env: K, ROUNDS, REPS, ORDER (rr,
wm), V (32 or 256)."""
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

hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipFree.argtypes = [C.c_void_p]
CONTIG = 0x4

dev = torch.device("cuda")
V = int(os.environ.get("V", 32))
W, n = 8, 26_214_400
slots = (1 << 17) if V == 256 else (1 << 20)
npk = n // V
N = W * npk
K, ROUNDS, REPS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 3)), int(os.environ.get("REPS", 3))
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
if os.environ.get("ORDER", "rr") == "rr":
    rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)
    base, base_desc = base[rr], base_desc[rr]
hdr0 = torch.zeros((N, 16), dtype=torch.uint8, device=dev)
hdr0[:, :15] = base[:, :15]
pay0 = base[:, 15:15 + 4 * V].contiguous()
desc = base_desc
del base
acts = torch.empty(N, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()


class _Raw:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def contiguous(nbytes, keep):
    p = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, CONTIG)
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags(contiguous, {nbytes}) = {rc}")
    keep.append(p.value)
    return torch.as_tensor(_Raw(p.value, nbytes), device=dev)


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


KINDS = os.environ.get("KINDS", "torch,contiguous").split(",")   # + rows (hdr + pay only), regs (regs only)
res = {k: [] for k in KINDS}
for rep in range(REPS):
    for kind in KINDS:
        churn = torch.empty((8 + 4 * rep) << 30, dtype=torch.uint8, device=dev)   # allocator history
        del churn
        keep = []
        rows_c = kind in ("contiguous", "rows")
        regs_c = kind in ("contiguous", "regs")
        if rows_c:
            hdr = contiguous(N * 16, keep).view(N, 16)
            pay = contiguous(N * 4 * V, keep).view(N, 4 * V)
        else:
            hdr = torch.empty((N, 16), dtype=torch.uint8, device=dev)
            pay = torch.empty((N, 4 * V), dtype=torch.uint8, device=dev)
        if regs_c:
            regs = contiguous(slots * V * 4, keep).view(torch.int32).view(slots, V)
            regs.zero_()
        else:
            regs = torch.zeros((slots, V), dtype=torch.int32, device=dev)
        hdr.copy_(hdr0)
        pay.copy_(pay0)
        sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        sw.regs = regs
        sw._state = _lib.SwitchState(slots, V, 1, 0, sw.count.data_ptr(), sw.frag.data_ptr(), regs.data_ptr())
        t = [timed(lambda: sw.process_split(hdr, pay, acts, desc=desc)) for _ in range(ROUNDS)]
        res[kind].append(round(statistics.median(t), 2))
        print(rep, kind, res[kind][-1], sw.batch_path(N), flush=True)
        del sw, hdr, pay, regs
        torch.cuda.synchronize()
        for p in keep:
            hip.hipFree(p)
        torch.cuda.empty_cache()
print(json.dumps(res))
