#!/usr/bin/env python3
"""Placement lab (experiment only): the headline W = 8 sum-reduce (config 3, 8 x 100 MiB int32,
two input sets alternated as in bench.py) with its inputs and outputs in torch's default
allocations, against the same arrays in physically contiguous allocations
(hipExtMallocWithFlags(hipDeviceMallocContiguous)).  Alternating, REPS times, a large allocation
freed between them; HIP events around STEPS back-to-back launches."""
import ctypes as C
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipFree.argtypes = [C.c_void_p]
dev = torch.device("cuda")
W, n = 8, 26_214_400
STEPS, REPS = int(os.environ.get("STEPS", 40)), int(os.environ.get("REPS", 3))
g = torch.Generator(device=dev).manual_seed(5)
src = [[torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
       for _ in range(2)]


class _Raw:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def contiguous(nbytes, keep):
    p = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, 0x4)
    if rc != 0:
        raise RuntimeError(f"contiguous alloc {nbytes}: {rc}")
    keep.append(p.value)
    return torch.as_tensor(_Raw(p.value, nbytes), device=dev)


res = {"torch": [], "contiguous": []}
for rep in range(REPS):
    for kind in ("torch", "contiguous"):
        churn = torch.empty((8 + 4 * rep) << 30, dtype=torch.uint8, device=dev)
        del churn
        keep = []
        if kind == "torch":
            sets = [[torch.empty(n, dtype=torch.int32, device=dev) for _ in range(W)] for _ in range(2)]
            outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
        else:
            sets = [[contiguous(4 * n, keep).view(torch.int32) for _ in range(W)] for _ in range(2)]
            outs = [contiguous(4 * n, keep).view(torch.int32) for _ in range(2)]
        for s, t in zip(sets, src):
            for a, b in zip(s, t):
                a.copy_(b)
        for i in range(5):
            ops.sum_reduce(sets[i % 2], out=outs[i % 2])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(STEPS):
            ops.sum_reduce(sets[i % 2], out=outs[i % 2])
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / STEPS
        res[kind].append(round(us, 2))
        print(rep, kind, res[kind][-1], "frac", round(9 * 4 * n / (us * 1e-6) / 8e12, 4), flush=True)
        del sets, outs
        torch.cuda.synchronize()
        for p in keep:
            hip.hipFree(p)
        torch.cuda.empty_cache()
print(json.dumps(res))
