#!/usr/bin/env python3
"""Launch-gap lab (experiment only): why C2's back-to-back event time (96.7 us per launch in
the r03a bench line) exceeds its kernel time (87.2 us under rocprof).  On C2's inputs
(4 x 25,557,032 fp32, two sets alternated) it times 20 back-to-back launches of the fused
quantise + reduce with HIP events as bench.py does:
  wrapper   ops.quantize_reduce (the Python wrapper: argument checks, pointer array)
  direct    the C entry point with prebuilt ctypes arguments (no Python checks)
  graph     the 20 launches captured once as a hipGraph and replayed
and the host time to ISSUE those 20 calls (no sync), so a host-bound loop shows up as
issue time >= event time.  The same for the headline reduce (W = 8 x 26,214,400 int32).
Run it twice, with and without HIP_FORCE_DEV_KERNARG=1, to see the kernarg placement."""
import ctypes as C
import json
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
K = 20
res = {"env_HIP_FORCE_DEV_KERNARG": os.environ.get("HIP_FORCE_DEV_KERNARG")}


def ev_time(issue):
    s = torch.cuda.current_stream()
    issue()
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(s)
        t0 = time.perf_counter()
        issue()
        t_issue = time.perf_counter() - t0
        b.record(s)
        torch.cuda.synchronize()
        out.append((a.elapsed_time(b) * 1e3 / K, t_issue * 1e6 / K))
    return {"event_us_per_launch": round(statistics.median(o[0] for o in out), 2),
            "host_issue_us_per_call": round(statistics.median(o[1] for o in out), 2)}


def case(name, fn_for, sets):
    lib = ops.load()

    def wrapper():
        for i in range(K):
            fn_for(i % 2)
    r = {"wrapper": ev_time(wrapper)}
    # direct C call with prebuilt arguments
    args = [sets["direct"](i) for i in range(2)]
    entry = getattr(lib, sets["entry"])

    def direct():
        for i in range(K):
            entry(*args[i % 2])
    r["direct"] = ev_time(direct)
    # hipGraph of the K launches
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        wrapper()
    torch.cuda.current_stream().wait_stream(cap)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        wrapper()
    r["graph"] = ev_time(g.replay)
    res[name] = r
    print(name, json.dumps(r), flush=True)


# C2: fused quantise + reduce, 4 x ResNet-50 fp32
n2, W2 = 25_557_032, 4
gen = torch.Generator(device=dev).manual_seed(1)
x2 = [[torch.randn(n2, device=dev, generator=gen) * 1e-2 for _ in range(W2)] for _ in range(2)]
o2 = [torch.empty(n2, dtype=torch.int32, device=dev) for _ in range(2)]
keep = []


def c2_direct(i):
    arr = _lib.ptr_array([t.data_ptr() for t in x2[i]])
    keep.append(arr)
    return (arr, W2, o2[i].data_ptr(), n2, 16, torch.cuda.current_stream().cuda_stream)


case("c2_quant_reduce", lambda i: ops.quantize_reduce(x2[i], 16, out=o2[i]),
     {"direct": c2_direct, "entry": "ina_quantize_reduce_f32_i32"})
del x2, o2
torch.cuda.empty_cache()

# headline: W = 8 int32 reduce
n3, W3 = 26_214_400, 8
x3 = [[torch.randint(-(1 << 20), 1 << 20, (n3,), dtype=torch.int32, device=dev, generator=gen)
       for _ in range(W3)] for _ in range(2)]
o3 = [torch.empty(n3, dtype=torch.int32, device=dev) for _ in range(2)]


def c3_direct(i):
    arr = _lib.ptr_array([t.data_ptr() for t in x3[i]])
    keep.append(arr)
    return (arr, W3, o3[i].data_ptr(), n3, torch.cuda.current_stream().cuda_stream)


case("c3_sum_reduce", lambda i: ops.sum_reduce(x3[i], out=o3[i]),
     {"direct": c3_direct, "entry": "ina_sum_reduce_i32"})
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
tag = "devkernarg" if os.environ.get("HIP_FORCE_DEV_KERNARG") == "1" else "default"
json.dump(res, open(os.path.join(REPO, "gpurun_out", f"launch_gap_lab_{tag}.json"), "w"), indent=1)
