#!/usr/bin/env python3
"""Zero-copy lab (experiment only): the PCIe-inclusive aggregation with the W-way reduce
kernel reading the workers' PINNED host buckets directly over PCIe (hipHostMalloc memory is
device-addressable) and writing the aggregate straight into pinned host memory -- no staging
copies, no chunk pipeline -- against the product's chunked pipeline (ina_sum_reduce_host_i32)
and the pinned H2D copy rate of the same bytes.  Config 3: 8 x 100 MiB int32."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

W, n = 8, 26_214_400
dev = torch.device("cuda")
rng = np.random.default_rng(3)
hosts = [torch.from_numpy(rng.integers(-(1 << 20), 1 << 20, n, dtype=np.int32)).pin_memory() for _ in range(W)]
want = np.zeros(n, np.uint32)
for h in hosts:
    want += h.numpy().view(np.uint32)
out = torch.empty(n, dtype=torch.int32).pin_memory()
lib = ops.load()
s = torch.cuda.current_stream()
res = {}


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


# H2D copy rate of the same bytes (two copy streams)
dbuf = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(W)]
cs = [torch.cuda.Stream(), torch.cuda.Stream()]


def h2d():
    for w in range(W):
        with torch.cuda.stream(cs[w % 2]):
            dbuf[w].copy_(hosts[w], non_blocking=True)


t = timed(h2d)
res["h2d_2streams_GBps"] = W * n * 4 / t / 1e9
del dbuf
# product pipeline
scratch = torch.empty(lib.ina_host_reduce_scratch_bytes(W, 0), dtype=torch.uint8, device=dev)
t = timed(lambda: ops.sum_reduce_host(hosts, out=out, scratch=scratch))
res["pipeline_GBps"] = W * n * 4 / t / 1e9
res["pipeline_ok"] = bool(np.array_equal(out.numpy().view(np.uint32), want))
# zero copy: the reduce kernel on the host buffers' DEVICE pointers (hipHostGetDevicePointer
# refuses memory that is not mapped for the device, so no kernel reads an unmapped address)
import ctypes as C  # noqa: E402
hip = C.CDLL("libamdhip64.so")


def devptr(t):
    p = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0)
    if rc != 0:
        raise SystemExit(f"hipHostGetDevicePointer rc={rc}: host buffer not device-mapped; no zero-copy run")
    return p.value


dptrs = [devptr(h) for h in hosts]
dout = devptr(out)
res["devptr_equals_hostptr"] = all(d == h.data_ptr() for d, h in zip(dptrs, hosts))
for blocks in (0, 256, 1024, 4096):
    lib.ina_set_tuning(3, blocks)
    for unroll in (1, 4):
        lib.ina_set_tuning(1, unroll)
        out.zero_()
        arr = _lib.ptr_array(dptrs)
        t = timed(lambda: _lib.check(lib.ina_sum_reduce_i32(arr, W, dout, n, s.cuda_stream)))
        res[f"zerocopy_blocks{blocks}_u{unroll}_GBps"] = W * n * 4 / t / 1e9
        res[f"zerocopy_blocks{blocks}_u{unroll}_ok"] = bool(np.array_equal(out.numpy().view(np.uint32), want))
lib.ina_set_tuning(3, 0)
lib.ina_set_tuning(1, 0)
for k, v in res.items():
    print(f"{k:36s} {v:.2f}" if isinstance(v, float) else f"{k:36s} {v}")
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "zerocopy_lab.json"), "w"), indent=1)
