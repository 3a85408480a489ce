#!/usr/bin/env python3
"""Floor lab (experiment only): the int16 elementwise kernels and C2's fused quantise +
reduce against copy kernels that move the same bytes in the same lane layout with no
arithmetic (tools/lab/ew16_lab.hip).  Same box, interleaved: every round times each case's
K back-to-back launches on two alternating buffer sets (bench.py's method) and the median
over rounds is reported with its fraction of 8 TB/s.
  build (C=distributed-training-ina_amd/csrc): hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -shared \
         -ffp-contract=off -I include -I $C tools/lab/ew16_lab.hip $C/ina_switch.hip $C/ina_shard.hip \
         $C/ina_host.cpp $C/ina_send.cpp -o tools/lab/ew16_lab.so -lpthread"""
import ctypes as C
import json
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
lab = C.CDLL(os.path.join(HERE, "ew16_lab.so"))
lab.lab_run.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
n = 25_556_992                       # ResNet-50 rounded down to whole 512-value regions
K, ROUNDS = 20, 8
st = torch.cuda.current_stream().cuda_stream

f32 = [[torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(4)] for _ in range(2)]
i16 = [torch.randint(-30000, 30000, (n,), dtype=torch.int16, device=dev, generator=g) for _ in range(2)]
o16 = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
o32 = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
flags = [torch.empty(n // 256, dtype=torch.uint8, device=dev) for _ in range(2)]
arr_f = [(C.c_void_p * 4)(*[t.data_ptr() for t in f32[s]]) for s in range(2)]
arr_h = [(C.c_void_p * 4)(*([i16[s].data_ptr()] * 4)) for s in range(2)]


def ew_grid(chunks):                      # one chunk per thread, the whole array
    return (chunks + 255) // 256


CASES = [  # name, which, grid, bytes, set -> (bufs, out, ovf)
    ("quantize_i16 (product, flags)", 0, ew_grid(n // 8), 6 * n + n // 256),
    ("copy 4->2 split layout", 1, ew_grid(n // 8), 6 * n),
    ("copy 4->2 row layout", 2, ew_grid(n // 8), 6 * n),
    ("copy 4->2 split, 8192 wg", 1, 8192, 6 * n),
    ("dequantize_i16 (product)", 3, ew_grid(n // 4), 6 * n),
    ("copy 2->4", 4, ew_grid(n // 4), 6 * n),
    ("copy 2->4, 8192 wg", 4, 8192, 6 * n),
    ("quant_reduce_i32<4> C2 (product grid 8192)", 5, 8192, 20 * n),
    ("quant_reduce_i32<4> C2, one chunk per thread", 5, ew_grid(n // 4), 20 * n),
    ("quant_reduce_i32<4> C2, 256 wg", 5, 256, 20 * n),
    ("quant_reduce_i32<4> C2, 512 wg", 5, 512, 20 * n),
    ("quant_reduce_i32<4> C2, 1024 wg", 5, 1024, 20 * n),
    ("quant_reduce_i32<4> C2, 2048 wg", 5, 2048, 20 * n),
    ("copy W=4 -> 1 (C2 bytes), 8192 wg", 6, 8192, 20 * n),
    ("copy W=4 -> 1, 256 wg", 6, 256, 20 * n),
    ("copy W=4 -> 1, 512 wg", 6, 512, 20 * n),
    ("copy W=4 -> 1, one chunk per thread", 6, ew_grid(n // 4), 20 * n),
    ("sum_reduce_i32<4,1> (int32, product kernel), 256 wg", 7, 256, 20 * n),
    ("sum_reduce_i32<4,1>, 8192 wg", 7, 8192, 20 * n),
]


def launch(which, grid, s):
    if which in (0, 1, 2):
        return lab.lab_run(which, grid, arr_f[s], o16[s].data_ptr(), n, flags[s].data_ptr(), st)
    if which in (3, 4):
        return lab.lab_run(which, grid, arr_h[s], o32[s].data_ptr(), n, None, st)
    return lab.lab_run(which, grid, arr_f[s], o32[s].data_ptr(), n, None, st)


times = {c[0]: [] for c in CASES}
for c in CASES:                            # warm every case
    for i in range(4):
        assert launch(c[1], c[2], i % 2) == 0, c[0]
torch.cuda.synchronize()
for _ in range(ROUNDS):
    for name, which, grid, _ in CASES:
        for i in range(6):                 # per-case warm-up inside the round
            launch(which, grid, i % 2)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(K):
            launch(which, grid, i % 2)
        b.record()
        torch.cuda.synchronize()
        times[name].append(a.elapsed_time(b) * 1e3 / K)
rows = []
for name, which, grid, nbytes in CASES:
    us = statistics.median(times[name])
    rows.append({"case": name, "grid": grid, "us": round(us, 2), "bytes": nbytes,
                 "GBps": round(nbytes / us / 1e3, 1), "frac": round(nbytes / us / 1e3 / 8000, 4)})
    print(f"{name:52s} grid {grid:8d}  {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s  frac {nbytes / us / 1e3 / 8000:.3f}")
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(REPO, "gpurun_out", "ew16_lab.json"), "w"), indent=1)
