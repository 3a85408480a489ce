#!/usr/bin/env python3
"""Time atomic_lab.so: 819,200 per-packet atomics on 102,400..131,072 slot counters."""
import ctypes as C
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lab = C.CDLL(os.path.join(HERE, "atomic_lab.so"))
lab.lab_bucket.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                           C.c_int, C.c_void_p]
dev = torch.device("cuda")
n, S, K = 819_200, 102_400, 16
layouts = {
    "worker-major": (torch.arange(n, device=dev) % S).to(torch.int32),
    "random": torch.randint(0, S, (n,), device=dev, dtype=torch.int32),
    "one-slot-x64": (torch.arange(n, device=dev) // 64 % S).to(torch.int32),
}
cnt = torch.zeros(1 << 17, dtype=torch.int32, device=dev)
slots = torch.zeros((1 << 17) * K, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
for name, keys in layouts.items():
    for mode in (0, 1, 2):
        for grid, block in ((3200, 256), (1024, 256), (8192, 256)):
            ts = []
            for r in range(12):
                cnt.zero_()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert lab.lab_bucket(keys.data_ptr(), n, cnt.data_ptr(), slots.data_ptr(), K, mode,
                                      grid, block, st) == 0
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ok = int(cnt.sum()) if mode < 2 else -1
            print(f"{name:14s} mode {mode} grid {grid:5d}: {statistics.median(ts[2:]):7.1f} us  (count sum {ok})")
