"""Lab: the one-launch worker pack (8 x 26,214,400 fp32 -> NGA-256, base read once) against
copy kernels of the same bytes (tools/lab/qpack_floor_lab.hip): its own layout with no
arithmetic, and an aligned 1,024-byte-stride stream copy.  Interleaved, back to back.
Build (container): hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -shared -ffp-contract=off
  -I include -I $C tools/lab/qpack_floor_lab.hip $C/ina_switch.hip $C/ina_shard.hip
  $C/ina_host.cpp $C/ina_send.cpp -o tools/lab/qpack_floor_lab.so -lpthread"""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

lab = C.CDLL(os.path.join(HERE, "qpack_floor_lab.so"))
lab.lab_copy.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
dev = torch.device("cuda:0")
W, n, V, k = 8, 26214400, 256, 16
npk = n // V
g = torch.Generator(device=dev)
g.manual_seed(1)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
base = torch.randn(n, device=dev, generator=g) * 1e-2
stride = ops.nga_stride(V)
rows = torch.empty((W, npk, stride), dtype=torch.uint8, device=dev)
flat = torch.empty((W, npk, 1024), dtype=torch.uint8, device=dev)
outs = list(rows.unbind(0))
s = torch.cuda.current_stream(dev)
xa = _lib.ptr_array([x.data_ptr() for x in xs])
oa = _lib.ptr_array([o.data_ptr() for o in outs])
fa = _lib.ptr_array([f.data_ptr() for f in flat.unbind(0)])
bm = [w + 1 for w in range(W)]
nbytes = W * (4 * n + npk * stride) + 4 * n
fbytes = W * (4 * n + npk * 1024) + 4 * n


def product():
    ops.quantize_pack_nga_multi(xs, k, V, bm, W, 1, 1, base=base, num_slots=1 << 17, outs=outs)


def copy_rows():
    assert lab.lab_copy(1, xa, base.data_ptr(), oa, stride, npk, s.cuda_stream) == 0


def copy_flat():
    assert lab.lab_copy(2, xa, base.data_ptr(), fa, 1024, npk, s.cuda_stream) == 0


def timed(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for r in range(4):
    tp, tr, tf = timed(product), timed(copy_rows), timed(copy_flat)
    print(f"round {r}: product {tp:6.1f} us ({nbytes / tp / 8e6:.3f})   copy, product layout "
          f"{tr:6.1f} us ({nbytes / tr / 8e6:.3f})   aligned stream copy {tf:6.1f} us ({fbytes / tf / 8e6:.3f})")
