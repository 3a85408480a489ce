"""Lab: the packet path's 8 worker quantise + packs as 8 launches (ina_quantize_pack_nga_desc
per worker) vs ONE launch (ina_quantize_pack_nga_multi), alone and inside the steady-state
step (acks in front, switch + PS fused), alternated; plus a grid sweep of the one launch.
Config-3 sizes (8 x 26,214,400 fp32, V = 256, 2^17 slots).  Prints one line per
measurement."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
W, n, V, k, slots = 8, 26214400, 256, 16, 1 << 17
npk = n // V
g = torch.Generator(device=dev)
g.manual_seed(6000)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
glob = torch.randn(n, device=dev, generator=g) * 1e-2
upd = torch.empty_like(glob)
stride = ops.nga_stride(V)
big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=dev)
ack_rows, rows_w = big[:npk], big[npk:].view(W, npk, stride)
desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
desc_ack, desc_w = desc[:npk], desc[npk:].view(W, npk)
outs, descs = list(rows_w.unbind(0)), list(desc_w.unbind(0))
acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
ws = 1.0 / (W + 1)
s = torch.cuda.current_stream(dev)


def packs8():
    for w in range(W):
        ops.quantize_pack_nga(xs[w], k, V, w + 1, W, 1, 1, base=glob, num_slots=slots,
                              out=outs[w], desc=descs[w])


def packs1():
    ops.quantize_pack_nga_multi(xs, k, V, [w + 1 for w in range(W)], W, 1, 1, base=glob,
                                num_slots=slots, outs=outs, descs=descs)


def step(pack):
    pack()
    ops.nga_descriptors(ack_rows, out=desc_ack)
    sw.process_apply(big, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False,
                     actions=acts, desc=desc)


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


# bytes: 8 launches read the base 8 times (algorithmic), one launch once
rb = stride
b8 = W * (8 * n + npk * rb)
b1 = W * (4 * n + npk * rb) + 4 * n
packs8()
ref = big.clone(), desc.clone()
packs1()
same = bool(torch.equal(big, ref[0]) and torch.equal(desc, ref[1]))
print(f"bytes equal (8 launches vs one): {same}")
step(packs1)
for r in range(3):
    t8 = timed(packs8)
    t1 = timed(packs1)
    print(f"round {r}: packs alone  8 launches {t8:7.1f} us ({b8 / t8 / 8e6:.3f} of 8 TB/s on its bytes)"
          f"   one launch {t1:7.1f} us ({b1 / t1 / 8e6:.3f})")
    s8 = timed(lambda: step(packs8), reps=10, warm=3)
    s1 = timed(lambda: step(packs1), reps=10, warm=3)
    print(f"round {r}: steady step  8 launches {s8:7.1f} us   one launch {s1:7.1f} us")
for gb in (4096, 8192, 16384, 32768, 65536):
    ops.set_tuning(stream_blocks=gb)
    t1 = timed(packs1)
    print(f"grid {gb:6d}: one launch {t1:7.1f} us ({b1 / t1 / 8e6:.3f})")
ops.set_tuning(stream_blocks=16384)

# variants of the one launch (tools/lab/libina_qpm_<layout>_<store>.so: flat chunk stream or a
# wave per packet; nt, write-through or default-policy stores), each called through its own library, alone and inside the step, alternated
import ctypes as C  # noqa: E402
from ina_amd import _lib  # noqa: E402
here = os.path.dirname(os.path.abspath(__file__))
libs = {}
for f in sorted(os.listdir(here)):          # libina_qpm_<layout>_<store>[_<grid>].so
    if f.startswith("libina_qpm_") and f.endswith(".so"):
        lib = C.CDLL(os.path.join(here, f))
        lib.ina_quantize_pack_nga_multi.argtypes = _lib.SIGNATURES["ina_quantize_pack_nga_multi"]
        libs[f[len("libina_qpm_"):-3]] = lib
prm = (_lib.NgaParams * W)(*[_lib.NgaParams(w + 1, W, 0, 1, 0, 1, slots, V) for w in range(W)])
xa = _lib.ptr_array([x.data_ptr() for x in xs])
oa = _lib.ptr_array([o.data_ptr() for o in outs])
da = _lib.ptr_array([d.data_ptr() for d in descs])


def via(lib):
    def f():
        assert lib.ina_quantize_pack_nga_multi(xa, W, glob.data_ptr(), n, k, prm, oa, stride, da,
                                               C.c_void_p(s.cuda_stream)) == 0
    return f


for nm, lib in libs.items():
    via(lib)()
    torch.cuda.synchronize()
    print(f"{nm}: bytes equal {bool(torch.equal(big[npk:], ref[0][npk:]) and torch.equal(desc[npk:], ref[1][npk:]))}")
for r in range(3):
    for nm, lib in libs.items():
        t1 = timed(via(lib))
        st = timed(lambda: step(via(lib)), reps=10, warm=3)
        print(f"round {r}: {nm:12s} one launch {t1:7.1f} us ({b1 / t1 / 8e6:.3f})   steady step {st:7.1f} us")
