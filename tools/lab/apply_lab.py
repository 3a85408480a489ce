#!/usr/bin/env python3
"""Interleaved A/B of PS-side / worker-side fused kernels across libina builds (experiment
only): every tools/lab/libina_*.so given runs ina_apply_completed_nga on the switch output
of an 8-worker NGA-256 stream and ina_quantize_pack_nga on a ResNet-50 delta; outputs must
agree across builds."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
n, W, V = 26_214_400, 8, 256
bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
stream = torch.cat([ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=1 << 17) for w, b in enumerate(bufs)])
del bufs
sw = ops.Switch(V, num_slots=1 << 17, switch_id=1, device=dev)
acts = sw.process(stream)
assert int((acts == _lib.ACT_FWD_AGG).sum()) == n // V, "every slot completes once"
npk_all, stride = stream.shape
nslot = n // V
local = torch.randn(n, device=dev, generator=g)
nr = 25_557_032
xr = torch.randn(nr, device=dev, generator=g) * 1e-2
br = torch.randn(nr, device=dev, generator=g) * 1e-2
st = torch.cuda.current_stream().cuda_stream
src_i32 = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)


class Variant:
    def __init__(self, path):
        self.name = os.path.basename(path)
        self.lib = C.CDLL(path)
        if os.environ.get("STREAM_BLOCKS"):
            self.lib.ina_set_tuning(4, int(os.environ["STREAM_BLOCKS"]))
        for nm in ("ina_apply_completed_nga", "ina_quantize_pack_nga", "ina_pack_nga", "ina_unpack_nga"):
            getattr(self.lib, nm).argtypes = _lib.SIGNATURES[nm]
        self.out = torch.empty_like(local)
        self.acks = torch.empty((nslot, stride), dtype=torch.uint8, device=dev)
        self.pk = torch.empty(((nr + V - 1) // V, stride), dtype=torch.uint8, device=dev)
        self.prm = _lib.NgaParams(1, 8, 0, 1, 0, 1, 16384, V)
        self.t = {"apply": [], "qpack": [], "pack": [], "unpack": []}
        self.pk3 = torch.empty((n // V, stride), dtype=torch.uint8, device=dev)
        self.vals = torch.empty(n, dtype=torch.int32, device=dev)

    def apply(self):
        return self.lib.ina_apply_completed_nga(stream.data_ptr(), npk_all, V, stride, acts.data_ptr(), 1,
                                                local.data_ptr(), 16, 0.1, self.out.data_ptr(), n,
                                                self.acks.data_ptr(), stride, st)

    def pack(self):
        return self.lib.ina_pack_nga(src_i32.data_ptr(), n, C.byref(self.prm), None, self.pk3.data_ptr(),
                                     stride, st)

    def unpack(self):
        return self.lib.ina_unpack_nga(self.pk3.data_ptr(), n // V, V, stride, None, self.vals.data_ptr(), st)

    def qpack(self):
        return self.lib.ina_quantize_pack_nga(xr.data_ptr(), br.data_ptr(), nr, 16, C.byref(self.prm),
                                              self.pk.data_ptr(), stride, st)


vs = [Variant(p) for p in sys.argv[1:]]
for v in vs:
    v.out.fill_(float("nan"))
    assert v.apply() == 0 and v.qpack() == 0 and v.pack() == 0 and v.unpack() == 0
torch.cuda.synchronize()
bad = False
for v in vs[1:]:
    if not (torch.equal(v.pk3, vs[0].pk3) and torch.equal(v.vals, vs[0].vals)):
        print("pack/unpack differ:", v.name)
        bad = True
    if not torch.equal(v.pk, vs[0].pk):
        print("qpack differs:", v.name, int((v.pk != vs[0].pk).sum()))
        bad = True
    d = (v.out.view(torch.int32) != vs[0].out.view(torch.int32)).nonzero().flatten()
    if d.numel():
        i = int(d[0])
        print("apply differs:", v.name, d.numel(), "first", i, "slot", i // V, float(v.out[i]), float(vs[0].out[i]),
              "last", int(d[-1]))
        bad = True

if bad:
    sys.exit(1)
for r in range(int(os.environ.get("ROUNDS", 8))):
    for v in vs:
        for op in ("apply", "qpack", "pack", "unpack"):
            evs = []
            for _ in range(4):
                ops.checksum(flush)                  # cold caches (read-only flush)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert getattr(v, op)() == 0
                b.record()
                evs.append((a, b))
            torch.cuda.synchronize()
            v.t[op] += [a.elapsed_time(b) * 1e3 for a, b in evs[1:]]
for v in vs:
    print(f"{v.name:22s} " + "  ".join(f"{op} {statistics.median(v.t[op]):6.1f} us" for op in v.t))
