#!/usr/bin/env python3
"""Interleaved A/B of the one-in one-out elementwise kernels (quantise, dequantise, PS
apply) across libina builds (experiment only); cold caches, outputs must agree."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
n = 26_214_400
g = torch.Generator(device=dev).manual_seed(9)
x = torch.randn(n, device=dev, generator=g) * 1e-2
q = torch.randint(-(1 << 24), 1 << 24, (n,), dtype=torch.int32, device=dev, generator=g)
local = torch.randn(n, device=dev, generator=g)
flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
n2 = 25_557_032                                   # config 2: ResNet-50 fp32, W = 4
b4 = [torch.randn(n2, device=dev, generator=g) * 1e-2 for _ in range(4)]
arr4 = (C.c_void_p * 4)(*[b.data_ptr() for b in b4])
loc2 = torch.randn(n2, device=dev, generator=g)
b16 = b4 + [torch.randn(n2, device=dev, generator=g) * 1e-2 for _ in range(12)]
arr16 = (C.c_void_p * 16)(*[b.data_ptr() for b in b16])
st = torch.cuda.current_stream().cuda_stream
K16 = int(os.environ.get("K16", 13))       # C4 scale; 20 saturates often (flag check)
ONLY = os.environ.get("ONLY", "").split(",") if os.environ.get("ONLY") else None


class Variant:
    def __init__(self, path):
        self.name = os.path.basename(path)
        self.lib = C.CDLL(path)
        for nm in ("ina_quantize_f32_i32", "ina_dequantize_i32_f32", "ina_ps_apply_i32",
                   "ina_quantize_reduce_f32_i32", "ina_ps_combine_f32", "ina_ps_combine_ina_f32",
                   "ina_quantize_reduce_f32_i16_sat", "ina_quantize_f32_i16_sat"):
            getattr(self.lib, nm).argtypes = _lib.SIGNATURES[nm]
        self.oq = torch.empty(n, dtype=torch.int32, device=dev)
        self.of = torch.empty(n, device=dev)
        self.oa = torch.empty(n, device=dev)
        self.oqr = torch.empty(n2, dtype=torch.int32, device=dev)
        self.oc = torch.empty(n2, device=dev)
        self.oci = torch.empty(n2, device=dev)
        self.o16 = torch.empty(n2, dtype=torch.int16, device=dev)
        self.f16 = torch.empty((n2 + 255) // 256, dtype=torch.uint8, device=dev)
        self.q16 = torch.empty(n, dtype=torch.int16, device=dev)
        self.fq16 = torch.empty((n + 255) // 256, dtype=torch.uint8, device=dev)
        self.t = {"quantize": [], "dequantize": [], "ps_apply": [], "qreduce_C2": [], "combine": [],
                  "combine_ina": [], "qreduce_C4": [], "quantize16": [], "quantize16_noflags": []}
        for key, env in ((5, "COMBINE_BLOCKS"), (6, "COMBINE_INA_BLOCKS"), (4, "STREAM_BLOCKS")):
            if os.environ.get(env):
                self.lib.ina_set_tuning(key, int(os.environ[env]))

    def quantize(self):
        return self.lib.ina_quantize_f32_i32(x.data_ptr(), self.oq.data_ptr(), n, 16, st)

    def dequantize(self):
        return self.lib.ina_dequantize_i32_f32(q.data_ptr(), self.of.data_ptr(), n, 16, st)

    def qreduce_C2(self):
        return self.lib.ina_quantize_reduce_f32_i32(arr4, 4, self.oqr.data_ptr(), n2, 16, st)

    def combine(self):
        return self.lib.ina_ps_combine_f32(loc2.data_ptr(), arr4, 4, 0.2, self.oc.data_ptr(), n2, st)

    def combine_ina(self):
        return self.lib.ina_ps_combine_ina_f32(loc2.data_ptr(), arr4, 4, 16, 0.2, self.oci.data_ptr(), n2, st)

    def qreduce_C4(self):
        return self.lib.ina_quantize_reduce_f32_i16_sat(arr16, 16, self.o16.data_ptr(), n2, K16, 256,
                                                        self.f16.data_ptr(), st)

    def quantize16(self):
        return self.lib.ina_quantize_f32_i16_sat(x.data_ptr(), self.q16.data_ptr(), n, K16 + 2, 256,
                                                 self.fq16.data_ptr(), st)

    def quantize16_noflags(self):
        return self.lib.ina_quantize_f32_i16_sat(x.data_ptr(), self.q16.data_ptr(), n, K16 + 2, 256,
                                                 None, st)

    def ps_apply(self):
        return self.lib.ina_ps_apply_i32(local.data_ptr(), q.data_ptr(), 16, 0.1, self.oa.data_ptr(), n, st)


vs = [Variant(p) for p in sys.argv[1:]]
for v in vs:
    assert v.quantize() == 0 and v.dequantize() == 0 and v.ps_apply() == 0 and v.qreduce_C2() == 0
    assert v.combine() == 0 and v.combine_ina() == 0 and v.qreduce_C4() == 0 and v.quantize16() == 0
torch.cuda.synchronize()
for v in vs[1:]:
    assert torch.equal(v.oq, vs[0].oq) and torch.equal(v.of, vs[0].of) and torch.equal(v.oa, vs[0].oa), v.name
    assert torch.equal(v.oqr, vs[0].oqr), v.name
    assert torch.equal(v.oc, vs[0].oc) and torch.equal(v.oci, vs[0].oci), v.name
    assert torch.equal(v.o16, vs[0].o16) and torch.equal(v.f16, vs[0].f16), v.name
    assert torch.equal(v.q16, vs[0].q16) and torch.equal(v.fq16, vs[0].fq16), v.name
for r in range(int(os.environ.get("ROUNDS", 6))):
    for v in vs:
        for op in v.t:
            if ONLY and op not in ONLY:
                continue
            evs = []
            for _ in range(4):
                ops.checksum(flush)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert getattr(v, op)() == 0
                b.record()
                evs.append((a, b))
            torch.cuda.synchronize()
            v.t[op] += [a.elapsed_time(b) * 1e3 for a, b in evs[1:]]
for v in vs:
    print(f"{v.name:16s} " + "  ".join(f"{op} {statistics.median(v.t[op]):6.1f} us" for op in v.t if v.t[op]))
print("C4 slots flagged:", int(vs[0].f16.sum()), "of", vs[0].f16.numel(),
      "| quantize16 slots flagged:", int(vs[0].fq16.sum()), "of", vs[0].fq16.numel())
