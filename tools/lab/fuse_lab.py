#!/usr/bin/env python3
"""Interleaved A/B of ina_switch with a PS step across libina builds (experiment only):
8 workers x NGA-256 packets of a config-3 bucket, PS step fused; switch state reset
between launches; outputs must agree."""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
n, W, V, slots = 26_214_400, 8, 256, 1 << 17
g = torch.Generator(device=dev).manual_seed(2)
bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
stream = torch.cat([ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots) for w, b in enumerate(bufs)])
del bufs
npk_all, stride = stream.shape
local = torch.randn(n, device=dev, generator=g)
st = torch.cuda.current_stream().cuda_stream
# every variant runs on the SAME buffers (only the library differs): with buffers per
# variant the first variant's placement ran ~7 % faster than any later one's, even for two
# copies of one library (profiles/r02/lab/fuse_lab_position.log)
early = None
if os.environ.get("SCRATCH_FIRST"):         # placement probe: scratch before the other buffers
    early = torch.empty(_lib.load().ina_switch_scratch_bytes(npk_all, slots) + (1 << 20), dtype=torch.uint8,
                        device=dev)
shared = dict(count=torch.zeros(slots, dtype=torch.uint8, device=dev),
              frag=torch.zeros(slots, dtype=torch.int32, device=dev),
              regs=torch.zeros((slots, V), dtype=torch.int32, device=dev),
              acts=torch.empty(npk_all, dtype=torch.uint8, device=dev), out=torch.empty_like(local),
              acks=torch.empty((n // V, stride), dtype=torch.uint8, device=dev))
shared["st"] = _lib.SwitchState(slots, V, 1, 0, shared["count"].data_ptr(), shared["frag"].data_ptr(),
                                shared["regs"].data_ptr())
scratch_bytes = 0
vs = []
for p in sys.argv[1:]:
    lib = C.CDLL(p)
    for nm in ("ina_switch", "ina_switch_scratch_bytes"):
        getattr(lib, nm).argtypes = _lib.SIGNATURES[nm]
    lib.ina_switch_scratch_bytes.restype = C.c_size_t
    scratch_bytes = max(scratch_bytes, lib.ina_switch_scratch_bytes(npk_all, slots))
    vs.append(dict(shared, name=os.path.basename(p), lib=lib, t=[]))
shared["scratch"] = early if early is not None and early.numel() >= scratch_bytes else \
    torch.empty(scratch_bytes, dtype=torch.uint8, device=dev)
for v in vs:
    v["scratch"] = shared["scratch"]


def run(v):
    v["count"].zero_()
    v["frag"].zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    b = _lib.SwitchBatch(stream.data_ptr(), None, npk_all, stride, None, v["acts"].data_ptr(),
                         v["scratch"].data_ptr())
    ps = _lib.SwitchPs(1, 16, 0.125, local.data_ptr(), v["out"].data_ptr(), n, v["acks"].data_ptr(), stride,
                       None, 0)
    rc = v["lib"].ina_switch(C.byref(v["st"]), C.byref(b), C.byref(ps), _lib.INA_SWITCH_ALL, st)
    e1.record()
    assert rc == 0
    return e0, e1


ref = None
for v in vs:
    run(v)
    torch.cuda.synchronize()
    got = (v["out"].clone(), v["acks"][:, :16].clone(), v["acts"].clone())
    if ref is None:
        ref = got
    else:
        assert all(torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                               b.view(torch.int32) if b.dtype == torch.float32 else b)
                   for a, b in zip(got, ref)), v["name"]
for r in range(int(os.environ.get("ROUNDS", 6))):
    for v in vs:
        evs = [run(v) for _ in range(4)]
        torch.cuda.synchronize()
        v["t"] += [a.elapsed_time(b) * 1e3 for a, b in evs[1:]]
for v in vs:
    print(f"{v['name']:18s} switch+PS fused {statistics.median(v['t']):7.1f} us")

# the same work as two calls (in-tree library): switch, then the PS apply kernel
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts2 = torch.empty(npk_all, dtype=torch.uint8, device=dev)
out2 = torch.empty_like(local)
acks2 = torch.empty((n // V, stride), dtype=torch.uint8, device=dev)
pk2 = stream.clone()
t2 = []
for r in range(int(os.environ.get("ROUNDS", 6)) * 3):
    sw.count.zero_()
    sw.frag.zero_()
    pk2.copy_(stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    sw.process(pk2, acts2)
    ops.apply_completed(pk2, acts2, V, 1, local, 16, 0.125, out=out2, acks=acks2)
    e1.record()
    torch.cuda.synchronize()
    t2.append(e0.elapsed_time(e1) * 1e3)
assert torch.equal(out2.view(torch.int32), ref[0].view(torch.int32))
print(f"{'two calls':18s} switch, apply     {statistics.median(t2):7.1f} us")
