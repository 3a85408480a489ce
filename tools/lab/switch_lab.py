#!/usr/bin/env python3
"""Interleaved A/B of device-switch builds (experiment only): every tools/lab/libina_*.so
given on the command line runs ina_switch_process on the same 8-worker NGA-256 stream
(config-3 bucket), timed with HIP events; actions and forwarded packets must agree."""
import ctypes as C
import os
import re
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

n, W, V = int(os.environ.get("N", 26_214_400)), 8, int(os.environ.get("V", 256))
slots = 1 << 17
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
        for _ in range(W)]
src = torch.cat([ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots) for w, b in enumerate(bufs)])
del bufs
if os.environ.get("ORDER", "wm") == "rr":      # a NIC's round-robin interleave of the workers
    src = src.view(W, -1, src.shape[1]).transpose(0, 1).reshape(-1, src.shape[1]).contiguous()
elif os.environ.get("ORDER", "").startswith("wmpad"):   # worker-major, PAD foreign rows between workers
    pad = int(os.environ["ORDER"][5:] or 3)
    rows = src.view(W, -1, src.shape[1])
    filler = rows[0, :pad].clone()
    filler[:, 10] = 7                          # another switch's packets: sorted last, not run
    src = torch.cat([torch.cat([rows[w], filler]) for w in range(W)]).contiguous()
elif os.environ.get("ORDER") == "random":       # uniformly shuffled arrival
    src = src[torch.randperm(src.shape[0], device=dev, generator=torch.Generator(device=dev).manual_seed(9))]
npk, stride = src.shape


SHARED = dict(count=torch.zeros(slots, dtype=torch.uint8, device=dev),
              frag=torch.zeros(slots, dtype=torch.int32, device=dev),
              regs=torch.zeros((slots, V), dtype=torch.int32, device=dev),
              acts=torch.empty(npk, dtype=torch.uint8, device=dev))


class Variant:
    def __init__(self, path):
        self.name = os.path.basename(path)
        self.lib = C.CDLL(path)
        for nm in ("ina_switch_process", "ina_switch_scratch_bytes"):
            getattr(self.lib, nm).argtypes = _lib.SIGNATURES[nm]
        self.lib.ina_switch_scratch_bytes.restype = C.c_size_t
        m = re.search(r"_w(\d+)\.so$", path)       # libina_w<N>.so: run-kernel window N (key 10)
        if m:
            assert self.lib.ina_set_tuning(10, int(m.group(1))) == 0
        # every variant runs on the SAME state, scratch and action buffers (only the library
        # differs): buffer placement alone moved a variant by several % (fuse_lab_position.log)
        self.count, self.frag, self.regs, self.acts = SHARED["count"], SHARED["frag"], SHARED["regs"], SHARED["acts"]
        self.st = _lib.SwitchState(slots, V, 1, 0, self.count.data_ptr(), self.frag.data_ptr(),
                                   self.regs.data_ptr())
        self.scratch_bytes = self.lib.ina_switch_scratch_bytes(npk, slots)
        self.times = []

    def run(self, pk):
        self.count.zero_()
        self.frag.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        rc = self.lib.ina_switch_process(C.byref(self.st), pk.data_ptr(), npk, stride,
                                         self.acts.data_ptr(), self.scratch.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
        b.record()
        assert rc == 0, rc
        return a, b


vs = [Variant(p) for p in sys.argv[1:]]
scratch = torch.empty(max(v.scratch_bytes for v in vs), dtype=torch.uint8, device=dev)
for v in vs:
    v.scratch = scratch
work = src.clone()
ref = None
for v in vs:                                   # correctness: identical outputs
    work.copy_(src)
    v.run(work)
    torch.cuda.synchronize()
    out = (v.acts.clone(), work[v.acts == 1].clone())
    if ref is None:
        ref = out
    else:
        assert torch.equal(ref[0], out[0]) and torch.equal(ref[1], out[1]), v.name
for r in range(int(os.environ.get("ROUNDS", 8))):
    for v in vs:
        evs = []
        for _ in range(3):
            work.copy_(src)
            evs.append(v.run(work))
        torch.cuda.synchronize()
        v.times += [a.elapsed_time(b) * 1e3 for a, b in evs]
for v in vs:
    print(f"{v.name:24s} median {statistics.median(v.times):8.1f} us  min {min(v.times):8.1f} us")
