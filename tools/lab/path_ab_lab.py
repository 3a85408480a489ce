#!/usr/bin/env python3
"""Packet-path A/B (experiment only): bench.py's packet path step (8 workers' quantise + split
NGA-V packs in one launch, the previous step's acks in front, the switch with the PS fused) at
config-3 size through the in-tree libina.so ("A") and other builds (env LIBS=name:path,...),
interleaved over ROUNDS rounds, K back-to-back steps each; per build the step time and the
switch + PS phase alone (HIP events), and the update / actions / ack rows compared byte for
byte with A's.  env V (default 32; slots 2^20, or 2^17 at V = 256)."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

libs = {"A": _lib.load()}
for spec in filter(None, os.environ.get("LIBS", "").split(",")):
    name, path = spec.split(":")
    libs[name] = _lib.open_library(os.path.join(REPO, path))
dev = torch.device("cuda")
V = int(os.environ.get("V", 32))
W, n, k = 8, 26_214_400, 16
slots = (1 << 17) if V == 256 else (1 << 20)
npk = n // V
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 3))
g = torch.Generator(device=dev).manual_seed(6032)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
glob = torch.randn(n, device=dev, generator=g) * 1e-2
ws = 1.0 / (W + 1)


class Step:
    def __init__(self):
        self.hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=dev)
        self.pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=dev)
        self.desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
        self.acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
        self.upd = torch.empty_like(glob)
        self.sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        self.hw = list(self.hdr[npk:].view(W, npk, 16).unbind(0))
        self.pw = list(self.pay[npk:].view(W, npk, 4 * V).unbind(0))
        self.dw = list(self.desc[npk:].view(W, npk).unbind(0))
        ops.nga_descriptors(self.hdr[:npk], out=self.desc[:npk])

    def pack(self):
        ops.quantize_pack_nga_multi_split(xs, k, V, [w + 1 for w in range(W)], W, 1, 1, base=glob, num_slots=slots,
                                          hdrs=self.hw, pays=self.pw, descs=self.dw)

    def switch(self):
        self.sw.process_apply_split(self.hdr, self.pay, 1, glob, k, ws, out=self.upd, ack_hdr=self.hdr[:npk],
                                    ack_desc=self.desc[:npk], keep_forwarded=False, actions=self.acts, desc=self.desc)


def use(name):
    _lib._lib = libs[name]


steps = {}
state = {}
for name in libs:
    use(name)
    st = Step()
    for _ in range(3):
        st.pack()
        st.switch()
    torch.cuda.synchronize()
    state[name] = [x.cpu() for x in (st.upd, st.acts, st.hdr[:npk])]
    steps[name] = st
out = {"V": V, "bytes_equal": {n_: all(torch.equal(a, b) for a, b in zip(state["A"], v)) for n_, v in state.items()}}
res, sw_res = {}, {}
for _ in range(ROUNDS):
    for name, st in steps.items():
        use(name)
        for _ in range(2):
            st.pack()
            st.switch()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(K):
            st.pack()
            st.switch()
        e[1].record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(e[0].elapsed_time(e[1]) * 1e3 / K)
        ev = []
        for _ in range(K):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.pack()
            a.record()
            st.switch()
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        sw_res.setdefault(name, []).append(statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev))
out["step_us"] = {k_: round(statistics.median(v), 2) for k_, v in res.items()}
out["switch_and_ps_us"] = {k_: round(statistics.median(v), 2) for k_, v in sw_res.items()}
out["batch_path"] = steps["A"].sw.batch_path((W + 1) * npk)
use("A")
print(json.dumps(out))
