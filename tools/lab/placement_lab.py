#!/usr/bin/env python3
"""Placement lab (experiment only): does the NGA-32 C3 round-robin split-row switch call's time
follow the byte offsets of its arrays (a channel / bank effect of where the header rows, the
payload rows and the slot registers start), or only their physical pages?  The same batch is
copied into views at chosen offsets inside larger buffers, and each configuration is timed
twice, in two passes over the configurations (HIP events around K back-to-back calls, median of
ROUNDS).  Env: K, ROUNDS, CONFIGS (name=hdr_off:pay_off:reg_off, byte offsets)."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
V, W, n = 32, 8, 26_214_400
slots = 1 << 20
npk = n // V
N = W * npk
K, ROUNDS = int(os.environ.get("K", 10)), int(os.environ.get("ROUNDS", 3))
g = torch.Generator(device=dev).manual_seed(21)
rows, descs = [], []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    rows.append(p)
    descs.append(d)
    del b
base, base_desc = torch.cat(rows), torch.cat(descs)
del rows, descs
rr = torch.arange(N, device=dev).view(W, npk).t().reshape(-1)
stream, desc = base[rr], base_desc[rr]
del base, base_desc
hdr0 = torch.zeros((N, 16), dtype=torch.uint8, device=dev)
hdr0[:, :15] = stream[:, :15]
pay0 = stream[:, 15:15 + 4 * V].contiguous()
del stream
acts = torch.empty(N, dtype=torch.uint8, device=dev)
SLACK = 4 << 20
hbuf = torch.empty(N * 16 + SLACK, dtype=torch.uint8, device=dev)
pbuf = torch.empty(N * 4 * V + SLACK, dtype=torch.uint8, device=dev)


def timed(fn):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(K):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / K


configs = {}
for spec in os.environ.get("CONFIGS", "o0=0:0:0,p4k=0:4096:0,p64k=0:65536:0,p1m=0:1048576:0,"
                                      "h4k=4096:0:0,r4k=0:0:4096,p2m4k=0:2101248:0").split(","):
    name, offs = spec.split("=")
    configs[name] = tuple(int(x) for x in offs.split(":"))
res = {name: [] for name in configs}
for rep in range(2):
    for name, (ho, po, ro) in configs.items():
        hdr = hbuf[ho:ho + N * 16].view(N, 16)
        pay = pbuf[po:po + N * 4 * V].view(N, 4 * V)
        hdr.copy_(hdr0)
        pay.copy_(pay0)
        sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        if ro:
            # the slot registers at an offset inside a larger allocation
            big = torch.zeros(sw.regs.numel() * sw.regs.element_size() + ro, dtype=torch.uint8, device=dev)
            sw.regs = big[ro:].view(sw.regs.dtype).view(sw.regs.shape)
            sw._state = _lib.SwitchState(slots, V, 1, 0, sw.count.data_ptr(), sw.frag.data_ptr(),
                                         sw.regs.data_ptr())
        t = [timed(lambda: sw.process_split(hdr, pay, acts, desc=desc)) for _ in range(ROUNDS)]
        res[name].append(round(statistics.median(t), 2))
        print(rep, name, (ho, po, ro), res[name][-1], sw.batch_path(N), flush=True)
        del sw
print(json.dumps(res))
