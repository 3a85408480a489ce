#!/usr/bin/env python3
"""Lab (experiment only): does the allocation history of the process move the NGA-256 worker
packs and the NGA-256 switch, the two phases whose times differ 7-10 % between sessions while the
streaming kernels agree within 2 %?  The same measurements -- the
8 workers' fused quantise + split packs (k_qpack_nga_multi_split<8>, one launch), the steady-state
switch + PS pass over their batch, and the switch alone on the round-robin NGA-256 batch (packed
rows, in slot order) -- each a median of 20 event-timed launches, are taken (1) in a fresh
process, (2) after ~90 GB of tensors of random sizes were allocated and all freed with
empty_cache() (what bench.py's earlier legs do), (3) with every other one of those tensors
still alive (fragmented free space), (4) again after all are freed."""
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
W, n, k, V, slots = 8, 26_214_400, 16, 256, 1 << 17
npk = n // V


def ev_median(fn, reps=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return round(statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3, 1)


def measure():
    g = torch.Generator(device=dev).manual_seed(6000)
    xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
    glob = torch.randn(n, device=dev, generator=g) * 1e-2
    upd = torch.empty_like(glob)
    hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=dev)
    pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=dev)
    ack_rows = hdr[:npk]
    hdrs_w, pays_w = list(hdr[npk:].view(W, npk, 16).unbind(0)), list(pay[npk:].view(W, npk, 4 * V).unbind(0))
    desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
    desc_ack, descs_w = desc[:npk], list(desc[npk:].view(W, npk).unbind(0))
    acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    bms = [w + 1 for w in range(W)]

    def pack():
        ops.quantize_pack_nga_multi_split(xs, k, V, bms, W, 1, 1, base=glob, num_slots=slots,
                                          hdrs=hdrs_w, pays=pays_w, descs=descs_w)

    def switch():
        sw.process_apply_split(hdr, pay, 1, glob, k, 1.0 / (W + 1), out=upd, ack_hdr=ack_rows, ack_desc=desc_ack,
                               keep_forwarded=False, actions=acts, desc=desc)
    ops.nga_descriptors(ack_rows, out=desc_ack)
    pack()
    switch()
    out = {"worker_packs_us": ev_median(pack)}

    def step():
        pack()
        switch()
    for _ in range(3):
        step()
    s = torch.cuda.current_stream()
    evs = []
    for _ in range(20):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        pack()
        e[0].record(s)
        switch()
        e[1].record(s)
        evs.append(e)
    torch.cuda.synchronize()
    out["switch_and_ps_us"] = round(statistics.median(a.elapsed_time(b) for a, b in evs) * 1e3, 1)
    del xs, glob, upd, hdr, pay, hdrs_w, pays_w, desc, descs_w, acts, sw
    torch.cuda.empty_cache()
    # the round-robin NGA-256 batch, packed rows (bench switch_c3.round_robin)
    bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
    packed = [ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True) for w, b in enumerate(bufs)]
    del bufs
    stream = torch.cat([p for p, _ in packed])
    dsc = torch.cat([d for _, d in packed])
    del packed
    rr = torch.arange(W * npk, device=dev).view(W, npk).t().reshape(-1)
    stream, dsc = stream[rr].contiguous(), dsc[rr].contiguous()
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    a = torch.empty(W * npk, dtype=torch.uint8, device=dev)
    out["switch_rr_us"] = ev_median(lambda: sw.process(stream, a, desc=dsc))
    out["switch_rr_path"] = sw.batch_path(W * npk)
    del stream, dsc, sw, a, rr
    torch.cuda.empty_cache()
    return out


res = {"fresh": measure()}
print(json.dumps(res), flush=True)
g = torch.Generator().manual_seed(3)
junk, total = [], 0
while total < 90 << 30:
    sz = int(torch.randint(1 << 20, 512 << 20, (1,), generator=g))
    junk.append(torch.empty(sz, dtype=torch.uint8, device=dev))
    total += sz
junk = []
torch.cuda.empty_cache()
res["after_90GB_freed"] = measure()
print(json.dumps(res), flush=True)
total = 0
while total < 90 << 30:
    sz = int(torch.randint(1 << 20, 512 << 20, (1,), generator=g))
    junk.append(torch.empty(sz, dtype=torch.uint8, device=dev))
    total += sz
junk = junk[::2]
res["half_of_90GB_alive"] = measure()
print(json.dumps(res), flush=True)
junk = []
torch.cuda.empty_cache()
res["all_freed_again"] = measure()
print(json.dumps(res))
