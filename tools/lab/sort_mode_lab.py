#!/usr/bin/env python3
"""Slot-sort lab (experiment only): a shuffled config-3 batch (NGA-32: 6,553,600 packets,
2^20 slots; NGA-256: 819,200 packets, 2^17 slots) through ina_switch_process with the chunk +
bucket sort (tuning key 12 = 0, the default) and the LSD digit passes (key 12 = 3), and the
chunk pass at 2,048-packet chunks (key 13 = 8; the default plan takes 4,096).  Same batch, results
compared byte for byte; HIP events around K back-to-back calls, interleaved over rounds."""
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
W, n = 8, 26_214_400
K, ROUNDS = int(os.environ.get("K", 8)), int(os.environ.get("ROUNDS", 4))
VARIANTS = {"bucket": dict(switch_sort=0), "lsd": dict(switch_sort=3),
            "bucket_r8": dict(switch_sort=0, switch_sort_rounds=8)}
out = {}
for V, slots in ((32, 1 << 20), (256, 1 << 17)):
    npk = n // V
    g = torch.Generator(device=dev).manual_seed(7)
    rows, descs = [], []
    for w in range(W):
        b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
        p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
        rows.append(p)
        descs.append(d)
        del b
    base, base_desc = torch.cat(rows), torch.cat(descs)
    del rows, descs
    perm = torch.randperm(W * npk, device=dev, generator=g)
    stream, desc = base[perm], base_desc[perm]
    del base, base_desc
    acts = torch.empty(W * npk, dtype=torch.uint8, device=dev)
    ref = None
    for name, tun in VARIANTS.items():
        ops.set_tuning(**tun)
        sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        st = stream.clone()
        a = sw.process(st, desc=desc)
        got = [a.cpu(), st.cpu(), sw.regs.cpu()]
        if ref is None:
            ref = got
        out[f"V{V}/{name}/bytes_equal"] = all(torch.equal(x, y) for x, y in zip(got, ref))
        out[f"V{V}/{name}/path"] = sw.batch_path(W * npk)
        del sw, st, a, got
    ops.set_tuning(switch_sort=0, switch_sort_rounds=0)
    sws = {name: ops.Switch(V, num_slots=slots, switch_id=1, device=dev) for name in VARIANTS}
    res = {}
    for r in range(ROUNDS):
        for name, tun in VARIANTS.items():
            ops.set_tuning(**tun)
            sw = sws[name]
            for _ in range(2):
                sw.process(stream, acts, desc=desc)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                sw.process(stream, acts, desc=desc)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(f"V{V}/{name}/us", []).append(e0.elapsed_time(e1) * 1e3 / K)
    ops.set_tuning(switch_sort=0, switch_sort_rounds=0)
    out.update({k: round(statistics.median(v), 2) for k, v in res.items()})
    del sws, stream, desc, acts, ref
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
