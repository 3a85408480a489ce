#!/usr/bin/env python3
"""Detection-pass tail lab (experiment only): is the NGA-32 detection pass (k_sort_chunks mode 1,
one 16-wave block per 8,192-packet chunk, two blocks resident per CU = 512 at once) paying for
its last partial round of blocks?  Round-robin NGA-32 split-row batches of nch chunks (a prefix
of one 8-worker round-robin stream, 2^20 slots, descriptors) for nch around 512 and 800 (config
3), K process_split calls each.  Run under rocprofv3 --kernel-trace: the trace's grid size names
nch (grid = nch x 1,024 threads); HIP events give each size's call time beside it."""
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
V, W, CH = 32, 8, 8192
slots = 1 << 20
NCH = [int(x) for x in os.environ.get("NCH", "256,384,448,480,512,528,576,640,704,768,800,1024").split(",")]
K = int(os.environ.get("K", 20))
per_w = max(NCH) * CH // W                      # packets per worker
g = torch.Generator(device=dev).manual_seed(77)
rows, descs = [], []
for w in range(W):
    b = torch.randint(-(1 << 20), 1 << 20, (per_w * V,), dtype=torch.int32, device=dev, generator=g)
    p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
    rows.append(p)
    descs.append(d)
    del b
stream = torch.stack(rows, 1).reshape(W * per_w, -1)        # round-robin: packet i of every worker
desc = torch.stack(descs, 1).reshape(-1)
del rows, descs
hdr_all = torch.zeros((W * per_w, 16), dtype=torch.uint8, device=dev)
hdr_all[:, :15] = stream[:, :15]
pay_all = stream[:, 15:15 + 4 * V].contiguous()
del stream
out = {}
for nch in NCH:
    n = nch * CH
    hdr, pay, ds = hdr_all[:n], pay_all[:n], desc[:n]
    acts = torch.empty(n, dtype=torch.uint8, device=dev)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    for _ in range(3):
        sw.process_split(hdr, pay, acts, desc=ds)
    res = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            sw.process_split(hdr, pay, acts, desc=ds)
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / K)
    out[nch] = {"npk": n, "call_us": round(statistics.median(res), 2), "path": sw.batch_path(n)}
    print(nch, json.dumps(out[nch]), flush=True)
    del sw, acts
    torch.cuda.empty_cache()
print(json.dumps(out))
