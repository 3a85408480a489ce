"""Profile target: the device packet-stream switch on 8 workers x NGA-256 packets of
a config-3 bucket (run under rocprofv3 --kernel-trace --stats); the slot sort reads the
pack kernels' packet descriptors (DESC=0: the packet headers).  Env: V, SLOTS, ORDER (wm,
rr, random), RUNS (tuning key 18), SPLIT=1 (split rows: 16-byte headers + 4V-byte payloads)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

n, W, V = int(os.environ.get("N", 26_214_400)), 8, int(os.environ.get("V", 256))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
bufs = [torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
        for _ in range(W)]
slots = int(os.environ.get("SLOTS", 1 << 17))
ops.set_tuning(switch_runs=os.environ.get("RUNS", "1") == "1")
packed = [ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True) for w, b in enumerate(bufs)]
stream = torch.cat([p for p, _ in packed])
desc = torch.cat([d for _, d in packed])     # the pack kernels' packet descriptors
del packed
order = os.environ.get("ORDER", "wm")           # wm: worker-major, rr: round-robin, random
if order != "wm":
    npw = stream.shape[0] // W
    rr = torch.arange(W * npw, device=dev).view(W, npw).t().reshape(-1)
    if order == "rr":
        perm = rr
    elif order.startswith("jit"):       # jitJ: round-robin, each packet displaced by < J positions
        key = torch.arange(W * npw, device=dev) + torch.randint(
            0, int(order[3:]), (W * npw,), device=dev, generator=torch.Generator(device=dev).manual_seed(9))
        perm = rr[torch.sort(key, stable=True).indices]
    else:
        perm = torch.randperm(W * npw, device=dev, generator=torch.Generator(device=dev).manual_seed(9))
    stream, desc = stream[perm].contiguous(), desc[perm].contiguous()
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
acts = torch.empty(stream.shape[0], dtype=torch.uint8, device=dev)
use_desc = os.environ.get("DESC", "1") == "1"
split = os.environ.get("SPLIT", "0") == "1"
if split:
    hdr = torch.zeros((stream.shape[0], 16), dtype=torch.uint8, device=dev)
    hdr[:, :15] = stream[:, :15]
    pay = stream[:, 15:15 + 4 * V].contiguous()
for i in range(int(os.environ.get("REPS", 5))):
    sw.count.zero_()
    sw.frag.zero_()
    if split:
        sw.process_split(hdr, pay, acts, desc=desc if use_desc else None)
    else:
        sw.process(stream, acts, desc=desc if use_desc else None)
torch.cuda.synchronize()
ok = torch.equal(stream.view(W, -1, stream.shape[1])[-1, :, 15:15 + 4 * V].contiguous().view(-1).view(torch.uint8)[:8], stream[stream.shape[0] // W * (W - 1), 15:23])
print("done", stream.shape, int((acts == 1).sum()))
