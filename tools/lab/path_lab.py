#!/usr/bin/env python3
"""Stage times of the one-GPU INA packet path step (experiment only): 8 x fused
quantise+pack -> switch -> PS apply -> acks through the switch; HIP events between
stages, median over repetitions."""
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
n3, Ws, V = 26_214_400, 8, 256
npk = n3 // V
stride = ops.nga_stride(V)
g = torch.Generator(device=dev).manual_seed(3)
xs = [torch.randn(n3, device=dev, generator=g) * 1e-2 for _ in range(Ws)]
glob_p = torch.randn(n3, device=dev, generator=g)
upd = torch.empty_like(glob_p)
stream = torch.empty((Ws * npk, stride), dtype=torch.uint8, device=dev)
rows_w = stream.view(Ws, npk, stride)
acts = torch.empty(Ws * npk, dtype=torch.uint8, device=dev)
acks = torch.empty((npk, stride), dtype=torch.uint8, device=dev)
ack_acts = torch.empty(npk, dtype=torch.uint8, device=dev)
sw = ops.Switch(V, num_slots=1 << 17, switch_id=1, device=dev)
names = ["qpack x8", "switch", "apply", "ack switch"]
WIN_DATA = int(os.environ.get("WIN_DATA", 0))    # switch run-kernel window (0 = auto)
WIN_ACK = int(os.environ.get("WIN_ACK", 0))
ts = {k: [] for k in names}
for rep in range(int(os.environ.get("REPS", 12))):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    ev[0].record()
    for w in range(Ws):
        ops.quantize_pack_nga(xs[w], 16, V, w + 1, Ws, 1, 1, base=glob_p, num_slots=1 << 17, out=rows_w[w])
    ev[1].record()
    ops.set_tuning(switch_window=WIN_DATA)
    sw.process(stream, acts)
    ev[2].record()
    ops.apply_completed(stream, acts, V, 1, glob_p, 16, 1.0 / (Ws + 1), out=upd, acks=acks)
    ev[3].record()
    ops.set_tuning(switch_window=WIN_ACK)
    sw.process(acks, ack_acts)
    ev[4].record()
    torch.cuda.synchronize()
    if rep >= 2:
        for i, k in enumerate(names):
            ts[k].append(ev[i].elapsed_time(ev[i + 1]) * 1e3)
assert int((acts == 1).sum()) == npk and bool((ack_acts == 3).all()) and not bool(sw.frag.any())
print(f"win data {WIN_DATA:2d} ack {WIN_ACK:2d}: " + "  ".join(f"{k} {statistics.median(v):7.1f} us" for k, v in ts.items()),
      f" total {sum(statistics.median(v) for v in ts.values()):7.1f} us")
