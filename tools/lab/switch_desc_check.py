import os, sys, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/distributed-training-ina_amd")
import torch
from ina_amd import ops
import bench_extra as be
n, V, Ws = 26_214_400, 256, 8
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
packed = [ops.pack_nga(torch.randint(-(1<<20), 1<<20, (n,), dtype=torch.int32, device=dev, generator=g), V, w + 1, Ws, 1, 1, num_slots=1 << 17, desc=True) for w in range(Ws)]
stream = torch.cat([p for p, _ in packed]); desc_all = torch.cat([d for _, d in packed]); del packed
sw = ops.Switch(V, num_slots=1 << 17, switch_id=1, device=dev)
acts = torch.empty(stream.shape[0], dtype=torch.uint8, device=dev)
res = {}
for rnd in range(3):
    for name, d in (("desc", desc_all), ("hdr", None)):
        for cold in (True, False):
            t = be._time(lambda: sw.process(stream, acts, desc=d), reps=5, warm=1, cold=cold)
            res.setdefault(f"{name}_cold{int(cold)}", []).append(round(t * 1e6, 1))
print(json.dumps(res))
