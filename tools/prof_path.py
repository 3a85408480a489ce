"""Profile target: the one-GPU INA packet path in steady state with the PS step fused into
the switch pass (the 8 workers' fused quantise+packs in one launch, one ina_switch with a PS step over
[last step's acks | 8 x 102,400 NGA-256 packets]); run under rocprofv3 --kernel-trace
--stats for the per-kernel breakdown of bench_extra's last packet-path row).  The run kernel
writes the ack rows' descriptors (ack_desc), as bench.py's packet_path does.  SPLIT=1: the
same step over split rows (16-byte header rows + 1 KiB payload rows).  V=32: NGA-32 packets
(8 x 819,200 + 819,200 acks, a 2^20-slot pool), bench.py's packet_path_v32."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

n, W = 26_214_400, 8
V = int(os.environ.get("V", 256))
slots = (1 << 17) if V == 256 else (1 << 20)
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
params = torch.randn(n, device=dev, generator=g)
npk = n // V
stride = ops.nga_stride(V)
split = os.environ.get("SPLIT", "0") == "1"
if split:
    hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=dev)      # [acks | workers]
    pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=dev)
    acks = hdr[:npk]
    hdrs_w, pays_w = list(hdr[npk:].view(W, npk, 16).unbind(0)), list(pay[npk:].view(W, npk, 4 * V).unbind(0))
else:
    batch = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=dev)
    acks, rows = batch[:npk], batch[npk:].view(W, npk, stride)
acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)     # packet descriptors
desc_ack, desc_w = desc[:npk], desc[npk:].view(W, npk)
out = torch.empty_like(params)
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
ops.nga_descriptors(acks, out=desc_ack)          # the first step's ack rows are another switch's
for step in range(int(os.environ.get("STEPS", 6))):
    if split:
        ops.quantize_pack_nga_multi_split(xs, 16, V, [w + 1 for w in range(W)], W, 1, 1, base=params,
                                          num_slots=slots, hdrs=hdrs_w, pays=pays_w, descs=list(desc_w.unbind(0)))
        sw.process_apply_split(hdr, pay, 1, params, 16, 1.0 / (W + 1), out=out, ack_hdr=acks, ack_desc=desc_ack,
                               keep_forwarded=False, actions=acts, desc=desc)
    else:
        ops.quantize_pack_nga_multi(xs, 16, V, [w + 1 for w in range(W)], W, 1, 1, base=params,
                                    num_slots=slots, outs=list(rows.unbind(0)), descs=list(desc_w.unbind(0)))
        sw.process_apply(batch, 1, params, 16, 1.0 / (W + 1), out=out, acks=acks, keep_forwarded=False,
                         actions=acts, desc=desc, ack_desc=desc_ack)
torch.cuda.synchronize()
assert int((acts[npk:] == 1).sum()) == npk and bool((acts[:npk] == 3).all())
print("done", "split" if split else "packed", (W + 1) * npk)
