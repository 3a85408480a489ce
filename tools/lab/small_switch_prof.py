#!/usr/bin/env python3
"""Profile target (experiment): the device switch on small NGA-32 batches, one-workgroup
sort path vs the radix path (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda")
small = os.environ.get("SMALL", "1") == "1"
ops.set_tuning(switch_small_sort=small)
for nb in (64, 1024, 4096):
    sw = ops.Switch(32, num_slots=16384, switch_id=1, device=dev)
    pk = torch.cat([ops.pack_nga(torch.randint(-99, 99, (32 * nb // 8,), dtype=torch.int32, device=dev),
                                 32, w + 1, 8, 1, 1) for w in range(8)])
    acts = torch.empty(pk.shape[0], dtype=torch.uint8, device=dev)
    for _ in range(20):
        sw.process(pk, acts)
    torch.cuda.synchronize()
print("done")
