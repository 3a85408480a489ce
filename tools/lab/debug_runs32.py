#!/usr/bin/env python3
"""Debug helper (experiment only): one NGA-32 batch of R dense runs through the device switch
and the oracle; prints where the rewritten rows differ (row, byte offsets, both byte strings)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
sys.path.insert(0, REPO)
from ina_amd import ops  # noqa: E402
from oracle import oracle as orc  # noqa: E402

V = 32
POOL = 1 << 17
stride = ops.nga_stride(V)
for R, collide, mix in ((2, 0.0, 0.0), (2, 0.02, 0.02), (8, 0.0, 0.0)):
    rng = np.random.default_rng(5)
    per = 1000
    parts = []
    for w in range(R):
        vals = rng.integers(-2**31, 2**31, size=per * V, dtype=np.int64).astype(np.int32)
        parts.append(orc.pack_nga(vals, V, w + 1, R, 1, 5, num_slots=POOL, stride=stride))
    pk = np.concatenate(parts)
    for i in np.flatnonzero(rng.random(len(pk)) < collide):
        f = int.from_bytes(pk[i, 11:15].tobytes(), "big") + 1
        pk[i, 11:15] = np.frombuffer((f & 0xFFFFFFFF).to_bytes(4, "big"), np.uint8)
    for i in np.flatnonzero(rng.random(len(pk)) < mix):
        pk[i, 4] = int(rng.choice([1, 2]))
    sw_o = orc.Switch(V, num_slots=POOL, switch_id=1)
    want_pk, want_act = sw_o.run(pk, stride=stride)
    sw = ops.Switch(V, num_slots=POOL, switch_id=1, device=torch.device("cuda"), write_dropped=True)
    d = torch.from_numpy(pk.copy()).cuda()
    act = sw.process(d, desc=ops.nga_descriptors(d))
    got = d.cpu().numpy()
    print(f"R={R} collide={collide} path={sw.batch_path(len(pk))} actions_equal={np.array_equal(act.cpu().numpy(), want_act)}")
    bad = np.argwhere(got != want_pk)
    print("  mismatching bytes:", len(bad))
    rows = np.unique(bad[:, 0])[:4]
    for r in rows:
        cols = bad[bad[:, 0] == r][:, 1]
        print(f"  row {r} (worker {r // per}, slot {5 + r % per}) act {want_act[r]} cols {cols[:12].tolist()} ... ({len(cols)})")
        print("   orig", pk[r, :40].tolist())
        print("   want", want_pk[r, :40].tolist())
        print("   got ", got[r, :40].tolist())
    cnt, frag, regs = sw_o.registers()
    print("  regs equal:", np.array_equal(sw.regs.cpu().numpy().view(np.uint32), regs),
          "count equal:", np.array_equal(sw.count.cpu().numpy(), cnt))
