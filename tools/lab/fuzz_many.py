#!/usr/bin/env python3
"""Extended switch fuzzing (experiment only): the parity tests' fuzz body over many more
seeds, with and without the lone-ack lane path."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
import test_gpu_parity as t  # noqa: E402

lo, hi = int(os.environ.get("LO", 16)), int(os.environ.get("HI", 216))
ops = t.ops()
bad = 0
for ack_fast in (True, False):
    ops.set_tuning(switch_ack_fast=ack_fast)
    for seed in range(lo, hi):
        try:
            t.test_switch_fuzz_vs_oracle(seed)
        except AssertionError as e:
            bad += 1
            print("FAIL seed", seed, "ack_fast", ack_fast, e, flush=True)
    print("ack_fast", ack_fast, "seeds", lo, hi, "done", flush=True)
ops.set_tuning(switch_ack_fast=True)
print("failures:", bad)

# radix-path batches (> 2,048 packets: ack bits in the sort keys, chunk tiers)
import numpy as np  # noqa: E402
orc = t.orc
bad2 = 0
for ack_fast in (True, False):
    ops.set_tuning(switch_ack_fast=ack_fast)
    for seed in range(int(os.environ.get("BIG", 60))):
        rng = np.random.default_rng(50_000 + seed)
        V = int(rng.choice([4, 8, 32, 64, 128, 256, 33]))
        num_slots = int(rng.choice([64, 1000, 16384, 1 << 17]))
        W = int(rng.integers(1, 9))
        used = int(rng.integers(2100 // W + 1, 6000 // W + 2))
        layout = rng.choice(["padded", "tight", "wide"])
        stride = {"padded": ops.nga_stride(V), "tight": 15 + 4 * V, "wide": ops.nga_stride(V) + 32}[layout]
        wd = bool(rng.integers(0, 2))
        sw_dev = ops.Switch(V, num_slots=num_slots, switch_id=1, device=t.DEV, write_dropped=wd)
        sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
        try:
            for rnd in range(3):
                stream = t.make_stream(rng, V, used, W, num_slots, collide=float(rng.uniform(0, 0.2)),
                                       ack=float(rng.uniform(0, 0.6)), other=float(rng.uniform(0, 0.2)),
                                       stride=stride)
                want_pk, want_act = sw_orc.run(stream, stride=stride)
                d = t.dev(stream)
                act = sw_dev.process(d)
                assert np.array_equal(t.host(act), want_act), ("act", rnd)
                got = t.host(d)
                if wd:
                    assert np.array_equal(got, want_pk), ("pk", rnd)
                else:
                    fwd = want_act != orc.ACT_DROP
                    assert np.array_equal(got[fwd], want_pk[fwd]), ("fwd", rnd)
            cnt, frag, regs = sw_orc.registers()
            assert np.array_equal(t.host(sw_dev.count), cnt)
            assert np.array_equal(t.host(sw_dev.frag).view(np.uint32), frag)
            assert np.array_equal(t.host(sw_dev.regs).view(np.uint32), regs)
        except AssertionError as e:
            bad2 += 1
            print("BIG FAIL seed", seed, "ack_fast", ack_fast, V, num_slots, W, used, layout, e, flush=True)
    print("big ack_fast", ack_fast, "done", flush=True)
ops.set_tuning(switch_ack_fast=True)
print("big failures:", bad2)
