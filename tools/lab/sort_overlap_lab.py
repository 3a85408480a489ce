"""Lab: the packet path's steady-state step with the switch's slot sort taken out of the
critical path.  The sort reads only descriptors, and descriptors follow from the header
fields, so the sort can be queued before the worker packs: (a) one call per step as in
bench.py (packs write the descriptors, then ina_switch with the PS step, INA_SWITCH_ALL); (b)
the same stream, sort first (ina_nga_make_descriptors + ack descriptors + ina_switch
INA_SWITCH_SORT, then the packs, then ina_switch INA_SWITCH_RUN with the PS step); (c) as (b)
with the sort on a second stream
beside the packs.  Alternated; every variant must leave the same update and actions.
Config-3 sizes (8 x 26,214,400 fp32, V = 256, 2^17 slots)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
W, n, V, k, slots = 8, 26214400, 256, 16, 1 << 17
npk = n // V
g = torch.Generator(device=dev)
g.manual_seed(6000)
xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
glob = torch.randn(n, device=dev, generator=g) * 1e-2
upd = torch.empty_like(glob)
stride = ops.nga_stride(V)
big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=dev)
ack_rows, rows_w = big[:npk], big[npk:].view(W, npk, stride)
desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
desc_ack, desc_w = desc[:npk], desc[npk:].view(W, npk)
outs, descs = list(rows_w.unbind(0)), list(desc_w.unbind(0))
acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
ws = 1.0 / (W + 1)
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
bm = [w + 1 for w in range(W)]


def step_a():
    ops.quantize_pack_nga_multi(xs, k, V, bm, W, 1, 1, base=glob, num_slots=slots, outs=outs, descs=descs)
    ops.nga_descriptors(ack_rows, out=desc_ack)
    sw.process_apply(big, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False,
                     actions=acts, desc=desc)


def _sort():
    ops.make_descriptors(npk, W, W, 1, 1, num_slots=slots, outs=descs)
    ops.nga_descriptors(ack_rows, out=desc_ack)
    sw.sort(big, desc, actions=acts)


def step_b():
    _sort()
    ops.quantize_pack_nga_multi(xs, k, V, bm, W, 1, 1, base=glob, num_slots=slots, outs=outs)
    sw.run_apply(big, acts, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False)


def step_c():
    side.wait_stream(main)
    with torch.cuda.stream(side):
        _sort()
    ops.quantize_pack_nga_multi(xs, k, V, bm, W, 1, 1, base=glob, num_slots=slots, outs=outs)
    main.wait_stream(side)
    sw.run_apply(big, acts, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False)


def step_d():
    # only the ack rows' descriptor gather beside the packs (a small kernel that fits in the
    # VGPRs the pack kernel leaves free), the sort + run after both
    side.wait_stream(main)
    with torch.cuda.stream(side):
        ops.nga_descriptors(ack_rows, out=desc_ack)
    ops.quantize_pack_nga_multi(xs, k, V, bm, W, 1, 1, base=glob, num_slots=slots, outs=outs, descs=descs)
    main.wait_stream(side)
    sw.process_apply(big, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False,
                     actions=acts, desc=desc)


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(reps):
        fn()
    e1.record(main)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


ref = None
for nm, fn in (("a", step_a), ("b", step_b), ("c", step_c), ("d", step_d)):
    fn()
    fn()
    torch.cuda.synchronize()
    got = (upd.clone(), acts.clone())
    if ref is None:
        ref = got
    print(f"{nm}: update and actions equal to (a): {bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))}")
for r in range(4):
    ta, tb, tc, td = timed(step_a), timed(step_b), timed(step_c), timed(step_d)
    print(f"round {r}: (a) one call {ta:7.1f} us   (b) sort first, one stream {tb:7.1f} us   "
          f"(c) sort on a second stream {tc:7.1f} us   (d) ack descriptors beside the packs {td:7.1f} us")
