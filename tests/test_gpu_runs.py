"""GPU parity of the switch's dense-run path (csrc/ina_switch.hip, kRunsMax): a batch made of
at most 64 runs of consecutive slots -- worker-major arrival, the PS's acks in front --
skips the slot sort and runs each slot's segment from a table of the runs.  Slots are
independent and keep arrival order (ngaa.p4:87-168, 120-196), so every result must equal
the oracle's P4 restatement packet for packet: actions, rewritten packets and the switch
registers after every batch.  65 runs, gapped runs and shuffled batches take the sort.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
POOL = 1 << 17


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd import ops  # noqa: F401  (fails loudly if libina.so is missing)


def ops():
    from ina_amd import ops as o
    return o


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def runs_batch(rng, V, specs, W, stride, num_slots=POOL, collide=0.02, degree_mix=0.02):
    """Packets for `specs` in arrival order: (seq0, length, kind), kind = worker index w
    (bitmap w + 1), "ack" (PS acks, flag 0x40) or "foreign" (switch id 2).  Each spec is one
    pack: packet p has frag_id = seq0 + p and index = (seq0 + p) % num_slots, so a spec is
    one dense run unless its slots wrap the pool.  A few packets get another frag id
    (collisions) or another degree."""
    parts = []
    for seq0, ln, kind in specs:
        vals = rng.integers(-2**31, 2**31, size=ln * V, dtype=np.int64).astype(np.int32)
        if kind == "ack":
            p = orc.pack_nga(vals, V, 0, W, 1, seq0, flags=orc.FLAG_ACK, num_slots=num_slots, stride=stride)
        elif kind == "foreign":
            p = orc.pack_nga(vals, V, 1, W, 2, seq0, num_slots=num_slots, stride=stride)
        else:
            p = orc.pack_nga(vals, V, int(kind) + 1, W, 1, seq0, num_slots=num_slots, stride=stride)
        parts.append(p)
    pk = np.concatenate(parts)
    n = len(pk)
    for i in np.flatnonzero(rng.random(n) < collide):
        f = int.from_bytes(pk[i, 11:15].tobytes(), "big") + 1
        pk[i, 11:15] = np.frombuffer((f & 0xFFFFFFFF).to_bytes(4, "big"), np.uint8)
    for i in np.flatnonzero(rng.random(n) < degree_mix):
        pk[i, 4] = int(rng.choice([1, 2]))
    return pk


def check_batches(o, V, batches, want_path, use_desc=True, write_dropped=True, num_slots=POOL,
                  regs_each=True):
    """Every batch through a fresh device switch and the oracle (state carried across the
    batches): bit-exact actions, packets and registers (after every batch, or only after the
    last with regs_each=False), and the slot-sort path taken."""
    stride = batches[0].shape[1]
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for i, stream in enumerate(batches):
        want_pk, want_act = sw_orc.run(stream, stride=stride)
        d = dev(stream)
        act = sw_dev.process(d, desc=o.nga_descriptors(d) if use_desc else None)
        assert np.array_equal(host(act), want_act), i
        got = host(d)
        if write_dropped:
            assert np.array_equal(got, want_pk), i
        else:
            fwd = want_act != orc.ACT_DROP
            assert np.array_equal(got[fwd], want_pk[fwd]), i
        if want_path is not None:
            # a tuple: any of these paths (V <= 32 batches the near-sorted path may take instead
            # of the sort -- small batches, whose windows stay within the scan budget)
            want = want_path if isinstance(want_path, tuple) else (want_path,)
            assert sw_dev.batch_path(len(stream)) in want, i
        if not regs_each and i < len(batches) - 1:
            continue
        cnt, frag, regs = sw_orc.registers()
        assert np.array_equal(host(sw_dev.count), cnt), i
        assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag), i
        assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs), i


def worker_major(W, per, seq0=1, acks=False):
    specs = [(seq0, per, "ack")] if acks else []
    return specs + [(seq0, per, w) for w in range(W)]


@pytest.mark.parametrize("V", [32, 256])
@pytest.mark.parametrize("R", [1, 2, 9, 64, 65])
def test_dense_runs_vs_oracle(R, V):
    """R worker runs over the same slots (R = 9: 8 workers behind an ack run).  R <= 64 takes
    the run table (R = 1 is already in slot order), 65 runs take the bucket sort."""
    o = ops()
    rng = np.random.default_rng(100 * R + V)
    stride = o.nga_stride(V)
    per = max(3000 // R + 1, 40)
    specs = worker_major(8, per, acks=True) if R == 9 else [(5, per, w) for w in range(R)]
    batches = [runs_batch(rng, V, specs, min(R, 255), stride) for _ in range(3)]
    assert len(batches[0]) > 2048
    path = "in_order" if R == 1 else "runs" if R <= 64 else (("sorted", "local") if V <= 32 else "sorted")
    check_batches(o, V, batches, path)


@pytest.mark.parametrize("rounds", [0, 16])
@pytest.mark.parametrize("at", ["in_round", "round_edge", "wave_edge", "chunk_edge", "last"])
def test_run_breaks_at_sort_edges(at, rounds):
    """Two runs whose boundary (a descent) falls inside a 64-packet round, on a round, wave
    (4 rounds) or chunk (4,096 packets) edge of the chunk pass, or at the last packet: the
    break is found by the DPP predecessor, the previous round's lane 63 or the loaded
    predecessor of the wave -- and recorded in the right chunk."""
    o = ops()
    rng = np.random.default_rng(7 + len(at) + rounds)
    V = 32
    n = 9000
    cut = {"in_round": 4096 + 70, "round_edge": 4096 + 128, "wave_edge": 4096 + 256,
           "chunk_edge": 4096, "last": n - 1}[at]
    specs = [(1000, cut, 0), (1000, n - cut, 1)]
    o.set_tuning(switch_sort_rounds=rounds)
    try:
        batches = [runs_batch(rng, V, specs, 2, o.nga_stride(V)) for _ in range(2)]
        check_batches(o, V, batches, "runs")
    finally:
        o.set_tuning(switch_sort_rounds=0)


@pytest.mark.parametrize("case", ["acks_in_front", "lone_acks", "acks_behind", "foreign_mid_run",
                                  "pool_wrap", "few_gaps", "many_gaps", "shuffled", "ack_fast_off",
                                  "generic_kernel"])
def test_run_batches_vs_oracle(case):
    """Structured batches around the run table: acks leading a segment (read-free) and alone
    in it (frag cleared only), acks behind the workers (the state machine reads them),
    foreign packets in the middle of a run (their own runs, skipped), a pool wrap inside the
    runs (a run breaks at slot 0), a few lost packets (more, shorter runs), many lost packets
    and a shuffled batch (> 64 breaks: the bucket sort), keys without the ack bit (tuning
    key 11 off: every ack is read), and V = 33 (the generic LDS-staged run kernel, which
    reads the bucket sort's arrays, so its batches are sorted)."""
    o = ops()
    rng = np.random.default_rng(len(case) * 31)
    V, W, per = (33 if case == "generic_kernel" else 64), 8, 500
    stride = o.nga_stride(V)
    path = "runs"
    specs = worker_major(W, per, seq0=10, acks=True)
    if case == "lone_acks":            # acks for 0..599, workers for 300..799
        specs = [(10, 600, "ack")] + [(310, per, w) for w in range(W)]
    elif case == "acks_behind":
        specs = worker_major(W, per, seq0=10) + [(10, per, "ack")]
    elif case == "pool_wrap":
        specs = worker_major(W, per, seq0=POOL - 200, acks=True)
    batches = []
    for _ in range(2):
        b = runs_batch(rng, V, specs, W, stride)
        if case == "foreign_mid_run":   # 3 foreign packets inside worker 3's run
            f = runs_batch(rng, V, [(77, 3, "foreign")], W, stride, collide=0)
            at = per * 4 + per // 2
            b = np.concatenate([b[:at], f, b[at:]])
        elif case == "few_gaps":        # 5 packets lost: 5 more runs
            b = np.delete(b, rng.choice(len(b), 5, replace=False), axis=0)
        elif case == "many_gaps":       # every 7th packet lost: > 64 breaks
            b = np.delete(b, np.arange(3, len(b), 7), axis=0)
            path = "sorted"
        elif case == "shuffled":
            b = b[rng.permutation(len(b))]
            path = "sorted"
        batches.append(b)
    if case == "generic_kernel":
        path = "sorted"
    if case == "ack_fast_off":
        o.set_tuning(switch_ack_fast=False)
    try:
        check_batches(o, V, batches, path)
    finally:
        o.set_tuning(switch_ack_fast=True)


def test_runs_tuning_off_takes_the_sort():
    """ina_set_tuning key 18 = 0: the same worker-major batch through the bucket sort --
    identical results."""
    o = ops()
    rng = np.random.default_rng(3)
    V = 256
    batches = [runs_batch(rng, V, worker_major(8, 400, acks=True), 8, o.nga_stride(V)) for _ in range(2)]
    o.set_tuning(switch_runs=False)
    try:
        check_batches(o, V, batches, "sorted")
    finally:
        o.set_tuning(switch_runs=True)
    check_batches(o, V, batches, "runs", use_desc=False, write_dropped=False)


def test_digit_passes_report_sorted():
    """Tuning key 12 = 3 (the LSD digit passes for every batch): a worker-major batch, which
    the default would run from its run table, is sorted -- same results, and the diagnostic
    says so."""
    o = ops()
    rng = np.random.default_rng(12)
    V = 64
    batches = [runs_batch(rng, V, worker_major(8, 300, acks=True), 8, o.nga_stride(V)) for _ in range(2)]
    o.set_tuning(switch_sort=3)
    try:
        check_batches(o, V, batches, "sorted")
    finally:
        o.set_tuning(switch_sort=0)
    check_batches(o, V, batches, "runs")


@pytest.mark.parametrize("pre_all", [False, True])
@pytest.mark.parametrize("case", ["runs", "in_order", "sorted", "acks_behind"])
def test_first_pass_whole_or_split(case, pre_all):
    """ina_set_tuning key 19: the slot sort's first pass whole (keys of <= 18 bits, 0) or split
    into detection + one-block decision + digits (1, the default) -- the same results on every
    path (the run table, in slot order, the bucket sort), with and without descriptors."""
    o = ops()
    rng = np.random.default_rng(19 + len(case) + int(pre_all))
    V, W, per = 64, 8, 600
    stride = o.nga_stride(V)
    specs = worker_major(W, per, seq0=3, acks=case != "acks_behind")
    if case == "acks_behind":
        specs = worker_major(W, per, seq0=3) + [(3, per, "ack")]
    batches = []
    for _ in range(2):
        b = runs_batch(rng, V, specs, W, stride)
        if case == "in_order":          # the workers' packets interleaved, slot by slot
            b = b[np.argsort(np.arange(len(b)) % per, kind="stable")]
        elif case == "sorted":
            b = b[rng.permutation(len(b))]
        batches.append(b)
    path = {"runs": "runs", "in_order": None, "sorted": "sorted", "acks_behind": "runs"}[case]
    o.set_tuning(switch_pre_all=pre_all)
    try:
        check_batches(o, V, batches, path)
        check_batches(o, V, batches, path, use_desc=False)
    finally:
        o.set_tuning(switch_pre_all=True)


@pytest.mark.parametrize("V,W,per", [(256, 8, 700), (32, 4, 3000)])
def test_runs_fused_ps_and_two_phase_equal_sorted(V, W, per):
    """The packet path's steady state through the run table -- the fused PS apply (one call
    and two phases: sort, then run), the ack rows' descriptors written by the run kernel
    (ack_desc) and used as the next step's -- equals the same steps with the run table off
    (bucket sort, descriptors gathered from the ack rows): actions, PS update bit for bit,
    ack rows, registers; every ack row's written descriptor equals its header bytes."""
    o = ops()
    rng = np.random.default_rng(V + W)
    n = V * per - 3
    npk = -(-n // V)
    stride = o.nga_stride(V)
    slots = 1 << 13
    xs = [dev((rng.standard_normal(n) * 1e-2).astype(np.float32)) for _ in range(W)]
    glob0 = rng.standard_normal(n).astype(np.float32) * 1e-2
    res = {}
    try:
        for mode in ("sorted", "runs", "runs_two_phase"):
            o.set_tuning(switch_runs=mode != "sorted")
            glob = dev(glob0.copy())
            upd = torch.empty_like(glob)
            big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=DEV)
            acks, rows = big[:npk], big[npk:]
            desc = torch.zeros((W + 1) * npk, dtype=torch.int64, device=DEV)
            acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=DEV)
            wrows = torch.empty((W, npk, stride), dtype=torch.uint8, device=DEV)
            wdesc = torch.empty((W, npk), dtype=torch.int64, device=DEV)
            sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
            steps = []
            for step in range(3):
                o.quantize_pack_nga_multi(xs, 16, V, list(range(1, W + 1)), W, 1, 1, base=glob,
                                          num_slots=slots, outs=list(wrows.unbind(0)),
                                          descs=list(wdesc.unbind(0)))
                rows.view(W * npk, stride)[:] = wrows.view(W * npk, stride)
                if mode == "sorted" or step == 0:
                    o.nga_descriptors(acks, out=desc[:npk])
                else:                            # written by the previous step's run kernel
                    desc[:npk] = adesc
                desc[npk:] = wdesc.reshape(-1)
                adesc = torch.zeros(npk, dtype=torch.int64, device=DEV)
                if mode == "runs_two_phase":
                    sw.sort(big, desc, actions=acts)
                    sw.run_apply(big, acts, 1, glob, 16, 1.0 / (W + 1), out=upd, acks=acks,
                                 keep_forwarded=False, ack_desc=adesc)
                else:
                    sw.process_apply(big, 1, glob, 16, 1.0 / (W + 1), out=upd, acks=acks,
                                     keep_forwarded=False, actions=acts, desc=desc,
                                     ack_desc=None if mode == "sorted" else adesc)
                if mode != "sorted":             # the ack rows' descriptors, beside the rows
                    assert torch.equal(adesc, o.nga_descriptors(acks)), (mode, step)
                if step:
                    want = "sorted" if mode == "sorted" else "runs"
                    assert sw.batch_path((W + 1) * npk) == want, (mode, step)
                steps.append((host(acts).copy(), host(upd).view(np.uint32).copy(), host(acks).copy()))
                glob.copy_(upd)
            res[mode] = (steps, host(sw.count), host(sw.frag), host(sw.regs))
    finally:
        o.set_tuning(switch_runs=True)
    s0, c0, f0, r0 = res["sorted"]
    for mode in ("runs", "runs_two_phase"):
        s1, c1, f1, r1 = res[mode]
        for (a0, u0, k0), (a1, u1, k1) in zip(s0, s1):
            assert np.array_equal(a0, a1), mode
            assert np.array_equal(u0, u1), mode
            assert np.array_equal(k0, k1), mode
        assert np.array_equal(c0, c1) and np.array_equal(f0, f1) and np.array_equal(r0, r1), mode
    assert int((s0[2][0] == orc.ACT_FWD_AGG).sum()) == npk
    assert bool((s0[2][0][:npk] == orc.ACT_FWD_ACK).all())


def test_two_phase_orders_itself_across_streams():
    """sort() on a side stream with no wait_stream by the caller, then run() on the main
    stream, step after step over the same scratch: the switch's own events order every call
    after the previous one (a side-stream sort never overwrites the key / id arrays or the
    run table a pending run still reads).  Equal to one-call process() step by step."""
    o = ops()
    rng = np.random.default_rng(11)
    V, W, per = 256, 8, 600
    stride = o.nga_stride(V)
    batches = [runs_batch(rng, V, worker_major(W, per, acks=True), W, stride) for _ in range(4)]
    batches.append(batches[0][rng.permutation(len(batches[0]))])          # and a sorted one
    res = {}
    side = torch.cuda.Stream(DEV)
    for two in (False, True):
        sw = o.Switch(V, num_slots=POOL, switch_id=1, device=DEV, write_dropped=True)
        got = []
        for b in batches:
            d = dev(b)
            desc = o.nga_descriptors(d)
            torch.cuda.synchronize()
            if two:
                acts = torch.empty(len(b), dtype=torch.uint8, device=DEV)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(2_000_000)          # the sort is queued late on purpose
                    sw.sort(d, desc, actions=acts)
                sw.run(d, acts)
            else:
                acts = sw.process(d, desc=desc)
            got.append((host(acts).copy(), host(d).copy()))
        res[two] = (got, host(sw.count), host(sw.frag), host(sw.regs))
    (g0, c0, f0, r0), (g1, c1, f1, r1) = res[False], res[True]
    for (a0, p0), (a1, p1) in zip(g0, g1):
        assert np.array_equal(a0, a1) and np.array_equal(p0, p1)
    assert np.array_equal(c0, c1) and np.array_equal(f0, f1) and np.array_equal(r0, r1)


@pytest.mark.parametrize("bad", ["seq0", "num_slots", "count"])
def test_two_phase_descriptor_mismatch_is_caught(bad):
    """Descriptors made from header parameters that disagree with the packed headers would
    aggregate into the wrong slots without an error; check_sorted_desc() compares them with
    the headers' bytes 4..11 between sort() and run() and raises."""
    o = ops()
    V, W, npk = 32, 4, 900
    slots = 1 << 13
    stride = o.nga_stride(V)
    rows = torch.empty((W, npk, stride), dtype=torch.uint8, device=DEV)
    for w in range(W):
        o.pack_nga(dev(np.arange(npk * V, dtype=np.int32)), V, w + 1, W, 1, 5, num_slots=slots, out=rows[w])
    big = rows.view(W * npk, stride)
    seq0 = 6 if bad == "seq0" else 5
    ns = 500 if bad == "num_slots" else slots          # indices wrap at 500 instead of 8192
    count = W + 1 if bad == "count" else W
    descs = torch.empty((W, npk), dtype=torch.int64, device=DEV)
    o.make_descriptors(npk, W, count, 1, seq0, num_slots=ns, outs=list(descs.unbind(0)), device=DEV)
    sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
    sw.sort(big, descs.view(-1))
    with pytest.raises(ValueError, match="disagree"):
        sw.check_sorted_desc(big)
    good = torch.empty_like(descs)
    o.make_descriptors(npk, W, W, 1, 5, num_slots=slots, outs=list(good.unbind(0)), device=DEV)
    acts = sw.sort(big, good.view(-1))
    sw.check_sorted_desc(big)                           # the matching ones pass
    sw.run(big, acts)
    assert int((host(acts) == orc.ACT_FWD_AGG).sum()) == npk


# pools of 2^18 .. 2^21 slots: keys of 19-22 bits, the 2,048-bin chunk + bucket sort (digits of
# 10-11 bits) instead of three LSD digit passes; its in-order and run-table paths as well
WIDE_POOLS = [1 << 18, (1 << 19) + 3, 1 << 20, (1 << 21) - 1, 1 << 21]


@pytest.mark.parametrize("order", ["shuffled", "worker_major", "round_robin", "skewed"])
@pytest.mark.parametrize("num_slots", WIDE_POOLS)
def test_wide_key_pools_vs_oracle(num_slots, order):
    """Bit-exact against the P4 restatement with state carried across batches, and the same
    batches through the LSD digit passes (tuning key 12 = 3) -- worker-major batches wrap the
    pool (a run breaks at slot 0), "skewed" puts every packet in three buckets (multi-tile
    buckets of the 2,048-bin sort)."""
    o = ops()
    rng = np.random.default_rng(num_slots % 1000 + len(order))
    V, W, per = 32, 8, 1200
    stride = o.nga_stride(V)
    seq0 = {"worker_major": num_slots - 500, "skewed": 1, "round_robin": 7}.get(order)
    if seq0 is None:
        seq0 = int(rng.integers(0, num_slots))
    specs = [(seq0, per, w) for w in range(W)]
    batches = []
    for _ in range(2):
        b = runs_batch(rng, V, specs, W, stride, num_slots=num_slots)
        if order in ("shuffled", "skewed"):
            b = b[rng.permutation(len(b))]
        elif order == "round_robin":
            b = b.reshape(W, per, stride).transpose(1, 0, 2).reshape(W * per, stride).copy()
        batches.append(b)
    sorted_ = ("sorted", "local") if V <= 32 else "sorted"      # small batches: the lists' budget holds
    want = {"shuffled": sorted_, "skewed": sorted_, "worker_major": "runs", "round_robin": "in_order"}[order]
    check_batches(o, V, batches, want, num_slots=num_slots, regs_each=False)
    if order in ("shuffled", "skewed"):                      # the 2,048-bin sort itself
        o.set_tuning(switch_local=False)
        try:
            check_batches(o, V, batches, "sorted", num_slots=num_slots, regs_each=False)
        finally:
            o.set_tuning(switch_local=True)
    o.set_tuning(switch_sort=3)
    try:
        check_batches(o, V, batches, None, num_slots=num_slots, regs_each=False)
    finally:
        o.set_tuning(switch_sort=0)


@pytest.mark.parametrize("acks", [False, True])
@pytest.mark.parametrize("num_slots", [1 << 18, 1 << 20, (1 << 21) - 1])
def test_wide_key_split_sorted_vs_oracle(num_slots, acks):
    """Shuffled NGA-32 batches in split rows over pools of 19-22-bit keys -- the 2,048-bin sort
    and the narrow sorted run over 16-byte header rows + 128-byte payload rows, the near-sorted
    path off.  Against the P4 restatement with 2 % collisions, 2 % other degrees and PS acks:
    actions, the header rows (collision flags), the payload rows (dropped packets rewritten
    too) and the registers, state carried across batches."""
    o = ops()
    rng = np.random.default_rng(num_slots % 997 + acks)
    V, W, per = 32, 8, 1500
    stride = o.nga_stride(V)
    seq0 = int(rng.integers(0, num_slots))
    specs = ([(seq0, per, "ack")] if acks else []) + [(seq0, per, w) for w in range(W)]
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=True)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    o.set_tuning(switch_local=False)                  # the sort itself (small batches fit the lists)
    try:
        for i in range(2):
            b = runs_batch(rng, V, specs, W, stride, num_slots=num_slots)
            b = b[rng.permutation(len(b))]
            want_pk, want_act = sw_orc.run(b, stride=stride)
            hdr = np.zeros((len(b), 16), np.uint8)
            hdr[:, :15] = b[:, :15]
            hd, pd = dev(hdr), dev(np.ascontiguousarray(b[:, 15:15 + 4 * V]))
            act = sw_dev.process_split(hd, pd, desc=o.nga_descriptors(dev(b)))
            assert sw_dev.batch_path(len(b)) == "sorted", i
            assert np.array_equal(host(act), want_act), i
            assert np.array_equal(host(hd)[:, :15], want_pk[:, :15]), i
            assert np.array_equal(host(pd), want_pk[:, 15:15 + 4 * V]), i
            assert (want_act == orc.ACT_FWD_COLLISION).any(), i
    finally:
        o.set_tuning(switch_local=True)
    cnt, frag, regs = sw_orc.registers()
    assert np.array_equal(host(sw_dev.count), cnt)
    assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
    assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


@pytest.mark.parametrize("tile", [0, 8])
def test_wide_key_multi_tile_buckets(tile):
    """2^20-slot pool, 24,000 packets in slots 0..2,999 (three 1,024-slot buckets of 8,000
    packets: several 4,096- or 8,192-item tiles each, the counting sweep first), shuffled."""
    o = ops()
    rng = np.random.default_rng(tile + 5)
    V, W, per, ns = 32, 8, 3000, 1 << 20
    b = runs_batch(rng, V, [(0, per, w) for w in range(W)], W, o.nga_stride(V), num_slots=ns)
    b = b[rng.permutation(len(b))]
    o.set_tuning(switch_bucket_tile=tile)
    try:
        check_batches(o, V, [b, b.copy()], "sorted", num_slots=ns, regs_each=False)
    finally:
        o.set_tuning(switch_bucket_tile=0)


@pytest.mark.parametrize("order", ["worker_major", "shuffled"])
def test_nga32_config3_full_size(order):
    """The P4 program's own format (NGA-32, headers.p4:40-73) at config-3 size: 8 workers x
    819,200 packets through a 2^20-slot pool (21-bit keys), worker-major (the run table) and
    shuffled (the 2,048-bin sort).  Size-independent checks: every slot completes exactly
    once, on the last packet of its slot; a strided sample of slots (every 997th + the last)
    carries the wrapping int32 sum of the workers' values in its completing packet and in
    the slot's registers."""
    o = ops()
    W, n, V, ns = 8, 26_214_400, 32, 1 << 20
    npk = n // V
    g = torch.Generator(device=DEV).manual_seed(31)
    samp = np.unique(np.concatenate([np.arange(0, npk, 997), [npk - 1]]))
    vidx = torch.from_numpy((samp[:, None] * V + np.arange(V)).ravel()).to(DEV)
    want = torch.zeros(vidx.numel(), dtype=torch.int64, device=DEV)
    rows, descs = [], []
    for w in range(W):
        b = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device=DEV, generator=g)
        want += b[vidx].to(torch.int64)
        p, d = o.pack_nga(b, V, w + 1, W, 1, 1, num_slots=ns, desc=True)
        rows.append(p)
        descs.append(d)
        del b
    want = ((want + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32).view(-1, V)
    stream, desc = torch.cat(rows), torch.cat(descs)
    del rows, descs
    perm = None if order == "worker_major" else torch.randperm(W * npk, device=DEV, generator=g)
    if perm is not None:
        stream, desc = stream[perm], desc[perm]
    sw = o.Switch(V, num_slots=ns, switch_id=1, device=DEV)
    act = sw.process(stream, desc=desc)
    assert sw.batch_path(W * npk) == ("runs" if perm is None else "sorted")
    assert int((act == orc.ACT_FWD_AGG).sum()) == npk
    assert int((act == orc.ACT_DROP).sum()) == (W - 1) * npk
    pos = torch.arange(W * npk, device=DEV) if perm is None else torch.argsort(perm)
    ts = torch.from_numpy(samp).to(DEV)
    cand = torch.stack([pos[w * npk + ts] for w in range(W)])
    fwd = act[cand] == orc.ACT_FWD_AGG
    assert bool((fwd.sum(0) == 1).all())
    last = cand.max(0).values                              # completes on its last arrival
    assert torch.equal(cand.gather(0, fwd.to(torch.int64).argmax(0, keepdim=True)).reshape(-1), last)
    pay = stream[last, 15:15 + 4 * V].contiguous().cpu().numpy().view(">u4").astype(np.uint32)
    assert np.array_equal(pay.reshape(-1, V), want.cpu().numpy().view(np.uint32))
    slot = (ts + 1) % ns                                   # packet p of a worker: slot (seq0 + p) % pool
    assert torch.equal(sw.regs[slot], want)
    assert int(sw.count.max()) == 0


@pytest.mark.parametrize("num_slots", [1 << 16, 1 << 20])
@pytest.mark.parametrize("order", ["shuffled", "worker_major", "round_robin"])
def test_big_batch_chunks_vs_digit_passes(order, num_slots):
    """More than 2 Mi packets through the chunk + bucket sort take 8,192-packet chunks
    (INA_RS_BIG_ITEMS).  Two batches of 8 x 300,000 NGA-4 packets (1 % frag-id collisions;
    at 2^16 slots every worker wraps the pool four times), state carried: actions, rewritten
    rows and registers byte for byte against the same batches through the LSD digit passes
    (tuning key 12 = 3, 4,096-packet chunks), in packed and in split rows."""
    o = ops()
    W, per, V = 8, 300_000, 4
    g = torch.Generator(device=DEV).manual_seed(num_slots % 97 + len(order))
    batches = []
    for bi in range(2):
        rows, descs = [], []
        for w in range(W):
            b = torch.randint(-(1 << 31), (1 << 31) - 1, (per * V,), dtype=torch.int32, device=DEV, generator=g)
            p, d = o.pack_nga(b, V, w + 1, W, 1, 1 + bi * per, num_slots=num_slots, desc=True)
            rows.append(p)
            descs.append(d)
        st, de = torch.cat(rows), torch.cat(descs)
        hit = torch.rand(st.shape[0], device=DEV, generator=g) < 0.01
        st[hit, 14] ^= 1                                   # frag id's low byte: not in the descriptor
        if order == "shuffled":
            perm = torch.randperm(st.shape[0], device=DEV, generator=g)
        elif order == "round_robin":
            perm = torch.arange(st.shape[0], device=DEV).view(W, per).t().reshape(-1)
        else:
            perm = None
        if perm is not None:
            st, de = st[perm], de[perm]
        batches.append((st, de))
    out = {}
    for mode in (0, 3):
        o.set_tuning(switch_sort=mode)
        try:
            sw, sws = (o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV) for _ in range(2))
            res, paths = [], []
            for st, de in batches:
                pk = st.clone()
                h = torch.zeros((st.shape[0], 16), dtype=torch.uint8, device=DEV)
                h[:, :15] = st[:, :15]
                pay = st[:, 15:15 + 4 * V].contiguous()
                res += [sw.process(pk, desc=de), pk]
                paths.append(sw.batch_path(st.shape[0]))
                res += [sws.process_split(h, pay, desc=de), h, pay]
            res += [sw.regs.clone(), sw.count.clone(), sw.frag.clone(), sws.regs.clone()]
            out[mode] = ([x.cpu() for x in res], paths)
            del sw, sws, res
        finally:
            o.set_tuning(switch_sort=0)
    for x, y in zip(out[0][0], out[3][0]):
        assert torch.equal(x, y)
    assert out[3][1] == ["sorted", "sorted"]
    if num_slots == 1 << 20:
        want = {"shuffled": "sorted", "worker_major": "runs", "round_robin": "in_order"}[order]
        assert out[0][1] == [want, want]
    n_fwd = int((out[0][0][0] == orc.ACT_FWD_AGG).sum())
    assert n_fwd > 0


def test_numpy_integer_seq0_broadcasts():
    """seq0 given as a numpy integer scalar is one seq0 for every worker (numbers.Integral),
    as a Python int is -- make_descriptors and the one-launch worker pack alike."""
    o = ops()
    a = o.make_descriptors(100, 3, 3, 1, np.int64(5), num_slots=1 << 13, device=DEV)
    b = o.make_descriptors(100, 3, 3, 1, 5, num_slots=1 << 13, device=DEV)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    xs = [torch.zeros(320, device=DEV) for _ in range(3)]
    p1 = o.quantize_pack_nga_multi(xs, 16, 32, [1, 2, 3], 3, 1, np.uint32(9))
    p2 = o.quantize_pack_nga_multi(xs, 16, 32, [1, 2, 3], 3, 1, 9)
    assert all(torch.equal(x, y) for x, y in zip(p1, p2))



def _check_split_vs_oracle(o, V, batches, want_paths, write_dropped, num_slots=POOL):
    """Split rows through a fresh device switch and the oracle (state carried): actions, the
    rewritten datagram bytes (all rows, or the forwarded ones without write_dropped) and the
    registers after every batch, and the path each batch took."""
    stride = batches[0].shape[1]
    sw = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    ref = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for i, stream in enumerate(batches):
        want_pk, want_act = ref.run(stream, stride=stride)
        d = dev(stream)
        desc = o.nga_descriptors(d)
        hdr = torch.zeros((d.shape[0], 16), dtype=torch.uint8, device=DEV)
        hdr[:, :15] = d[:, :15]
        pay = d[:, 15:15 + 4 * V].contiguous()
        act = sw.process_split(hdr, pay, desc=desc)
        d[:, :15] = hdr[:, :15]
        d[:, 15:15 + 4 * V] = pay
        assert np.array_equal(host(act), want_act), i
        got = host(d)
        rows = slice(None) if write_dropped else want_act != orc.ACT_DROP
        assert np.array_equal(got[rows], want_pk[rows]), i
        assert sw.batch_path(len(stream)) in want_paths, (i, sw.batch_path(len(stream)))
        cnt, frag, regs = ref.registers()
        assert np.array_equal(host(sw.count), cnt), i
        assert np.array_equal(host(sw.frag).view(np.uint32), frag), i
        assert np.array_equal(host(sw.regs).view(np.uint32), regs), i


@pytest.mark.parametrize("write_dropped", [False, True])
@pytest.mark.parametrize("order", ["worker_major", "round_robin", "jitter", "shuffled"])
@pytest.mark.parametrize("case", ["clean", "collide", "count_open", "ack_inside", "degree4", "small_V"])
def test_whole_segments_vs_oracle(case, order, write_dropped):
    """Round 6 (seg8_fast): split-row narrow batches whose slots hold exactly 8 packets of
    degree 8 take the whole-segment path in every run path -- the run table (worker-major), the
    in-order windows (round-robin), the near-sorted lists (jitter 64) and the sorted windows
    (shuffled).  Any other segment in a wave sends that wave back to the packet-by-packet walk:
    a frag-id collision, a slot whose count is not 0 when the batch arrives (its first 4 packets
    came in the previous batch), a PS ack among the 8, degree 4 (two completions per segment).
    V = 8 leaves 6 of a group's 8 lanes without payload.  Bit-exact against the P4 restatement
    with registers after every batch, with and without write_dropped."""
    o = ops()
    V = 8 if case == "small_V" else 32
    W, per = 8, 2000
    rng = np.random.default_rng(1000 * len(case) + 10 * len(order) + int(write_dropped))
    stride = o.nga_stride(V)
    collide = 0.01 if case == "collide" else 0.0

    def arrive(b, k):
        n = len(b)
        if order == "worker_major":
            return b
        rr = b.reshape(k, n // k, stride).transpose(1, 0, 2).reshape(n, stride)
        if order == "round_robin":
            return rr.copy()
        if order == "jitter":
            return rr[np.argsort(np.arange(n) + rng.integers(0, 64, n), kind="stable")].copy()
        return rr[rng.permutation(n)].copy()

    batches = []
    for bi in range(2):
        if case == "count_open" and bi == 0:
            specs = [(5, per // 2, w) for w in range(4)]           # half the slots: 4 of 8 packets
        else:
            specs = [(5, per, w) for w in range(W)]
        k = len(specs)
        b = runs_batch(rng, V, specs, W, stride, collide=collide, degree_mix=0.0)
        if case == "degree4":
            b[:, 4] = 4
        if case == "ack_inside":
            for i in rng.choice(len(b), 20, replace=False):    # (<= 48 run breaks: still a run table)
                b[i, 5] |= orc.FLAG_ACK                            # a PS ack among a slot's packets
        batches.append(arrive(b, k))
    want = {"worker_major": ("runs",), "round_robin": ("in_order",), "jitter": ("local",),
            "shuffled": ("sorted", "local")}[order]
    if case == "count_open" and order == "worker_major":
        want = ("runs",)
    _check_split_vs_oracle(o, V, batches, want, write_dropped)


@pytest.mark.parametrize("write_dropped", [False, True])
@pytest.mark.parametrize("case", ["base", "base_b", "row0_foreign", "index_high", "flags", "refrag",
                                  "wrap", "degree4"])
def test_plain_packets_vs_oracle(case, write_dropped):
    """Round 6 (kPlainBit): the digit pass of a shuffled narrow split-row batch marks each packet
    whose header fields follow from its slot -- flags 0, index == slot, count == C, frag id ==
    index + B, with B and C taken from header row 0 -- and the sorted run makes those fields
    instead of gathering the header row.  Cases: B = 0 and B = 3 x pool; row 0 another switch's
    packet with its own frag id (B and C from it: few packets plain); 10 % of the rows with index
    + pool (same slot, not plain); 5 % with the resend flag; a second batch whose frag ids are
    one pool further on (every plain packet collides with the slot's stored frag id: the
    collision rewrite writes the made header word); a pool of 2^10 slots that the batch wraps
    (B holds for one pass of the pool only); degree 4 (plain with C = 4: not whole segments).
    Bit-exact against the P4 restatement, registers after every batch."""
    o = ops()
    V, W, per = 32, 8, 2000
    num_slots = (1 << 10) if case == "wrap" else POOL
    rng = np.random.default_rng(7000 + 10 * len(case) + int(write_dropped))
    stride = o.nga_stride(V)
    seq0 = 3 * num_slots + 5 if case == "base_b" else 5
    batches = []
    for bi in range(2):
        s0 = seq0 + (num_slots if case == "refrag" and bi == 1 else 0)
        specs = [(s0, per, w) for w in range(W)]
        b = runs_batch(rng, V, specs, W, stride, num_slots=num_slots, collide=0.0, degree_mix=0.0)
        if case == "degree4":
            b[:, 4] = 4
        if case == "index_high":
            for i in np.flatnonzero(rng.random(len(b)) < 0.1):
                ix = int.from_bytes(b[i, 6:10].tobytes(), "big") + num_slots
                b[i, 6:10] = np.frombuffer(ix.to_bytes(4, "big"), np.uint8)
        if case == "flags":
            b[rng.random(len(b)) < 0.05, 5] |= orc.FLAG_RESEND
        b = b[rng.permutation(len(b))].copy()
        if case == "row0_foreign":
            f = runs_batch(rng, V, [(999999, 1, "foreign")], W, stride, num_slots=num_slots,
                           collide=0.0, degree_mix=0.0)
            b = np.concatenate([f, b])
        batches.append(b)
    o.set_tuning(switch_local=False)          # small shuffled batches may take the lists instead
    try:
        _check_split_vs_oracle(o, V, batches, ("sorted",), write_dropped, num_slots=num_slots)
    finally:
        o.set_tuning(switch_local=True)
