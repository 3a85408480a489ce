"""GPU parity of the switch's near-sorted path (csrc/ina_switch.hip, local_decide in the
detect pass, k_local_lists, lists_slots_narrow in k_switch_run2): W sequence-ordered senders (DataManager.py:116-134) interleaved with local
disorder -- round-robin arrival with every packet displaced by less than J positions -- are
neither in slot order nor a few dense runs, yet need no sort: each unit of slots is run from
per-slot lists built in LDS over the window of granules that can hold its packets.  Slots are
independent and keep arrival order (ngaa.p4:87-168, 120-196), so every result must equal the
oracle's P4 restatement packet for packet (actions, rewritten packets, registers after every
batch), and, at config-3 size, the sorted path's bytes.  Jitter wider than the path's scan
budget, shuffled batches and pool wraps take the sort; results are identical either way.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


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


def jitter_perm(rng, n, J):
    """Arrival order of n packets given in round-robin order: each moves by less than J
    positions (sort key = position + U[0, J), stable)."""
    if J <= 1:
        return np.arange(n)
    return np.argsort(np.arange(n) + rng.integers(0, J, n), kind="stable")


def rr_batch(rng, V, W, per, seq0, num_slots, stride, J, acks=False, collide=0.02, degree_mix=0.02,
             foreign=0.0):
    """W workers x `per` packets for slots seq0.., in round-robin arrival (slot s: worker 0..W-1)
    with jitter J; acks=True puts a PS ack per slot in front of each slot's packets (the steady
    state: step t's acks beside step t+1's packets).  A few packets get another frag id
    (collisions), another degree, or (foreign) another switch id."""
    rows = []
    if acks:
        vals = rng.integers(-2**31, 2**31, size=per * V, dtype=np.int64).astype(np.int32)
        rows.append(orc.pack_nga(vals, V, 0, W, 1, seq0, flags=orc.FLAG_ACK, num_slots=num_slots, stride=stride))
    for w in range(W):
        vals = rng.integers(-2**31, 2**31, size=per * V, dtype=np.int64).astype(np.int32)
        rows.append(orc.pack_nga(vals, V, w + 1, W, 1, seq0, num_slots=num_slots, stride=stride))
    K = len(rows)
    rr = np.stack(rows, 1).reshape(K * per, stride)          # slot-major: slot s, then sender
    pk = rr[jitter_perm(rng, K * per, J)].copy()
    n = len(pk)
    for i in np.flatnonzero(rng.random(n) < collide):
        f = int.from_bytes(pk[i, 11:15].tobytes(), "big") + 1
        pk[i, 11:15] = np.frombuffer((f & 0xFFFFFFFF).to_bytes(4, "big"), np.uint8)
    for i in np.flatnonzero(rng.random(n) < degree_mix):
        pk[i, 4] = int(rng.choice([1, 2]))
    for i in np.flatnonzero(rng.random(n) < foreign):
        pk[i, 10] = 2
    return pk


def split_of(d, V):
    hdr = torch.zeros((d.shape[0], 16), dtype=torch.uint8, device=d.device)
    hdr[:, :15] = d[:, :15]
    return hdr, d[:, 15:15 + 4 * V].contiguous()


def check_vs_oracle(o, V, batches, num_slots, want_paths, split=False, write_dropped=True):
    stride = batches[0].shape[1]
    sw = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    ref = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for i, stream in enumerate(batches):
        want_pk, want_act = ref.run(stream, stride=stride)
        d = dev(stream)
        desc = o.nga_descriptors(d)
        if split:
            hdr, pay = split_of(d, V)
            act = sw.process_split(hdr, pay, desc=desc)
            d[:, :15] = hdr[:, :15]
            d[:, 15:15 + 4 * V] = pay
        else:
            act = sw.process(d, desc=desc)
        assert np.array_equal(host(act), want_act), i
        got = host(d)
        if write_dropped:
            assert np.array_equal(got, want_pk), i
        else:
            fwd = want_act != orc.ACT_DROP
            assert np.array_equal(got[fwd], want_pk[fwd]), i
        assert sw.batch_path(len(stream)) in want_paths, (i, sw.batch_path(len(stream)))
        cnt, frag, regs = ref.registers()
        assert np.array_equal(host(sw.count), cnt), i
        assert np.array_equal(host(sw.frag).view(np.uint32), frag), i
        assert np.array_equal(host(sw.regs).view(np.uint32), regs), i


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("num_slots", [1 << 17, 1 << 20])
@pytest.mark.parametrize("J", [8, 64, 700, 4096])
def test_jitter_vs_oracle(J, num_slots, split):
    """Round-robin W = 8 arrival with jitter J over 9,000 slots (72,000 packets, 64 KiB of
    keys: granules of 128 packets), three batches over the same slots (the registers carry),
    collisions and mixed degrees inside the jitter windows: the near-sorted path, bit-exact."""
    o = ops()
    V, W, per = 32, 8, 9000
    rng = np.random.default_rng(J + num_slots % 977 + 5 * split)
    stride = o.nga_stride(V)
    batches = [rr_batch(rng, V, W, per, 1 + 3 * b, num_slots, stride, J) for b in range(3)]
    # (at this size granules hold 128 packets: jitter 4096 exceeds the scan budget, the sort)
    paths = {"local"} if J < 4096 else {"local", "sorted"}
    check_vs_oracle(o, V, batches, num_slots, paths, split=split, write_dropped=not split)


@pytest.mark.parametrize("J", [64, 2000])
def test_jitter_acks_and_foreign(J):
    """The steady state's batch: a PS ack per slot in front of its 8 packets, jittered with
    them (an ack may land behind a packet of its slot: a collision then, as on the Tofino),
    and 0.5 % foreign packets (switch id 2: FWD_OTHER, outside every list)."""
    o = ops()
    V, W, per, num_slots = 32, 8, 6000, 1 << 20
    rng = np.random.default_rng(40 + J)
    stride = o.nga_stride(V)
    batches = [rr_batch(rng, V, W, per, 1, num_slots, stride, J, acks=True, foreign=0.005) for _ in range(3)]
    check_vs_oracle(o, V, batches, num_slots, {"local"} if J < 1000 else {"local", "sorted"})


@pytest.mark.parametrize("V", [4, 16, 32])
def test_jitter_small_V(V):
    """NGA-V with V < 32 (fewer value lanes per group): same lists, same per-packet code."""
    o = ops()
    rng = np.random.default_rng(V)
    stride = o.nga_stride(V)
    batches = [rr_batch(rng, V, 4, 5000, 9, 1 << 17, stride, 300) for _ in range(2)]
    check_vs_oracle(o, V, batches, 1 << 17, {"local"})


def test_unit_and_window_edges():
    """Unit and window edges: units of 4 granules whose windows reach far back (24 senders,
    jitter 3,000: a unit's packets come from many granules before its own), a slot with 600
    packets (one slot's list longer than a wave), and a pool of 1,000 slots (one-digit keys).
    These cases may exceed the scan budget, so either path is accepted; the path itself is
    asserted in test_multi_pass_lists and the jitter tests."""
    o = ops()
    V, stride = 32, o.nga_stride(32)
    rng = np.random.default_rng(3)
    # 24 senders, 2,048 slots: jitter 3,000 spreads a slot's packets over many granules
    a = [rr_batch(rng, V, 24, 2048, 1, 1 << 20, stride, 3000) for _ in range(2)]
    check_vs_oracle(o, V, a, 1 << 20, {"local", "sorted"})
    # one heavy slot: 600 packets of slot 77 spread through a jittered batch
    b = rr_batch(rng, V, 8, 4000, 1, 1 << 17, stride, 100)
    heavy = orc.pack_nga(rng.integers(-9, 9, 600 * V).astype(np.int32), V, 1, 255, 1, 77, num_slots=1 << 17,
                         stride=stride)
    heavy[:, 6:10] = np.frombuffer((77).to_bytes(4, "big"), np.uint8)     # same slot index
    heavy[:, 11:15] = np.frombuffer((77).to_bytes(4, "big"), np.uint8)    # same frag id
    pos = np.sort(rng.choice(len(b) + 600, 600, replace=False))
    mixed = np.empty((len(b) + 600, stride), np.uint8)
    mask = np.zeros(len(mixed), bool)
    mask[pos] = True
    mixed[mask] = heavy
    mixed[~mask] = b
    check_vs_oracle(o, V, [mixed], 1 << 17, {"local", "sorted"})
    c = [rr_batch(rng, V, 8, 1000, 1, 1000, stride, 40) for _ in range(2)]
    check_vs_oracle(o, V, c, 1000, {"local"})


@pytest.mark.parametrize("W,npk", [(2, 600_000), (1, 400_000)])
def test_multi_pass_lists(W, npk):
    """a unit whose slot range is wider than one LDS pass (kLlBins = 1,024 slots)
    builds its lists in several passes (k_local_lists' q loop: the area's count taken on the
    first pass only, the area advanced by each pass's packets).  600,000 packets take 4,096-packet
    chunks (granules of 512 packets, units of 2,048) and 400,000 take 2,048-packet chunks (units
    of 1,024): two senders, or one, then give units of 1,024 +- the jitter slots, so about half
    of them take two passes.  Jitter 64 keeps the scan within budget (one sender over 2,048-packet
    units would need three passes a unit and sort), so the near-sorted path is asserted, packet
    for packet against the oracle."""
    o = ops()
    V, per = 32, npk // W
    rng = np.random.default_rng(91 + W)
    stride = o.nga_stride(V)
    batches = [rr_batch(rng, V, W, per, 1 + 5 * b, 1 << 20, stride, 64, collide=0.001, degree_mix=0.001)
               for b in range(2)]
    check_vs_oracle(o, V, batches, 1 << 20, {"local"}, split=W == 2, write_dropped=W == 1)


@pytest.mark.parametrize("split", [False, True])
def test_late_decision_block(split):
    """Verdict r05 item 4: the digit pass's blocks wait for block 0's near-sorted verdict only
    for a bounded time (kLocPollTicks, 50 us), so no block's progress depends on when block 0 is
    dispatched.  Key 21 holds block 0 back 300 us: every other block's wait runs out and it
    sorts its chunk; block 0 then still chooses the near-sorted path, whose lists overwrite what
    those digits wrote.  The results must be the oracle's, packet for packet, and the path
    'local'; a sort-only / run pair and a whole call agree."""
    o = ops()
    V, W, per, num_slots = 32, 8, 40_000, 1 << 20
    rng = np.random.default_rng(123 + split)
    stride = o.nga_stride(V)
    batches = [rr_batch(rng, V, W, per, 1 + 3 * b, num_slots, stride, 64) for b in range(2)]
    o.set_tuning(switch_decide_delay_us=300)
    try:
        check_vs_oracle(o, V, batches, num_slots, {"local"}, split=split, write_dropped=not split)
    finally:
        o.set_tuning(switch_decide_delay_us=0)


def test_wide_disorder_takes_the_sort():
    """Jitter far past the scan budget (shuffled, and a pool wrap whose low slots arrive
    after the high ones) takes the bucket sort; the results are the oracle's either way."""
    o = ops()
    V, stride = 32, o.nga_stride(32)
    rng = np.random.default_rng(11)
    shuf = rr_batch(rng, V, 8, 5000, 1, 1 << 17, stride, 1 << 30)
    check_vs_oracle(o, V, [shuf], 1 << 17, {"sorted"})
    wrap = rr_batch(rng, V, 8, 5000, (1 << 17) - 2500, 1 << 17, stride, 64)
    check_vs_oracle(o, V, [wrap], 1 << 17, {"local", "sorted"})


@pytest.mark.parametrize("split", [False, True])
def test_local_ps_fused_equals_sorted(split):
    """process_apply with the PS fused, steady-state batch (acks in front of the 8 workers'
    packets, jitter 500): the near-sorted path's update, ack rows and ack descriptors equal
    the sorted path's (tuning key 20 off) bit for bit."""
    o = ops()
    V, W, per, num_slots = 32, 8, 7000, 1 << 20
    rng = np.random.default_rng(77 + split)
    stride = o.nga_stride(V)
    stream = rr_batch(rng, V, W, per, 1, num_slots, stride, 500, acks=True, collide=0, degree_mix=0)
    n = per * V - 5
    local = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(DEV)
    res = {}
    for mode in ("local", "sorted"):
        o.set_tuning(switch_local=mode == "local")
        try:
            sw = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV)
            d = dev(stream)
            desc = o.nga_descriptors(d)
            acks = torch.zeros((per, 16 if split else stride), dtype=torch.uint8, device=DEV)
            ad = torch.zeros(per, dtype=torch.int64, device=DEV)
            if split:
                hdr, pay = split_of(d, V)
                act, out = sw.process_apply_split(hdr, pay, 1, local, 16, 1 / 9, ack_hdr=acks, ack_desc=ad,
                                                  desc=desc)
                rows = (hdr, pay)
            else:
                act, out = sw.process_apply(d, 1, local, 16, 1 / 9, acks=acks, ack_desc=ad, desc=desc)
                rows = (d,)
            res[mode] = [host(x) for x in (act, out, acks, ad, sw.count, sw.frag, sw.regs, *rows)]
            res[mode + "_path"] = sw.batch_path(len(stream))
        finally:
            o.set_tuning(switch_local=True)
    assert res["local_path"] == "local" and res["sorted_path"] == "sorted"
    assert int((res["local"][0] == orc.ACT_FWD_AGG).sum()) == per
    for a, b in zip(res["local"], res["sorted"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("J", [64, 4096])
def test_config3_v32_local_equals_sorted(J):
    """Config 3 at the P4's NGA-32: 8 x 819,200 packets, 2^20-slot pool, round-robin with
    jitter J, split rows: the near-sorted path's actions, payload rows and registers equal the
    sorted path's (tuning key 20 off) byte for byte, and every slot completes once."""
    o = ops()
    V, W, n, slots = 32, 8, 26_214_400, 1 << 20
    npk = n // V
    g = torch.Generator(device=DEV).manual_seed(5 + J)
    hdrs, pays, descs = [], [], []
    for w in range(W):
        b = torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=DEV, generator=g)
        p, d = o.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
        h, y = split_of(p, V)
        hdrs.append(h)
        pays.append(y)
        descs.append(d)
        del b, p
    N = W * npk
    rr = torch.arange(N, device=DEV).view(W, npk).t().reshape(-1)
    key = torch.arange(N, device=DEV) + torch.randint(0, J, (N,), device=DEV, generator=g)
    perm = rr[torch.sort(key, stable=True).indices]
    hdr0, pay0, desc = torch.cat(hdrs)[perm], torch.cat(pays)[perm], torch.cat(descs)[perm]
    del hdrs, pays, descs, rr, key, perm
    out = {}
    for mode in ("local", "sorted"):
        o.set_tuning(switch_local=mode == "local")
        try:
            sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
            hdr, pay = hdr0.clone(), pay0.clone()
            act = sw.process_split(hdr, pay, desc=desc)
            out[mode + "_path"] = sw.batch_path(N)
            out[mode] = (act, pay, sw.count, sw.frag, sw.regs)
        finally:
            o.set_tuning(switch_local=True)
    assert out["local_path"] == "local" and out["sorted_path"] == "sorted"
    assert int((out["local"][0] == orc.ACT_FWD_AGG).sum()) == npk
    for a, b in zip(out["local"], out["sorted"]):
        assert torch.equal(a, b)
