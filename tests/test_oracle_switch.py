"""Known-answer tests for the oracle's P4 aggregator restatement.

The P4 program (src/p4/p4src/ngaa.p4, processor.p4, fragcheck.p4) cannot be
compiled or run here (no Tofino SDE), so these answers are derived by hand
from the P4 source; each test names the lines it exercises.
"""
import numpy as np
import pytest

from oracle import oracle as orc

V = 32


def pkt(vals, bitmap=1, count=2, switch_id=1, index=0, frag=1, flags=0):
    vals = np.asarray(vals, np.int64).astype(np.uint32).view(np.int32)
    p = orc.pack_nga(vals, V, bitmap, count, switch_id, seq0=frag, flags=flags,
                     num_slots=2**32 - 1 if index is None else 16384)
    p = p.copy()
    if index is not None:
        p[0, 6:10] = np.frombuffer(int(index).to_bytes(4, "big"), np.uint8)
    return p


def vals_of(p):
    return orc.unpack_nga(p.reshape(-1), V)[1]


@pytest.mark.parametrize("W", [2, 3, 8, 16])
def test_w_way_completion_and_sum(W):
    """ngaa.p4:64-82 count, processor.p4:16-22 first-overwrite then add, 170-175 route/drop."""
    sw = orc.Switch(V)
    rng = np.random.default_rng(W)
    data = rng.integers(-2**31, 2**31, size=(W, V), dtype=np.int64)
    for w in range(W):
        out, act = sw.run(pkt(data[w], bitmap=w + 1, count=W, index=5, frag=9))
        if w < W - 1:
            assert act[0] == orc.ACT_DROP
        else:
            assert act[0] == orc.ACT_FWD_AGG
            want = (data.sum(0) % 2**32).astype(np.uint32).view(np.int32)
            assert np.array_equal(vals_of(out), want)
    cnt, frag, regs = sw.registers()
    assert cnt[5] == 0 and frag[5] == 9


def test_intermediate_packets_carry_running_sum():
    """processor.p4:22 out_value = register after the add (written into the packet)."""
    sw = orc.Switch(V)
    a = np.arange(V)
    out, act = sw.run(np.concatenate([pkt(a, count=3), pkt(10 * a, count=3)]))
    assert list(act) == [orc.ACT_DROP, orc.ACT_DROP]
    assert np.array_equal(vals_of(out[1:]), 11 * a)


def test_mod_2_32_wrap():
    sw = orc.Switch(V)
    big = np.full(V, 2**31 - 1)
    sw.run(pkt(big, count=2))
    out, act = sw.run(pkt(np.full(V, 2), count=2))
    assert act[0] == orc.ACT_FWD_AGG
    assert (vals_of(out) == np.int32(-2**31 + 1)).all()


def test_next_round_overwrites_stale_register():
    """count==1 (first packet of a round) overwrites: processor.p4:16-17."""
    sw = orc.Switch(V)
    sw.run(np.concatenate([pkt(np.full(V, 7)), pkt(np.full(V, 7))]))
    out, act = sw.run(np.concatenate([pkt(np.full(V, 1)), pkt(np.full(V, 2))]))
    assert list(act) == [orc.ACT_DROP, orc.ACT_FWD_AGG]
    assert (vals_of(out[1:]) == 3).all()


def test_degree_one_adds_to_stale_register():
    """Degree 1: count goes 1 == hdr.count -> reset to 0, so meta.count == 0 and the
    Processor ADDS to whatever the slot held (ngaa.p4:68-76, processor.p4:16-20)."""
    sw = orc.Switch(V)
    sw.run(np.concatenate([pkt(np.full(V, 100)), pkt(np.full(V, 5))]))  # slot holds 105
    out, act = sw.run(pkt(np.full(V, 1), count=1))
    assert act[0] == orc.ACT_FWD_AGG
    assert (vals_of(out) == 106).all()
    out, act = sw.run(pkt(np.full(V, 1), count=1))
    assert (vals_of(out) == 107).all()


def test_collision_passes_through_unaggregated():
    """fragcheck.p4:14-24 holder mismatch -> collision=1, route (ngaa.p4:177-181)."""
    sw = orc.Switch(V)
    sw.run(pkt(np.full(V, 4), count=2, frag=1))
    p = pkt(np.full(V, 9), count=2, frag=2)
    out, act = sw.run(p)
    assert act[0] == orc.ACT_FWD_COLLISION
    assert out[0, 5] & orc.FLAG_COLLISION
    assert (vals_of(out) == 9).all()
    cnt, frag, regs = sw.registers()
    assert frag[0] == 1 and cnt[0] == 1 and (regs[0] == 4).all()


def test_ack_clears_frag_and_keeps_registers():
    """is_ack: reset_id sets the frag register to 0 (fragcheck.p4:26-31), routed (130-132)."""
    sw = orc.Switch(V)
    sw.run(np.concatenate([pkt(np.full(V, 1), frag=3), pkt(np.full(V, 1), frag=3)]))
    out, act = sw.run(pkt(np.zeros(V), frag=3, flags=orc.FLAG_ACK))
    assert act[0] == orc.ACT_FWD_ACK
    cnt, frag, regs = sw.registers()
    assert frag[0] == 0 and (regs[0] == 2).all()
    out, act = sw.run(pkt(np.full(V, 8), frag=4))   # new fragment claims the slot
    assert act[0] == orc.ACT_DROP
    assert sw.registers()[1][0] == 4


def test_frag_zero_looks_free_and_merges():
    """A slot 'held' by frag 0 still reads as unused, so the next fragment claims it
    and joins the aggregation in progress (fragcheck.p4:16-18)."""
    sw = orc.Switch(V)
    out, act = sw.run(pkt(np.full(V, 1), count=2, frag=0))
    assert act[0] == orc.ACT_DROP and sw.registers()[1][0] == 0
    out, act = sw.run(pkt(np.full(V, 2), count=2, frag=7))
    assert act[0] == orc.ACT_FWD_AGG
    assert (vals_of(out) == 3).all()


def test_u8_count_wraps_with_degree_zero():
    """bit<8> count register: with hdr.count 0 the slot completes only when value+1
    wraps to 0, i.e. on the 256th packet (ngaa.p4:68-71)."""
    sw = orc.Switch(V)
    stream = np.concatenate([pkt(np.full(V, 1), count=0) for _ in range(256)])
    out, act = sw.run(stream)
    assert (act[:255] == orc.ACT_DROP).all() and act[255] == orc.ACT_FWD_AGG
    # the 256th packet: meta.count == 0 != 1 so it adds; packet 1 had count 1 (overwrite)
    assert (vals_of(out[255:]) == 256).all()


def test_other_switch_id_is_forwarded_untouched():
    """switch_check miss -> unset_agg -> ipRoute (ngaa.p4:27-37,184-186)."""
    sw = orc.Switch(V, switch_id=1)
    p = pkt(np.full(V, 3), switch_id=2)
    out, act = sw.run(p)
    assert act[0] == orc.ACT_FWD_OTHER and np.array_equal(out, p)
    cnt, frag, regs = sw.registers()
    assert not cnt.any() and not frag.any() and not regs.any()


def test_index_wraps_into_register_pool():
    """index is bit<32>; the pool holds NUM_REGISTER=16384 slots (config.p4:5)."""
    sw = orc.Switch(V)
    sw.run(pkt(np.full(V, 1), index=16384 + 3, frag=5))
    assert sw.registers()[1][3] == 5


@pytest.mark.parametrize("W,V_", [(2, 32), (4, 128), (8, 256)])
def test_stateful_equals_bulk_sum_collision_free(W, V_):
    """Collision-free streams with PS acks: the packet-level switch yields exactly the
    bulk W-way wrapping sum."""
    rng = np.random.default_rng(W * V_)
    n = 40 * V_ + 7
    bufs = [rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
            for _ in range(W)]
    want = orc.sum_reduce_i32(bufs)
    pk = [orc.pack_nga(b, V_, bitmap=w + 1, count=W, switch_id=1, seq0=1)
          for w, b in enumerate(bufs)]
    sw = orc.Switch(V_, num_slots=16)      # small pool -> slots are reused after acks
    got = np.zeros(pk[0].shape[0] * V_, np.int32)
    for s in range(pk[0].shape[0]):
        order = rng.permutation(W)
        out, act = sw.run(np.stack([pk[w][s] for w in order]))
        assert (act[:-1] == orc.ACT_DROP).all() and act[-1] == orc.ACT_FWD_AGG
        got[s * V_:(s + 1) * V_] = orc.unpack_nga(out[-1], V_)[1]
        ack = out[-1:].copy()
        ack[0, 5] = orc.FLAG_ACK
        assert sw.run(ack)[1][0] == orc.ACT_FWD_ACK
    assert np.array_equal(got[:n], want)


def test_cpu_pipeline_equals_bulk_sum():
    rng = np.random.default_rng(3)
    n = 5000
    bufs = [rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
            for _ in range(8)]
    want = orc.sum_reduce_i32(bufs)
    for threads in (1, 3):
        got, secs = orc.cpu_packetise_aggregate(bufs, 256, threads)
        assert np.array_equal(got, want) and secs > 0
