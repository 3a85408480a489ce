"""N>1 path on CPU: the sharded reduce-scatter / all-gather plumbing of
ina_amd.dist over gloo with world_size 2 and 3 (127.0.0.1 rendezvous).  Inputs
are quantised by the CPU oracle (test infrastructure) since the product's
quantiser is device-only; the integer aggregate must be bit-identical to the
oracle's W-way wrapping sum (the switch's Processor add), and the int16 wire
(q16 + saturated << 22, summed in int32, decoded once per shard) bit-identical
to the single-bucket int16 saturating path with its per-slot overflow flags."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import PKG_ROOT, REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, k, results):
    import sys
    for p in (REPO, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from ina_amd.dist import (ShardPlan, all_gather_shards, all_reduce_sum, reduce_scatter_a2a,
                              reduce_scatter_sum)
    from oracle import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(1000 + rank)
        g = (rng.standard_normal(n) * 3e3).astype(np.float32)     # wraps at k=20
        q = orc.quantize_i32(g, k)
        plan = ShardPlan(n, world, align=1024)
        qp = torch.zeros(plan.padded, dtype=torch.int32)
        qp[:n] = torch.from_numpy(q)
        shard = reduce_scatter_sum(qp, plan)
        full = all_gather_shards(shard, plan)
        ar = all_reduce_sum(qp.clone())              # the collective="allreduce" variant
        a2a = reduce_scatter_a2a(qp, plan)           # the collective="a2a" variant
        results[rank] = (shard.numpy().copy(), full[:n].numpy().copy(), plan.range_of(rank),
                         ar[:n].numpy().copy(), a2a.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 100_003), (3, 5000), (2, 1), (8, 50_001)])
def test_sharded_integer_aggregate_gloo(world, n):
    k = 20
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, k, results), nprocs=world, join=True)
    from oracle import oracle as orc
    qs = [orc.quantize_i32((np.random.default_rng(1000 + r).standard_normal(n) * 3e3)
                           .astype(np.float32), k) for r in range(world)]
    want = orc.sum_reduce_i32(qs)
    for r in range(world):
        shard, full, (lo, hi), ar, a2a = results[r]
        assert np.array_equal(full, want)
        assert np.array_equal(ar, want)
        assert np.array_equal(a2a, shard)          # all-to-all + local sum == reduce-scatter
        assert np.array_equal(shard[: hi - lo], want[lo:hi])
        assert not shard[hi - lo:].any()        # padding stays zero


def test_shard_plan_alignment():
    from ina_amd.dist import ShardPlan
    p = ShardPlan(268_435_456, 8)
    assert p.shard % 1024 == 0 and p.padded >= p.n and p.shard * 8 == p.padded
    assert p.range_of(7)[1] == p.n
    p = ShardPlan(25_557_032, 3, align=256)
    rs = [p.range_of(r) for r in range(3)]
    assert rs[0][0] == 0 and rs[-1][1] == p.n and all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    assert ShardPlan(0, 4).padded == 0


def _worker_i16(rank, world, port, n, k, V, results):
    import sys
    for p in (REPO, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import math
    from ina_amd.dist import ShardPlan, all_gather_shards, all_reduce_sum, reduce_scatter_sum
    from oracle import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = _i16_bucket(rank, n)
        wire = orc.quantize_i16_wire(x, k)
        plan = ShardPlan(n, world, align=1024 * V // math.gcd(1024, V))
        wp = torch.zeros(plan.padded, dtype=torch.int32)
        wp[:n] = torch.from_numpy(wire)
        shard = reduce_scatter_sum(wp, plan)
        o16, y, ovf = orc.i16_wire_finish(shard.numpy(), k, V)
        full16 = all_gather_shards(torch.from_numpy(o16), plan)
        fully = all_gather_shards(torch.from_numpy(y), plan)
        fullf = all_gather_shards(torch.from_numpy(ovf), plan)
        results[rank] = (full16[:n].numpy().copy(), fully[:n].numpy().copy(),
                         fullf[: (n + V - 1) // V].numpy().copy())
    finally:
        dist.destroy_process_group()


def _i16_bucket(rank, n):
    """~N(0, 1) gradients with a few 100x outliers: at k=11 a single value saturates
    past |x| = 16, and the sum of several ranks saturates more often."""
    rng = np.random.default_rng(1000 + rank)
    x = rng.standard_normal(n).astype(np.float32)
    idx = rng.choice(n, max(1, n // 200), replace=False)
    x[idx] *= 100
    if n > 7:
        x[7] = np.nan
    return x


@pytest.mark.parametrize("world,n,V", [(2, 100_003, 256), (3, 5000, 32), (2, 1, 256), (4, 9000, 100), (8, 60_000, 32)])
def test_sharded_i16_wire_gloo(world, n, V):
    k = 11
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker_i16, args=(world, _free_port(), n, k, V, results), nprocs=world, join=True)
    from oracle import oracle as orc
    want16, want_ovf = orc.quantize_reduce_i16_sat([_i16_bucket(r, n) for r in range(world)], k, V)
    assert 0 < want_ovf.sum() < want_ovf.size or n < 2 * V     # the flag path is exercised
    for r in range(world):
        o16, y, ovf = results[r]
        assert np.array_equal(o16, want16)
        assert np.array_equal(y, orc.dequantize_i16(want16, k))
        assert np.array_equal(ovf, want_ovf)


def test_i16_wire_oracle_identity():
    """The wire decode equals the one-GPU int16 path for every rank count up to the
    wire's limit (64): extremes of the 22-bit field included."""
    from oracle import oracle as orc
    rng = np.random.default_rng(5)
    n, V, k = 4096, 256, 0
    for world in (1, 2, 7, 64):
        xs = [rng.integers(-40000, 40000, n).astype(np.float32) for _ in range(world)]
        xs[0][:64] = 32767.0                       # all ranks at the top: 64 * 32767 < 2^21
        for x in xs:
            x[:64] = 32767.0
            x[64:128] = -32768.0                   # and the bottom: 64 * -32768 = -2^21
        s = np.zeros(n, np.int64)
        for x in xs:
            s += orc.quantize_i16_wire(x, k)
        assert np.abs(s).max() < 2 ** 31
        o16, y, ovf = orc.i16_wire_finish(s.astype(np.int32), k, V)
        w16, wovf = orc.quantize_reduce_i16_sat(xs, k, V)
        assert np.array_equal(o16, w16) and np.array_equal(ovf, wovf)


def test_range_aggregator_host_checks():
    """Layout B's host side without a GPU: one rank owns the whole range; worker slices of
    the wrong length and unknown wires are refused before any kernel runs."""
    from ina_amd.dist import RangeAggregator
    agg = RangeAggregator(5000, device=torch.device("cpu"))
    assert agg.range == (0, 5000) and agg.plan.padded >= 5000
    with pytest.raises(ValueError):
        agg.aggregate_int([torch.zeros(4999), torch.zeros(5000)])
    with pytest.raises(ValueError):
        agg([])
    with pytest.raises(ValueError):
        RangeAggregator(10, wire="i8", device=torch.device("cpu"))
    a16 = RangeAggregator(3000, wire="i16", V=100, device=torch.device("cpu"))
    assert a16.plan.shard % 100 == 0 and a16.ovf_shard.numel() == a16.plan.shard // 100
    with pytest.raises(AttributeError):
        _ = agg.overflow
    from ina_amd.dist import ShardedAggregator
    with pytest.raises(ValueError):
        ShardedAggregator(10, device=torch.device("cpu"), collective="tree")
    with pytest.raises(ValueError):             # chunks pipeline the RS + AG pair only
        ShardedAggregator(10, device=torch.device("cpu"), collective="allreduce", chunks=2)
    one = ShardedAggregator(5000, device=torch.device("cpu"), chunks=4)
    assert one.chunks == 1 and one.gather_bytes == 0      # one rank: nothing to pipeline


def _worker_chunk_plan(rank, world, port, results):
    import math
    import sys
    for p in (REPO, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from ina_amd.dist import ShardedAggregator
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for n, wire, V, C in [(1, "i32", 256, 2), (1_000_003, "i32", 256, 4), (300_001, "i16", 100, 3),
                              (268_435_456 // 64, "i16", 256, 4)]:
            a = ShardedAggregator(n, device=torch.device("cpu"), wire=wire, V=V, chunks=C)
            align = 1024 if wire == "i32" else 1024 * V // math.gcd(1024, V)
            L = a.cplan.padded
            out.append((a.chunks == C, a.cplan.shard == a.sc, a.sc % align == 0, L == world * a.sc,
                        a.cpad == C * L >= n, (C - 1) * L < n or n < C * world * align,
                        a._qbuf.numel() >= max(a.cpad, a.plan.padded),
                        a.gather_bytes == (world - 1) * (C * a.sc * (4 if wire == "i32" else 2)
                                                         + (0 if wire == "i32" else C * a.sc // V)),
                        not a._shard_bufs))    # whole-bucket shard buffers: lazy when chunked
        full = ShardedAggregator(1000, device=torch.device("cpu"))      # unchunked: allocated up front
        out.append((set(full._shard_bufs) == {"sum", "f"}, full.sum_shard.numel() == full.plan.shard))
        results[rank] = out
    finally:
        dist.destroy_process_group()


def test_sharded_chunk_plan_invariants_gloo():
    """The pipelined layout-A plan at world 2 (host side, no kernels): every chunk is
    world x Sc values, Sc a whole number of aligned slots, the chunks cover the bucket
    without a wholly empty tail beyond the alignment, and the gather bytes add up."""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker_chunk_plan, args=(2, _free_port(), results), nprocs=2, join=True)
    for r in range(2):
        for case in results[r]:
            assert all(case), case
