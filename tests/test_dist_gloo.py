"""N>1 path on CPU: the sharded reduce-scatter / all-gather plumbing of
ina_amd.dist over gloo with world_size 2 and 3 (127.0.0.1 rendezvous).  Inputs
are quantised by the CPU oracle (test infrastructure) since the product's
quantiser is device-only; the integer aggregate must be bit-identical to the
oracle's W-way wrapping sum (the switch's Processor add)."""
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
    from ina_amd.dist import ShardPlan, all_gather_shards, reduce_scatter_sum
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
        results[rank] = (shard.numpy().copy(), full[:n].numpy().copy(), plan.range_of(rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 100_003), (3, 5000), (2, 1)])
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
        shard, full, (lo, hi) = results[r]
        assert np.array_equal(full, want)
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
