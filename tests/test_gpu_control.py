"""GPU: ipRoute on the device (ops.route_ipv4) against the oracle's restatement of
ngaa.p4:39-61, and the control plane driving the device switch -- an empty
switch_check, and a two-aggregator bucket plan whose forwarded packets reach their
owner and end as the single-switch oracle's sums."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests.test_gpu_parity import dev, host, make_stream, ops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _table(rng, rows, pool):
    keys = rng.choice(pool, size=rows, replace=False).astype(np.uint32)
    ports = rng.integers(-2, 512, size=rows).astype(np.int32)
    return list(zip(keys.tolist(), ports.tolist()))


@pytest.mark.parametrize("npk,rows,per_packet", [(1, 1, True), (1000, 0, True), (4099, 3, False),
                                                 (200_001, 256, True), (70_000, 17, False)])
def test_route_matches_oracle(npk, rows, per_packet):
    rng = np.random.default_rng(npk + rows)
    o = ops()
    pool = rng.integers(0, 2**32, size=600, dtype=np.uint64).astype(np.uint32)
    table = _table(rng, rows, pool)
    act = rng.integers(0, 5, size=npk).astype(np.uint8)
    dst = rng.choice(pool, size=npk).astype(np.uint32) if per_packet else None
    dflt = int(pool[3])
    want = orc.route_ipv4(act, table, dst, dflt)
    keys = dev(np.array([k for k, _ in table], np.uint32).view(np.int32))
    ports = dev(np.array([p for _, p in table], np.int32))
    got = o.route_ipv4(dev(act), keys, ports, None if dst is None else dev(dst.view(np.int32)), dflt)
    assert np.array_equal(host(got), want)


def test_route_empty_batch_and_bad_table():
    o = ops()
    e = torch.empty(0, dtype=torch.uint8, device=DEV)
    k = torch.zeros(1, dtype=torch.int32, device=DEV)
    assert o.route_ipv4(e, k, k).numel() == 0
    big = torch.zeros(257, dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        o.route_ipv4(torch.zeros(4, dtype=torch.uint8, device=DEV), big, big)


def test_empty_switch_check_forwards_everything():
    from ina_amd import control
    o = ops()
    rng = np.random.default_rng(5)
    cp = control.reference_setup()
    cp.clear_all()                                   # no set_agg row: unset_agg for all
    cp.Ingress.ipRoute.add_with_ipv4_forward("172.16.170.1", dst_mac=1, port=132)
    sw = cp.make_switch(32, num_slots=64, device=DEV)
    stream = make_stream(rng, 32, 20, 4, 64)
    d = dev(stream)
    act = sw.process(d)
    assert (host(act) == orc.ACT_FWD_OTHER).all()
    assert np.array_equal(host(d), stream)           # untouched, like the P4 pass-through
    assert not host(sw.regs).any() and not host(sw.count).any()
    eg = cp.egress(act, dst_default="172.16.170.1")
    assert (host(eg) == 132).all()
    assert (host(cp.egress(act, dst_default="172.16.170.9")) == -1).all()


def test_two_aggregator_bucket_plan_matches_single_switch():
    """Buckets split over two device aggregators (switch ids 1, 2).  Every packet goes to
    aggregator A first; A aggregates its buckets and forwards the rest by ipRoute to B's
    port; B aggregates those.  Each completed slot equals the bulk sum."""
    from ina_amd import control
    o = ops()
    rng = np.random.default_rng(11)
    V, W = 64, 4
    sizes = [V * 40 + 3, V * 25, V * 31 + 9, V * 12]
    plan = control.BucketPlan(sizes, 2, base_id=1)
    ps, a_ip, b_ip = "10.0.0.100", "10.0.0.1", "10.0.0.2"
    cps = [plan.control_plane(r, ps, 5, agg_addrs=[a_ip, b_ip], agg_ports=[1, 2]) for r in range(2)]
    sws = [cp.make_switch(V, num_slots=4096, device=DEV) for cp in cps]
    bufs = [[rand(rng, n) for _ in range(W)] for n in sizes]
    streams, dsts, seq0 = [], [], 1
    starts = []
    for b, n in enumerate(sizes):
        starts.append(seq0)
        owner_ip = control.ip2int([a_ip, b_ip][plan.owner(b)])
        for w in range(W):
            pk = o.pack_nga(dev(bufs[b][w]), V, w + 1, W, plan.switch_id(b), seq0, num_slots=4096)
            streams.append(pk)
            # the owner's own packets are addressed to the PS (it sits in the path);
            # packets for the other aggregator carry that aggregator's address
            want_dst = control.ip2int(ps) if plan.owner(b) == 0 else owner_ip
            dsts.append(np.full(pk.shape[0], want_dst, np.uint32))
        seq0 += -(-n // V)
    stream = torch.cat(streams)
    dst = dev(np.concatenate(dsts).view(np.int32))
    perm = torch.from_numpy(rng.permutation(stream.shape[0])).to(DEV)
    stream, dst = stream[perm].contiguous(), dst[perm].contiguous()
    act_a = sws[0].process(stream)
    eg_a = cps[0].egress(act_a, dst)
    to_b = torch.nonzero(eg_a == 2).flatten()
    assert int(to_b.numel()) == sum(W * -(-sizes[b] // V) for b in plan.buckets_of(1))
    stream_b = stream[to_b].contiguous()
    act_b = sws[1].process(stream_b)
    eg_b = cps[1].egress(act_b, dst_default=ps)
    done = [stream[torch.nonzero((act_a == orc.ACT_FWD_AGG) & (eg_a == 5)).flatten()],
            stream_b[torch.nonzero((act_b == orc.ACT_FWD_AGG) & (eg_b == 5)).flatten()]]
    fin = torch.cat(done)
    f, vals = o.unpack_nga(fin, V)
    frag = host(f["frag_id"]).view(np.uint32).astype(np.int64)
    vals = host(vals).reshape(-1, V)
    assert len(frag) == sum(-(-n // V) for n in sizes)
    for b, n in enumerate(sizes):
        npk = -(-n // V)
        sel = (frag >= starts[b]) & (frag < starts[b] + npk)
        got = vals[sel][np.argsort(frag[sel])].reshape(-1)[:n]
        want = orc.sum_reduce_i32([x for x in bufs[b]])
        assert np.array_equal(got, want), b
        assert (host(f["switch_id"])[sel] == plan.switch_id(b)).all()


def rand(rng, n):
    return rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
