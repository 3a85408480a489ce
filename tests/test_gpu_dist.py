"""Sharded aggregation (SURVEY.md 8e, config 5 layout A) at world size > 1 with the
device kernels: 2, 3 and 8 ranks launched by torch.distributed.run, all on cuda:0 with a gloo
group (the collectives stage through host memory; one GPU cannot hold two RCCL ranks),
quantise / wire decode / dequantise through libina.so.  Every rank's full aggregate is
compared bit for bit with the oracle's single-bucket path over all ranks' buckets:
  i32: dequantize_i32(quantize_reduce_i32)           (the switch's wrapping slot sum)
  i16: dequantize_i16(quantize_reduce_i16_sat) + the per-slot overflow flags
Layout B (RangeAggregator: every worker's slice of a rank's range on that rank, a local
fused quantise + reduce, an all-gather) against the same oracle.
Plus config 5 at its full size on one rank (1 GiB bucket), checked on a strided sample."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import REPO
from tests._dist_gpu_rank import bucket

# the ranks load the library this run tests (INA_LIBRARY: a checked variant build)
LIB_NAME = os.path.basename(os.environ.get("INA_LIBRARY", "libina.so"))

RANK_SCRIPT = os.path.join(REPO, "tests", "_dist_gpu_rank.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, world, n, wire, k, V=256, layout="A", workers=0, collective="rs_ag", chunks=1):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", RANK_SCRIPT,
           "--size", str(n), "--wire", wire, "--k", str(k), "--V", str(V), "--out", str(tmp_path),
           "--layout", layout, "--workers", str(workers), "--collective", collective,
           "--chunks", str(chunks)]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return [dict(np.load(os.path.join(tmp_path, f"rank{i}.npz"))) for i in range(world)]


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,coll", [(2, 1_000_003, "rs_ag"), (3, 70_001, "rs_ag"), (2, 1, "rs_ag"),
                                          (8, 400_001, "rs_ag"), (3, 70_001, "allreduce"), (3, 70_001, "a2a"), (8, 400_001, "a2a"),
                                          (3, 70_001, "chunks3"), (2, 1, "chunks2"), (8, 400_001, "chunks4")])
def test_sharded_i32_two_ranks_device_kernels(tmp_path, world, n, coll):
    """Layout A, int32 wire: reduce-scatter + all-gather, the all-reduce variant, the
    all-to-all + device-sum reduce-scatter (a2a), and the pipelined chunks (chunksC: C
    async reduce-scatters / all-gathers)."""
    from oracle import oracle as orc
    k = 20
    chunks = int(coll[6:]) if coll.startswith("chunks") else 1
    res = _run_ranks(tmp_path, world, n, "i32", k, collective="rs_ag" if chunks > 1 else coll,
                     chunks=chunks)
    want_int = orc.quantize_reduce_i32([bucket(r, n, "i32") for r in range(world)], k)
    want = orc.dequantize_i32(want_int, k)
    for r, d in enumerate(res):
        assert int(d["world"][0]) == world
        assert d["lib"][0].endswith(LIB_NAME)
        assert np.array_equal(d["full"].view(np.uint32), want.view(np.uint32)), f"rank {r}"
        lo, hi = d["range"]
        assert np.array_equal(d["shard"], want_int[lo:hi])
        gb, shard = (int(v) for v in d["gather_bytes"])      # fp32 aggregate (or int32 wire) gathered
        assert gb == (world - 1) * 4 * shard


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,V,coll", [(2, 1_000_003, 256, "rs_ag"), (3, 50_000, 32, "rs_ag"),
                                            (2, 300, 100, "rs_ag"), (8, 200_000, 32, "rs_ag"),
                                            (3, 50_000, 32, "allreduce"), (3, 50_000, 32, "chunks4"), (4, 60_000, 32, "a2a"),
                                            (2, 300_001, 100, "chunks3")])
def test_sharded_i16_two_ranks_device_kernels(tmp_path, world, n, V, coll):
    from oracle import oracle as orc
    k = 11
    chunks = int(coll[6:]) if coll.startswith("chunks") else 1
    res = _run_ranks(tmp_path, world, n, "i16", k, V, collective="rs_ag" if chunks > 1 else coll,
                     chunks=chunks)
    want16, want_ovf = orc.quantize_reduce_i16_sat([bucket(r, n, "i16") for r in range(world)], k, V)
    assert want_ovf.any() and not want_ovf.all()
    want = orc.dequantize_i16(want16, k)
    for r, d in enumerate(res):
        assert np.array_equal(d["full"].view(np.uint32), want.view(np.uint32)), f"rank {r}"
        assert np.array_equal(d["ovf"], want_ovf), f"rank {r}"
        lo, hi = d["range"]
        assert np.array_equal(d["shard"], want16[lo:hi])
        gb, shard = (int(v) for v in d["gather_bytes"])      # int16 sums + flags gathered
        assert gb == (world - 1) * (4 * shard if coll == "allreduce" else 2 * shard + shard // V)


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,W", [(2, 1_000_003, 2), (3, 70_001, 5), (8, 400_001, 8), (8, 3000, 3)])
def test_range_layout_b_i32_device_kernels(tmp_path, world, n, W):
    """Layout B: each rank reduces the W workers' slices of its own range (fused quantise +
    reduce kernel), decodes, all-gathers -- the same bits as the single-bucket path."""
    from oracle import oracle as orc
    k = 20
    res = _run_ranks(tmp_path, world, n, "i32", k, layout="B", workers=W)
    want_int = orc.quantize_reduce_i32([bucket(w, n, "i32") for w in range(W)], k)
    want = orc.dequantize_i32(want_int, k)
    for r, d in enumerate(res):
        assert d["lib"][0].endswith(LIB_NAME)
        assert np.array_equal(d["full"].view(np.uint32), want.view(np.uint32)), f"rank {r}"
        lo, hi = d["range"]
        assert np.array_equal(d["shard"], want_int[lo:hi])
        gb, shard = (int(v) for v in d["gather_bytes"])      # fp32 aggregate gathered
        assert gb == (world - 1) * 4 * shard


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,V,W", [(2, 1_000_003, 256, 2), (3, 50_000, 32, 4), (8, 200_000, 32, 8),
                                         (3, 300_001, 100, 3)])
def test_range_layout_b_i16_device_kernels(tmp_path, world, n, V, W):
    from oracle import oracle as orc
    k = 11
    res = _run_ranks(tmp_path, world, n, "i16", k, V, layout="B", workers=W)
    want16, want_ovf = orc.quantize_reduce_i16_sat([bucket(w, n, "i16") for w in range(W)], k, V)
    assert want_ovf.any() and not want_ovf.all()
    want = orc.dequantize_i16(want16, k)
    for r, d in enumerate(res):
        assert np.array_equal(d["full"].view(np.uint32), want.view(np.uint32)), f"rank {r}"
        assert np.array_equal(d["ovf"], want_ovf), f"rank {r}"
        lo, hi = d["range"]
        assert np.array_equal(d["shard"], want16[lo:hi])
        gb, shard = (int(v) for v in d["gather_bytes"])      # int16 sums + flags gathered
        assert gb == (world - 1) * (2 * shard + shard // V)


@pytest.mark.gpu
def test_c5_full_size_one_rank_strided_sample():
    """Config 5's 1 GiB fp32 bucket (268,435,456 values) through ShardedAggregator on one
    rank, both wires; every 4099th value plus the last 10,000 against the oracle."""
    import torch
    from ina_amd.dist import ShardedAggregator
    from oracle import oracle as orc
    n, dev = 268_435_456, torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1000)
    x = torch.randn(n, device=dev, generator=g) * 1e-2
    idx = np.concatenate([np.arange(0, n, 4099), np.arange(n - 10_000, n)])
    tidx = torch.from_numpy(idx).to(dev)
    xs = x[tidx].cpu().numpy()
    agg = ShardedAggregator(n, k=16, device=dev)
    y = agg(x)
    assert np.array_equal(y[tidx].cpu().numpy(), orc.dequantize_i32(orc.quantize_i32(xs, 16), 16))
    del agg, y
    agg = ShardedAggregator(n, k=20, device=dev, wire="i16", V=256)   # 1e-2 * 2^20 saturates often
    y = agg(x)
    w16, _ = orc.quantize_reduce_i16_sat([xs], 20, 1)
    assert np.array_equal(y[tidx].cpu().numpy(), orc.dequantize_i16(w16, 20))
    ovf = agg.overflow.cpu().numpy()
    assert ovf.size == n // 256
    slots = np.unique(idx // 256)
    sat = np.zeros(n // 256, bool)
    _, f1 = orc.quantize_reduce_i16_sat([xs], 20, 1)
    np.logical_or.at(sat, idx // 256, f1.astype(bool))
    # a sampled saturating value flags its slot; unsampled values may flag more
    assert (ovf[slots][sat[slots]] == 1).all()
    full_slot = x[: 256 * 64].cpu().numpy()                   # 64 whole slots exactly
    _, f64 = orc.quantize_reduce_i16_sat([full_slot], 20, 256)
    assert np.array_equal(ovf[:64], f64)


@pytest.mark.gpu
def test_c5_layout_b_full_size_one_rank_strided_sample():
    """Layout B at config 5's size on one rank: two workers' 1 GiB fp32 slices (the whole
    range) through RangeAggregator's fused quantise + reduce and decode; every 4099th
    value plus the last 10,000 against the oracle."""
    import torch
    from ina_amd.dist import RangeAggregator
    from oracle import oracle as orc
    n, dev = 268_435_456, torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(2000)
    xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(2)]
    idx = np.concatenate([np.arange(0, n, 4099), np.arange(n - 10_000, n)])
    tidx = torch.from_numpy(idx).to(dev)
    agg = RangeAggregator(n, k=16, device=dev)
    assert agg.range == (0, n)
    y = agg(xs)
    want = orc.dequantize_i32(orc.quantize_reduce_i32([x[tidx].cpu().numpy() for x in xs], 16), 16)
    assert np.array_equal(y[tidx].cpu().numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3, 4, 255, 1000, 65_536, 1_000_003])
@pytest.mark.parametrize("V", [32, 256, 100, 512])
def test_i16_wire_kernels_vs_oracle(n, V):
    """ina_quantize_f32_i16_wire and ina_i16_wire_finish bit-exact against the oracle,
    aligned (vector) and offset-by-one (scalar) buffers, summed over 3 ranks' wires."""
    import torch
    from ina_amd import ops
    from oracle import oracle as orc
    k, dev = 11, torch.device("cuda", 0)
    xs = [bucket(r, n, "i16") for r in range(3)]
    for off in (0, 1):
        wires = []
        for x in xs:
            buf = torch.zeros(n + off, dtype=torch.float32, device=dev)
            buf[off:] = torch.from_numpy(x).to(dev)
            wbuf = torch.zeros(n + off, dtype=torch.int32, device=dev)
            ops.quantize_i16_wire(buf[off:], k, out=wbuf[off:])
            w = wbuf[off:].cpu().numpy()
            assert np.array_equal(w, orc.quantize_i16_wire(x, k)), (off, n, V)
            wires.append(w.astype(np.int64))
        wsum = np.sum(wires, axis=0).astype(np.int32)
        src = torch.zeros(n + off, dtype=torch.int32, device=dev)
        src[off:] = torch.from_numpy(wsum).to(dev)
        o16 = torch.empty(n + off, dtype=torch.int16, device=dev)
        yv = torch.empty(n + off, dtype=torch.float32, device=dev)
        g16, gy, govf = ops.i16_wire_finish(src[off:], k, V, out16=o16[off:], y=yv[off:])
        w16, wy, wovf = orc.i16_wire_finish(wsum, k, V)
        assert np.array_equal(g16.cpu().numpy(), w16), (off, n, V)
        assert np.array_equal(gy.cpu().numpy().view(np.uint32), wy.view(np.uint32))
        assert np.array_equal(govf.cpu().numpy(), wovf), (off, n, V)
        r16, rovf = orc.quantize_reduce_i16_sat(xs, k, V)         # the one-GPU int16 path
        assert np.array_equal(w16, r16) and np.array_equal(wovf, rovf)
        # flags only (no value outputs) writes every slot flag too
        ovf = torch.full(((n + V - 1) // V,), 7, dtype=torch.uint8, device=dev)
        ops.i16_wire_finish(src[off:], k, V, overflow=ovf, want_out16=False, want_y=False)
        assert np.array_equal(ovf.cpu().numpy(), wovf)


@pytest.mark.gpu
def test_rccl_world1_collectives_on_this_image():
    """The config-5 collectives through RCCL itself (backend nccl, one rank: one GPU
    cannot host two RCCL ranks), so the N > 1 bench's calls -- process group with
    device_id, reduce_scatter_tensor(int32, SUM), all_gather_into_tensor (fp32, int16, uint8),
    all_reduce(float64, MAX/MIN) -- are known to run on this ROCm/RCCL image."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "_rccl_world1.py")]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rccl world-1 collectives ok" in r.stdout
