"""GPU parity: every libina.so device entry point against the CPU oracle (and,
where the reference left outputs, against the reference's own bytes).

Integer / byte / index work must be bit-exact.  The PS combine is bit-exact to
the reference's torch fp32 sequence (tolerance 0 ULP).  The quantiser is
build-defined (the reference's is missing), so its parity is against the
oracle's restatement of the same definition (bit-exact).
"""
import socket

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests._golden import load_capture, manifest, ps_cases

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


def rand_i32(rng, n, full=True):
    if full:
        return rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    return rng.integers(-2**20, 2**20, size=n, dtype=np.int64).astype(np.int32)


# --------------------------------------------------------------------------------------
# sum-reduce (processor.p4:14-24)
# --------------------------------------------------------------------------------------
@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 8, 16, 17, 64])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 4097, 100003])
def test_sum_reduce_matches_oracle(W, n):
    rng = np.random.default_rng(W * 1000 + n)
    bufs = [rand_i32(rng, n) for _ in range(W)]
    got = host(ops().sum_reduce([dev(b) for b in bufs]))
    assert np.array_equal(got, orc.sum_reduce_i32(bufs))


def test_sum_reduce_unaligned_views_take_scalar_path():
    rng = np.random.default_rng(5)
    n = 5001
    big = [dev(rand_i32(rng, n + 1)) for _ in range(8)]
    views = [b[1:] for b in big]            # 4-byte offset: not 16-byte aligned
    got = host(ops().sum_reduce(views))
    assert np.array_equal(got, orc.sum_reduce_i32([host(v) for v in views]))


def test_sum_reduce_in_place_alias():
    rng = np.random.default_rng(6)
    bufs = [rand_i32(rng, 4099) for _ in range(4)]
    want = orc.sum_reduce_i32(bufs)
    d = [dev(b) for b in bufs]
    ops().sum_reduce(d, out=d[0])
    assert np.array_equal(host(d[0]), want)


def test_sum_reduce_stacked_tensor_input():
    rng = np.random.default_rng(7)
    stack = np.stack([rand_i32(rng, 777) for _ in range(8)])
    got = host(ops().sum_reduce(dev(stack)))
    assert np.array_equal(got, orc.sum_reduce_i32(list(stack)))


@pytest.mark.parametrize("unroll,blocks,nt", [(1, 2048, True), (4, 512, True), (2, 4096, False), (0, 0, True)])
def test_sum_reduce_tunings_identical(unroll, blocks, nt):
    rng = np.random.default_rng(8)
    bufs = [rand_i32(rng, 300007) for _ in range(8)]
    o = ops()
    try:
        o.set_tuning(reduce_blocks=blocks, unroll=unroll, nontemporal=nt)
        got = host(o.sum_reduce([dev(b) for b in bufs]))
    finally:
        o.set_tuning(max_blocks=16384, unroll=0, nontemporal=True, reduce_blocks=0)   # library defaults
    assert np.array_equal(got, orc.sum_reduce_i32(bufs))


def test_sum_reduce_config3_full_size():
    """BASELINE config 3: 8 workers x 100 MiB int32, full-range values (wraps)."""
    n = 26_214_400
    rng = np.random.default_rng(1234)
    bufs = [rand_i32(rng, n) for _ in range(8)]
    got = ops().sum_reduce([dev(b) for b in bufs])
    want = orc.sum_reduce_i32(bufs)
    g = host(got)
    assert np.array_equal(g, want)
    # size-independent property: the checksum of the sum == wrapped sum of checksums
    cs = int(host(ops().checksum(got))[0]) & 0xFFFFFFFF
    assert cs == sum(orc.checksum_i32(b) for b in bufs) % 2**32 == orc.checksum_i32(want)


# PCIe-inclusive path: pinned host buckets reduced in place over PCIe (zero copy), or host
# buckets -> HBM -> reduce -> host, chunked over a 3-slot ring
@pytest.mark.parametrize("W,n,chunk", [(1, 1, 0), (3, 63, 64), (8, 100_003, 4096),
                                       (8, 100_003, 0), (17, 65_537, 1000), (64, 5000, 128)])
@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("zero_copy", [True, False])
def test_sum_reduce_host_matches_oracle(W, n, chunk, pinned, zero_copy):
    rng = np.random.default_rng(W * 31 + n + chunk)
    bufs = [rand_i32(rng, n) for _ in range(W)]
    hb = [torch.from_numpy(b) for b in bufs]
    if pinned:
        hb = [b.pin_memory() for b in hb]
    o = ops()
    try:
        o.set_tuning(host_zero_copy=zero_copy)
        got = o.sum_reduce_host(hb, chunk=chunk)
    finally:
        o.set_tuning(host_zero_copy=True)
    assert not got.is_cuda
    assert np.array_equal(got.numpy(), orc.sum_reduce_i32(bufs))


def test_sum_reduce_host_zero_copy_views_and_mixed_memory():
    """Zero copy on interior views of pinned allocations (odd offsets: the unaligned
    kernel reads host memory), and a pageable output with pinned inputs (not device-
    mapped: the call falls back to the copy pipeline) -- bit-exact either way, and a
    refused mapping query leaves no HIP error behind for the next call."""
    rng = np.random.default_rng(77)
    W, n = 5, 40_001
    big = [torch.from_numpy(rand_i32(rng, n + 3)).pin_memory() for _ in range(W)]
    o = ops()
    for off in (0, 1, 3):
        views = [b[off:off + n] for b in big]
        want = orc.sum_reduce_i32([v.numpy() for v in views])
        assert np.array_equal(o.sum_reduce_host(views).numpy(), want), off
        pageable_out = torch.empty(n, dtype=torch.int32)
        got = o.sum_reduce_host(views, out=pageable_out)
        assert got.data_ptr() == pageable_out.data_ptr() and np.array_equal(got.numpy(), want), off
    assert np.array_equal(host(o.sum_reduce([dev(b.numpy()) for b in big])),
                          orc.sum_reduce_i32([b.numpy() for b in big]))


@pytest.mark.parametrize("h2d", [1, 2])
def test_sum_reduce_host_ring_reuse_and_copy_streams(h2d):
    """Many more chunks than ring slots, both copy-stream settings, called twice with
    the same scratch: every chunk is bit-exact (slot reuse waits on the right events)."""
    rng = np.random.default_rng(h2d)
    W, n = 8, 64 * 1000 + 7
    bufs = [rand_i32(rng, n) for _ in range(W)]
    hb = [torch.from_numpy(b).pin_memory() for b in bufs]
    o = ops()
    scratch = torch.empty(o.load().ina_host_reduce_scratch_bytes(W, 64), dtype=torch.uint8, device=DEV)
    try:
        o.set_tuning(h2d_streams=h2d, host_zero_copy=False)    # the copy pipeline itself
        for _ in range(2):
            got = o.sum_reduce_host(hb, chunk=64, scratch=scratch)
            assert np.array_equal(got.numpy(), orc.sum_reduce_i32(bufs))
    finally:
        o.set_tuning(h2d_streams=2, host_zero_copy=True)


# --------------------------------------------------------------------------------------
# quantise / dequantise (build-defined; parity vs the oracle's restatement)
# --------------------------------------------------------------------------------------
EDGE = np.array([0.0, -0.0, 0.5, 1.5, 2.5, -0.5, -1.5, 1e-45, -1e-45, 1e-38, np.inf, -np.inf,
                 np.nan, 3e38, -3e38, 32767.5, -32768.5, 2147483520.0, 2147483648.0,
                 -2147483648.0, -2147483904.0, 0.49999997, -0.49999997], np.float32)


def mixed_floats(rng, n):
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-8, 8, n)).astype(np.float32)
    x[:min(n, len(EDGE))] = EDGE[:min(n, len(EDGE))]
    return x


@pytest.mark.parametrize("k", [0, 16, 24, -4, 127, -126])
@pytest.mark.parametrize("n", [1, 23, 4096, 100001])
def test_quantize_i32(k, n):
    x = mixed_floats(np.random.default_rng(n * 1000 + k + 200), n)
    assert np.array_equal(host(ops().quantize(dev(x), k)), orc.quantize_i32(x, k))


@pytest.mark.parametrize("V", [32, 128, 256, 8, 512, 100])
@pytest.mark.parametrize("n", [7, 8, 1000, 65537])
def test_quantize_i16_flags(V, n):
    x = (np.random.default_rng(V + n).standard_normal(n) * 40).astype(np.float32)
    x[: min(n, len(EDGE))] = EDGE[: min(n, len(EDGE))]
    q, ovf = ops().quantize_i16(dev(x), 10, V)
    qo, ovfo = orc.quantize_i16_sat(x, 10, V)
    assert np.array_equal(host(q), qo)
    assert np.array_equal(host(ovf), ovfo)


@pytest.mark.parametrize("k", [0, 16, 30])
def test_dequantize(k):
    rng = np.random.default_rng(k)
    s = rand_i32(rng, 70001)
    got = host(ops().dequantize(dev(s), k))
    assert np.array_equal(got.view(np.uint32), orc.dequantize_i32(s, k).view(np.uint32))
    s16 = rng.integers(-32768, 32768, 1001).astype(np.int16)
    got16 = host(ops().dequantize(dev(s16), k))
    assert np.array_equal(got16.view(np.uint32), orc.dequantize_i16(s16, k).view(np.uint32))


@pytest.mark.parametrize("n", [1, 3, 4, 257, 100003, 25_557_032])
@pytest.mark.parametrize("off", [0, 1, 4])
def test_dequantize_i16_sizes_and_alignment(n, off):
    """Vector path (8-byte aligned int16, 16-byte aligned fp32, 4 values per lane) and the
    scalar path for unaligned views; the remainder values after n/4 chunks."""
    if n > 200_000 and off:
        pytest.skip("alignment covered at small n")
    rng = np.random.default_rng(n + off)
    s16 = rng.integers(-32768, 32768, n + off).astype(np.int16)
    d = dev(s16)[off:]
    got = host(ops().dequantize(d, 13))
    assert np.array_equal(got.view(np.uint32), orc.dequantize_i16(s16[off:], 13).view(np.uint32))


def test_quantize_dequantize_round_trip_bound():
    x = (np.random.default_rng(3).standard_normal(1 << 20) * 1e-2).astype(np.float32)
    k = 16
    y = host(ops().dequantize(ops().quantize(dev(x), k), k))
    assert np.abs(y - x).max() <= 2.0 ** -(k + 1)


# --------------------------------------------------------------------------------------
# fused quantise + reduce (configs 2 and 4) and the int16 narrow reduce
# --------------------------------------------------------------------------------------
@pytest.mark.parametrize("W", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("n", [5, 1024, 50003])
def test_quantize_reduce_i32(W, n):
    rng = np.random.default_rng(W + n)
    bufs = [mixed_floats(rng, n) for _ in range(W)]
    got = host(ops().quantize_reduce([dev(b) for b in bufs], 16))
    assert np.array_equal(got, orc.quantize_reduce_i32(bufs, 16))


@pytest.mark.parametrize("W", [1, 3, 4, 8, 16])
@pytest.mark.parametrize("V", [32, 256, 96])
def test_quantize_reduce_i16(W, V):
    rng = np.random.default_rng(W * V)
    n = 20 * V + 13
    bufs = [(rng.standard_normal(n) * 3).astype(np.float32) for _ in range(W)]
    bufs[0][:len(EDGE)] = EDGE
    out, ovf = ops().quantize_reduce_i16([dev(b) for b in bufs], 10, V)
    wo, wf = orc.quantize_reduce_i16_sat(bufs, 10, V)
    assert np.array_equal(host(out), wo)
    assert np.array_equal(host(ovf), wf)
    assert 0 < wf.sum() < len(wf)     # the overflow path is exercised, not universal


@pytest.mark.parametrize("W,V", [(2, 32), (16, 256), (5, 100)])
def test_sum_reduce_i16(W, V):
    rng = np.random.default_rng(W + V)
    n = 33 * V + 3
    bufs = [rng.integers(-9000, 9000, n).astype(np.int16) for _ in range(W)]
    out, ovf = ops().sum_reduce_i16([dev(b) for b in bufs], V)
    wo, wf = orc.sum_reduce_i16_sat(bufs, V)
    assert np.array_equal(host(out), wo) and np.array_equal(host(ovf), wf)


def test_config2_full_size_fused():
    """BASELINE config 2: ResNet-50-sized fp32 bucket (25,557,032), 4 workers, int32."""
    n = 25_557_032
    bufs = [(np.random.default_rng(1000 + w).standard_normal(n) * 1e-2).astype(np.float32)
            for w in range(4)]
    got = host(ops().quantize_reduce([dev(b) for b in bufs], 16))
    assert np.array_equal(got, orc.quantize_reduce_i32(bufs, 16))


def test_config4_full_size_int16():
    """BASELINE config 4: ResNet-50 gradient, 16 workers, int16 saturating."""
    n, W, V = 25_557_032, 16, 256
    bufs = []
    for w in range(W):
        r = np.random.default_rng(1000 + w)
        g = (r.standard_normal(n) * 1e-2).astype(np.float32)
        out = r.random(n) < 0.01
        g[out] *= 100
        bufs.append(g)
    k = 13   # |sum| * 2^k exceeds int16 only for rare outlier sums: ~0.3% of slots
    q, ovf = ops().quantize_reduce_i16([dev(b) for b in bufs], k, V)
    wq, wf = orc.quantize_reduce_i16_sat(bufs, k, V)
    assert np.array_equal(host(q), wq) and np.array_equal(host(ovf), wf)
    assert 0 < wf.sum() < len(wf)


# --------------------------------------------------------------------------------------
# PS combine (launch.py:42-52): bit-exact against the reference's own outputs
# --------------------------------------------------------------------------------------
def test_ps_combine_matches_reference_aggregate_outputs():
    for name, c in ps_cases().items():
        W, K = int(c["W"]), int(c["K"])
        paras = list(c["paras"])
        if K > 0:
            paras, weight = paras[:K], 1.0 / K
        else:
            weight = 1.0 / (W + 1)
        got = host(ops().ps_combine(dev(c["local"]), [dev(p) for p in paras],
                                    weight * float(c["step"])))
        assert np.array_equal(got.view(np.uint32), c["out"].view(np.uint32)), name


def test_ps_combine_random_vs_oracle():
    rng = np.random.default_rng(11)
    n = 100_000
    local = rng.standard_normal(n).astype(np.float32)
    paras = [(local + rng.standard_normal(n).astype(np.float32) * 1e-3) for _ in range(7)]
    got = host(ops().ps_combine(dev(local), [dev(p) for p in paras], 1.0 / 8))
    want = orc.ps_combine_f32(local, paras, 1.0 / 8)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("n", [1, 3, 4, 1023, 100_003])
@pytest.mark.parametrize("with_base", [False, True])
def test_absmax_matches_numpy(n, with_base):
    """Dynamic-scale absmax: max |x - base| with NaN ignored (the quantiser maps NaN to 0),
    +-inf counted, over aligned and tail elements."""
    rng = np.random.default_rng(n + 7 * with_base)
    x = mixed_floats(rng, n)
    base = (rng.standard_normal(n) * 3).astype(np.float32) if with_base else None
    d = (x - base).astype(np.float32) if with_base else x
    a = np.abs(d[~np.isnan(d)])
    want = np.float32(a.max()) if a.size else np.float32(0)
    got = host(ops().absmax(dev(x), dev(base) if with_base else None))[0]
    assert got.view(np.uint32) == want.view(np.uint32)


@pytest.mark.parametrize("W", [1, 3, 4, 5, 16])
@pytest.mark.parametrize("n", [1, 6, 1023, 100_003])
@pytest.mark.parametrize("with_base", [False, True])
def test_absmax_multi_equals_max_of_single(W, n, with_base):
    """ina_absmax_multi_f32 (one pass over W buckets, base read once) == the max of the W
    single-bucket absmax values, bit for bit; NaN ignored, +-inf counted; W not a multiple
    of the kernel's 4-worker groups, aligned and tail elements."""
    rng = np.random.default_rng(W * 1000 + n + with_base)
    xs = [mixed_floats(rng, n) for _ in range(W)]
    base = (rng.standard_normal(n) * 3).astype(np.float32) if with_base else None
    o = ops()
    db = dev(base) if with_base else None
    got = host(o.absmax_multi([dev(x) for x in xs], db))[0]
    want = max(host(o.absmax(dev(x), db))[0] for x in xs)
    assert got.view(np.uint32) == np.float32(want).view(np.uint32)
    # an unaligned view takes the element path
    got_u = host(o.absmax_multi([dev(x)[1:] if n > 1 else dev(x) for x in xs],
                                (db[1:] if n > 1 else db) if with_base else None))[0]
    want_u = max(host(o.absmax(dev(x)[1:] if n > 1 else dev(x),
                               (db[1:] if n > 1 else db) if with_base else None))[0] for x in xs)
    assert got_u.view(np.uint32) == np.float32(want_u).view(np.uint32)


def test_absmax_unaligned_view_and_finite_pick():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(10_001) * 5).astype(np.float32)
    x[5000] = -123.25
    got = host(ops().absmax(dev(x)[1:]))[0]
    assert got == np.float32(123.25)


@pytest.mark.parametrize("W", [2, 8])
def test_combine_ina_auto_scale_never_saturates(W):
    """k="auto": the scale from the deltas' absmax keeps every quantised delta and the W-way
    integer sum inside int32, and the update equals the oracle's at that k."""
    from ina_amd import ps
    rng = np.random.default_rng(W)
    n = 40_000
    local = rng.standard_normal(n).astype(np.float32)
    paras = [(local + rng.standard_normal(n).astype(np.float32) * 10.0 ** rng.uniform(-4, 4)).astype(np.float32)
             for _ in range(W)]
    deltas = [(p - local).astype(np.float32) for p in paras]
    amax = max(float(np.abs(d).max()) for d in deltas)
    k = ops().scale_for(amax, W)
    qs = [orc.quantize_i32(d, k) for d in deltas]
    wide = np.sum([q.astype(np.int64) for q in qs], axis=0)
    assert np.abs(wide).max() <= 2**31 - 1                      # no wrap at this k
    assert all(np.abs(q.astype(np.int64)).max() < 2**31 - 1 for q in qs)
    got = host(ps.combine_ina(dev(local), [dev(p) for p in paras], "auto", 1.0 / (W + 1)))
    d = orc.dequantize_i32(orc.sum_reduce_i32(qs), k)
    want = (local + (d * np.float32(1.0 / (W + 1))).astype(np.float32)).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert k == ops().scale_for_workers([dev(p) for p in paras], base=dev(local))


def test_ps_apply_ina_update():
    rng = np.random.default_rng(12)
    n, W, k = 50_001, 4, 16
    local = rng.standard_normal(n).astype(np.float32)
    paras = [(local + rng.standard_normal(n).astype(np.float32) * 1e-2) for _ in range(W)]
    deltas = [dev(p - local) for p in paras]
    s = ops().quantize_reduce(deltas, k)
    out = host(ops().ps_apply(dev(local), s, k, 1.0 / (W + 1)))
    d = orc.dequantize_i32(orc.quantize_reduce_i32([p - local for p in paras], k), k)
    want = (local + (d * np.float32(1.0 / (W + 1))).astype(np.float32)).astype(np.float32)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))
    ref = orc.ps_combine_f32(local, paras, 1.0 / (W + 1))
    # quantisation error bound: W * 2^-(k+1) * weight (+ fp32 rounding of the combine)
    assert np.abs(out - ref).max() <= W * 2.0 ** -(k + 1) / (W + 1) + 4 * np.finfo(np.float32).eps * np.abs(ref).max()


# --------------------------------------------------------------------------------------
# packets
# --------------------------------------------------------------------------------------
# V = 100: a multiple of 4 that is not 4 x a power of two; "wide": 3 spare 16-byte
# chunks of padding per packet (the flat unpack must skip them)
@pytest.mark.parametrize("V", [32, 128, 256, 4, 1, 33, 100])
@pytest.mark.parametrize("n", [1, 31, 32, 33, 300, 8191])
@pytest.mark.parametrize("layout", ["padded", "tight", "wide"])
def test_pack_nga_matches_oracle(V, n, layout):
    o = ops()
    rng = np.random.default_rng(V * 7 + n)
    vals = rand_i32(rng, n)
    npk = -(-n // V)
    ovf = (rng.random(npk) < 0.3).astype(np.uint8)
    stride = {"padded": o.nga_stride(V), "tight": 15 + 4 * V, "wide": o.nga_stride(V) + 48}[layout]
    got = host(o.pack_nga(dev(vals), V, bitmap=0xDEADBEEF, count=8, switch_id=3, seq0=16380,
                          flags=0x11, stride=stride, overflow=dev(ovf)))
    want = orc.pack_nga(vals, V, 0xDEADBEEF, 8, 3, 16380, flags=0x11, stride=stride, ovf=ovf)
    assert np.array_equal(got, want)
    f, v = o.unpack_nga(dev(got), V, stride=stride)
    fo, vo = orc.unpack_nga(want, V, stride=stride)
    assert np.array_equal(host(v), vo)
    for key in fo:
        assert np.array_equal(host(f[key]).view(fo[key].dtype), fo[key]), key


@pytest.mark.parametrize("chunks", [65, 100, 7 * 65])
def test_flat_packet_kernels_split_launches(chunks):
    """Batches longer than one launch's chunk range (2^31 16-byte chunks) go in packet
    ranges; a small range forces the split here: pack, fused quantise+pack and unpack
    stay byte-exact with ragged last ranges and header sequence numbers carried over."""
    o = ops()
    rng = np.random.default_rng(chunks)
    V, n = 256, 256 * 37 + 19
    vals = rand_i32(rng, n)
    x = mixed_floats(rng, n)
    npk = -(-n // V)
    ovf = (rng.random(npk) < 0.5).astype(np.uint8)
    try:
        o.set_tuning(launch_chunks=chunks)
        pk = host(o.pack_nga(dev(vals), V, 5, 8, 1, 4000, overflow=dev(ovf)))
        qp = host(o.quantize_pack_nga(dev(x), 12, V, 5, 8, 1, 4000))
        f, v = o.unpack_nga(dev(pk), V)
        v = host(v)
    finally:
        o.set_tuning(launch_chunks=2**31 - 1)
    st = o.nga_stride(V)
    assert np.array_equal(pk, orc.pack_nga(vals, V, 5, 8, 1, 4000, ovf=ovf, stride=st))
    assert np.array_equal(qp, orc.pack_nga(orc.quantize_i32(x, 12), V, 5, 8, 1, 4000, stride=st))
    assert np.array_equal(v, np.concatenate([vals, np.zeros(npk * V - n, np.int32)]))
    fo, _ = orc.unpack_nga(pk, V, stride=st)
    for key in fo:
        assert np.array_equal(host(f[key]).view(fo[key].dtype), fo[key]), key


@pytest.mark.parametrize("case", manifest("nga_cases.json"), ids=lambda c: c["name"])
def test_pack_nga_matches_reference_datagrams(case):
    """Device packets == the datagrams DataManager._send_data emitted (same int payload)."""
    q, pkts = load_capture(case["file"])
    seq0 = {"send_data": 1, "fast_send_data": 0, "_send_data_end": 5}[case["entry"]]
    data = [p for p in pkts if len(p) == 143]
    got = host(ops().pack_nga(dev(q), 32, case["worker_id"], case["degree"], case["switch_id"],
                              seq0))
    assert len(got) == len(data)
    for g, p in zip(got, data):
        assert g[:143].tobytes() == p and not g[143:].any()


@pytest.mark.parametrize("case", manifest("c128_cases.json"), ids=lambda c: c["name"])
def test_pack_c128_matches_reference_bytes(case):
    data, pkts = load_capture(case["file"])
    if case["kind"] == "wrapper":
        args = (case["packet_num"], case["worker_id"], case["aggregator_index"], case["tensor_index"])
    elif case["kind"] == "single":
        args = (len(data) // 128, 0, 0, 0)
    else:
        pytest.skip("thread fan-out compared in test_oracle_golden (host-side split)")
    g = dev(data.view(np.int32))
    got = host(ops().pack_c128(g, *args))
    assert got.tobytes() == b"".join(pkts)


@pytest.mark.parametrize("packet_num", [1, 2, 3, 7, 1000, 199_665])
@pytest.mark.parametrize("offset", [0, 4, 12])
def test_pack_c128_paths_vs_oracle(packet_num, offset):
    """C-128 packing into 16-byte aligned buffers (4 words per thread, one 16-byte store)
    and into 4-byte aligned ones (a word per thread) equals the oracle's communicator.cc
    restatement, ragged word counts (131 * packet_num) and ResNet-50's packet count included."""
    rng = np.random.default_rng(packet_num + offset)
    g = rng.integers(0, 1 << 32, packet_num * 128, dtype=np.uint32)
    want = orc.pack_c128(g, packet_num, 3, 7, 10)
    buf = torch.zeros(packet_num * 524 + 16, dtype=torch.uint8, device=DEV)
    out = buf[offset: offset + packet_num * 524].view(packet_num, 524)
    got = host(ops().pack_c128(dev(g.view(np.int32)), packet_num, 3, 7, 10, out=out))
    assert np.array_equal(got.reshape(-1), np.asarray(want, np.uint8).reshape(-1))


def test_send_gradients_fd_over_socketpair():
    """The host send path (legacy send_gradients body) delivers exactly the reference's
    packet_t datagrams, one per packet, over a datagram socket."""
    from ina_amd import _lib
    data, pkts = load_capture("c128_w3_agg7_t10.bin")
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        arr = np.ascontiguousarray(data)
        rc = _lib.load().ina_send_gradients_fd(a.fileno(), arr.ctypes.data, 3, 0, 3, 7, 10)
        assert rc == 3
        got = [b.recv(2048) for _ in range(3)]
    finally:
        a.close()
        b.close()
    assert got == pkts


# --------------------------------------------------------------------------------------
# device packet-stream switch vs the oracle's P4 restatement
# --------------------------------------------------------------------------------------
def make_stream(rng, V, nslots_used, W, num_slots, collide=0.05, ack=0.1, other=0.05, stride=None,
                idx_hi=None):
    pk = []
    for s in range(nslots_used):
        frag = int(rng.integers(0, 4)) if rng.random() < 0.1 else 1000 + s
        deg = int(rng.choice([W, W, W, 1, 0, 2]))
        idx = int(rng.integers(0, idx_hi or num_slots * 2))
        for w in range(W):
            vals = rand_i32(rng, V)
            f = frag if rng.random() > collide else frag + 1
            flags = orc.FLAG_ACK if rng.random() < ack else 0
            sw = 2 if rng.random() < other else 1
            p = orc.pack_nga(vals, V, w + 1, deg, sw, 0, flags=flags,
                             stride=stride or ops().nga_stride(V))[0].copy()
            p[6:10] = np.frombuffer(idx.to_bytes(4, "big"), np.uint8)
            p[11:15] = np.frombuffer(f.to_bytes(4, "big"), np.uint8)
            pk.append(p)
    pk = np.stack(pk)
    return pk[rng.permutation(len(pk))] if rng.random() < 0.5 else pk


# (V, num_slots, W, slots used per batch, stride): multi-chunk batches (> 1024 packets),
# 1-3 digit passes of the slot sort (num_slots 4 .. 2^18), segments longer than a wave
# (small pools), and the LDS-staged path (V % 4 != 0 or a stride that is not 16-aligned)
SWITCH_CASES = [(32, 16384, 4, 60, None), (32, 64, 8, 60, None), (256, 128, 3, 60, None),
                (128, 16, 16, 60, None), (32, 4096, 8, 300, None), (64, 1 << 18, 4, 400, None),
                (32, 4, 16, 40, None), (33, 256, 4, 60, None), (32, 512, 4, 80, 143),
                (256, 1024, 8, 200, None)]


@pytest.mark.parametrize("write_dropped", [True, False])
@pytest.mark.parametrize("V,num_slots,W,used,stride", SWITCH_CASES)
def test_switch_stream_matches_oracle(V, num_slots, W, used, stride, write_dropped):
    rng = np.random.default_rng(V + num_slots + W + used)
    o = ops()
    stride = stride or o.nga_stride(V)
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for rnd in range(3):                  # state persists across batches
        stream = make_stream(rng, V, used, W, num_slots, stride=stride)
        want_pk, want_act = sw_orc.run(stream, stride=stride)
        d = dev(stream)
        act = sw_dev.process(d)
        assert np.array_equal(host(act), want_act), rnd
        got_pk = host(d)
        if write_dropped:
            assert np.array_equal(got_pk, want_pk), rnd
        else:   # forwarded packets exact; dropped ones left as they arrived
            fwd = want_act != orc.ACT_DROP
            assert np.array_equal(got_pk[fwd], want_pk[fwd]), rnd
            assert np.array_equal(got_pk[~fwd], stream[~fwd]), rnd
        cnt, frag, regs = sw_orc.registers()
        assert np.array_equal(host(sw_dev.count), cnt)
        assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
        assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


@pytest.mark.parametrize("seed", range(16))
def test_switch_fuzz_vs_oracle(seed):
    """Randomised configurations: V (incl. the LDS-staged path for V % 4 != 0 or unaligned
    strides), pool size (1..2^18 slots: 1-3 sort passes, long segments in small pools),
    worker count, collision / ack / foreign-switch rates, write_dropped, 2-4 batches with
    the switch state carried over -- bit-exact actions, packets and registers."""
    rng = np.random.default_rng(90_000 + seed)
    o = ops()
    V = int(rng.choice([4, 8, 32, 64, 100, 128, 256, 33, 7]))
    num_slots = int(rng.choice([1, 3, 64, 1000, 16384, 1 << 17, (1 << 18) - 5]))
    W = int(rng.integers(1, 21))
    used = int(rng.integers(1, 120))
    layout = rng.choice(["padded", "tight", "wide"])
    stride = {"padded": o.nga_stride(V), "tight": 15 + 4 * V, "wide": o.nga_stride(V) + 32}[layout]
    wd = bool(rng.integers(0, 2))
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=wd)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for rnd in range(int(rng.integers(2, 5))):
        stream = make_stream(rng, V, used, W, num_slots, collide=float(rng.uniform(0, 0.3)),
                             ack=float(rng.uniform(0, 0.3)), other=float(rng.uniform(0, 0.2)),
                             stride=stride)
        want_pk, want_act = sw_orc.run(stream, stride=stride)
        d = dev(stream)
        act = sw_dev.process(d)
        assert np.array_equal(host(act), want_act), (seed, rnd)
        got_pk = host(d)
        if wd:
            assert np.array_equal(got_pk, want_pk), (seed, rnd)
        else:
            fwd = want_act != orc.ACT_DROP
            assert np.array_equal(got_pk[fwd], want_pk[fwd]), (seed, rnd)
            assert np.array_equal(got_pk[~fwd], stream[~fwd]), (seed, rnd)
    cnt, frag, regs = sw_orc.registers()
    assert np.array_equal(host(sw_dev.count), cnt)
    assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
    assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


# slot sort variants: (sort 0 = auto: chunk + bucket for keys of one or two digits / 3 = the
# LSD digit passes, descriptors, chunk rounds)
SORT_VARIANTS = [(3, True, 0, 0), (3, False, 0, 0), (0, False, 4, 0), (0, True, 16, 0), (0, False, 8, 0),
                 (0, True, 0, 0), (0, False, 0, 0), (3, True, 8, 0), (0, True, 0, 8), (0, False, 16, 8)]


@pytest.mark.parametrize("variant", SORT_VARIANTS)
@pytest.mark.parametrize("seed", range(8))
def test_switch_sort_paths_vs_oracle(seed, variant):
    """Batches above the one-workgroup size (> 2,048 packets) through each slot sort --
    the chunk + bucket sort (the default for pools of < 2^18 slots; chunks of 1,024 / 2,048
    / 4,096 packets; keys from the packet headers or from the batch's descriptors) and the
    LSD histogram / column-scan / scatter digit passes -- bit-exact against the P4
    restatement, state carried across batches, pools of 1 .. 2^18 slots (keys of 1-3 digits)."""
    sort, use_desc, rounds, tile = variant
    rng = np.random.default_rng(40_000 + seed)
    o = ops()
    V = int(rng.choice([4, 32, 64, 256, 33]))
    num_slots = int(rng.choice([1, 64, 1000, 16384, 1 << 17, (1 << 18) - 5]))
    W = int(rng.integers(1, 17))
    stride = o.nga_stride(V) if rng.random() < 0.7 else 15 + 4 * V
    wd = bool(rng.integers(0, 2))
    o.set_tuning(switch_sort=sort, switch_sort_rounds=rounds, switch_bucket_tile=tile)
    try:
        sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=wd)
        sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
        for rnd in range(3):
            used = int(rng.integers(2100 // W + 1, 9000 // W + 2))
            stream = make_stream(rng, V, used, W, num_slots, collide=float(rng.uniform(0, 0.2)),
                                 ack=float(rng.uniform(0, 0.3)), other=float(rng.uniform(0, 0.1)),
                                 stride=stride)
            assert stream.shape[0] > 2048
            want_pk, want_act = sw_orc.run(stream, stride=stride)
            d = dev(stream)
            desc = o.nga_descriptors(d) if use_desc else None
            act = sw_dev.process(d, desc=desc)
            assert np.array_equal(host(act), want_act), (seed, rnd)
            got_pk = host(d)
            if wd:
                assert np.array_equal(got_pk, want_pk), (seed, rnd)
            else:
                fwd = want_act != orc.ACT_DROP
                assert np.array_equal(got_pk[fwd], want_pk[fwd]), (seed, rnd)
                assert np.array_equal(got_pk[~fwd], stream[~fwd]), (seed, rnd)
        cnt, frag, regs = sw_orc.registers()
        assert np.array_equal(host(sw_dev.count), cnt)
        assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
        assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)
    finally:
        o.set_tuning(switch_sort=0, switch_sort_rounds=0, switch_bucket_tile=0)


@pytest.mark.parametrize("sort,tile", [(3, 0), (0, 0), (0, 8)])
@pytest.mark.parametrize("case", ["one_bucket", "one_slot", "two_buckets", "foreign_heavy"])
def test_switch_skewed_buckets_vs_oracle(sort, tile, case):
    """Slot use concentrated in one or two sort buckets (2^8 consecutive slots of a 2^17
    pool), so a bucket holds more than one 4,096-item tile and the chunk + bucket sort takes
    its multi-tile path (a counting sweep, then the tiles in order); one case puts every
    packet in ONE slot (a segment of > 4,096 packets), one is 70 % foreign packets (their
    bucket is left unsorted at the end and the run kernel stops before it).  Bit-exact against the P4
    restatement with state carried across batches, for the bucket sort and the digit passes."""
    rng = np.random.default_rng({"one_bucket": 1, "one_slot": 2, "two_buckets": 3, "foreign_heavy": 4}[case])
    o = ops()
    V, num_slots, W = 32, 1 << 17, 16
    idx_hi = {"one_bucket": 256, "one_slot": 1, "two_buckets": 512, "foreign_heavy": None}[case]
    other = 0.7 if case == "foreign_heavy" else 0.05      # packets for another switch
    o.set_tuning(switch_sort=sort, switch_bucket_tile=tile)
    try:
        sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=True)
        sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
        for rnd in range(2):
            stream = make_stream(rng, V, 700, W, num_slots, collide=0.05, ack=0.05, other=other,
                                 idx_hi=idx_hi)
            assert stream.shape[0] > 2 * 4096
            want_pk, want_act = sw_orc.run(stream, stride=o.nga_stride(V))
            d = dev(stream)
            act = sw_dev.process(d)
            assert np.array_equal(host(act), want_act), rnd
            assert np.array_equal(host(d), want_pk), rnd
        cnt, frag, regs = sw_orc.registers()
        assert np.array_equal(host(sw_dev.count), cnt)
        assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
        assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)
    finally:
        o.set_tuning(switch_sort=0, switch_bucket_tile=0)


@pytest.mark.parametrize("num_slots", [513, 1023, 1024, 4097, 65536, (1 << 18) - 1])
def test_switch_bucket_sort_pool_edges(num_slots):
    """Pool sizes at the bucket sort's digit-split edges (2^9+1 .. 2^18-1 slots: high / low
    digits of 5..9 bits, pools that are and are not a multiple of the bucket width, i.e.
    with and without the unsorted foreign-only bucket), 30 % foreign packets and PS acks:
    the chunk + bucket sort and the LSD digit passes both bit-exact against the P4 restatement."""
    o = ops()
    V, W = 32, 8
    res = {}
    for sort in (0, 3):
        rng = np.random.default_rng(num_slots)
        o.set_tuning(switch_sort=sort)
        try:
            sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV)
            sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
            for rnd in range(2):
                stream = make_stream(rng, V, 600, W, num_slots, collide=0.05, ack=0.1, other=0.3)
                assert stream.shape[0] > 2048
                want_pk, want_act = sw_orc.run(stream, stride=o.nga_stride(V))
                d = dev(stream)
                act = sw_dev.process(d, desc=o.nga_descriptors(d))
                assert np.array_equal(host(act), want_act), (sort, rnd)
                fwd = want_act != orc.ACT_DROP
                assert np.array_equal(host(d)[fwd], want_pk[fwd]), (sort, rnd)
            cnt, frag, regs = sw_orc.registers()
            assert np.array_equal(host(sw_dev.count), cnt)
            assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
            assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)
        finally:
            o.set_tuning(switch_sort=0)


def _slot_keys(stream, num_slots, switch_id=1):
    """The sort key of every packet (slot, or num_slots for another switch's)."""
    idx = stream[:, 6:10].copy().view(">u4").reshape(-1).astype(np.int64)
    return np.where(stream[:, 10] == switch_id, idx % num_slots, num_slots)


PRESORTED_CASES = ["sorted", "descent_in_round", "descent_at_round", "descent_at_wave",
                   "descent_at_chunk", "descent_at_end", "foreign_in_middle", "equal_keys"]


@pytest.mark.parametrize("rounds,use_desc", [(0, True), (16, False), (16, True)])
@pytest.mark.parametrize("case", PRESORTED_CASES)
def test_switch_presorted_batches_vs_oracle(case, rounds, use_desc):
    """Batches already in slot order (a NIC's round-robin interleave of workers sending in
    lockstep) take the chunk sort's fast path: A finds no key below its predecessor and B
    only copies A's output.  One descent anywhere -- inside a 64-packet round, at a round
    edge (lane 0 reads the previous round's lane 63), at a wave or chunk edge (the loaded
    predecessor), at the last packet, or another switch's packets in the middle -- must take
    the full sort.  Bit-exact against the P4 restatement, state carried across batches, with
    collisions, acks and degree-1 slots in the stream.  rounds 0: 1,024-packet chunks, one
    64-packet round per wave; 16: 4,096-packet chunks, four rounds per wave."""
    rng = np.random.default_rng(1000 * PRESORTED_CASES.index(case) + rounds + use_desc)
    o = ops()
    V, W, num_slots = 32, 8, 1 << 17
    o.set_tuning(switch_sort_rounds=rounds)
    try:
        _presorted_batches(o, rng, case, use_desc, V, W, num_slots)
    finally:
        o.set_tuning(switch_sort_rounds=0)


@pytest.mark.parametrize("case", ["sorted", "descent_at_chunk", "foreign_in_middle"])
def test_switch_presorted_batches_generic_run_kernel(case):
    """The in-order fast path when the generic (LDS-staged) run kernel takes the batch (V =
    33: not a multiple of 4): the bucket pass then copies the chunk pass's output into the
    arrays that kernel reads."""
    rng = np.random.default_rng(77 + PRESORTED_CASES.index(case))
    o = ops()
    _presorted_batches(o, rng, case, False, 33, 8, 1 << 17)


def _presorted_batches(o, rng, case, use_desc, V, W, num_slots):
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=True)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for rnd in range(2):
        stream = make_stream(rng, V, 1300, W, num_slots, collide=0.05, ack=0.1,
                             other=0.1 if case == "foreign_in_middle" else 0.05)
        if case == "equal_keys":                        # every packet in a handful of slots
            stream[:, 6:10] = np.frombuffer(np.repeat(np.arange(5, dtype=">u4"),
                                            -(-len(stream) // 5))[:len(stream)].tobytes(),
                                            np.uint8).reshape(-1, 4)
        keys = _slot_keys(stream, num_slots)
        stream = stream[np.argsort(keys, kind="stable")]
        n = len(stream)
        assert n > 8192
        at = {"descent_in_round": 4096 + 70 + 10, "descent_at_round": 4096 + 128,
              "descent_at_wave": 4096 + 256, "descent_at_chunk": 4096, "descent_at_end": n - 1}.get(case)
        if at is not None:          # the packet at `at` gets a key below its predecessor's
            if case == "descent_at_end":                # the smallest key moves to the end
                stream = np.concatenate([stream[1:], stream[:1]])
            else:                                       # a large key moves to at - 1
                stream = np.insert(np.delete(stream, n - 3, axis=0), at - 1, stream[n - 3], axis=0)
            k2 = _slot_keys(stream, num_slots)
            assert k2[at] < k2[at - 1] and (np.diff(k2) < 0).sum() == 1, case
        if case == "foreign_in_middle":                 # the foreign packets sit mid-batch
            k2 = _slot_keys(stream, num_slots)
            foreign = stream[k2 == num_slots]
            mine = stream[k2 != num_slots]
            stream = np.concatenate([mine[: len(mine) // 2], foreign, mine[len(mine) // 2:]])
        want_pk, want_act = sw_orc.run(stream, stride=o.nga_stride(V))
        d = dev(stream)
        act = sw_dev.process(d, desc=o.nga_descriptors(d) if use_desc else None)
        assert np.array_equal(host(act), want_act), (case, rnd)
        assert np.array_equal(host(d), want_pk), (case, rnd)
    cnt, frag, regs = sw_orc.registers()
    assert np.array_equal(host(sw_dev.count), cnt)
    assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
    assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


@pytest.mark.parametrize("V,stride_kind", [(32, "padded"), (256, "padded"), (33, "tight"),
                                           (64, "tight"), (4, "padded")])
def test_pack_descriptors_are_header_bytes(V, stride_kind):
    """pack_nga / quantize_pack_nga desc output == ina_nga_descriptors == header bytes
    4..11 of each packet (byte 4 lowest), flat and generic pack paths alike."""
    o = ops()
    rng = np.random.default_rng(V)
    n = 97 * V + 3
    stride = o.nga_stride(V) if stride_kind == "padded" else 15 + 4 * V
    vals = dev(rand_i32(rng, n))
    pk, d = o.pack_nga(vals, V, 5, 3, 2, 4_000_000_000, flags=0x40, num_slots=1000, stride=stride,
                       desc=True)
    hb = host(pk)[:, 4:12].copy().view(np.int64).reshape(-1)
    assert np.array_equal(host(d), hb)
    assert np.array_equal(host(o.nga_descriptors(pk)), hb)
    x = dev(rng.standard_normal(n).astype(np.float32))
    pk2, d2 = o.quantize_pack_nga(x, 16, V, 2, 3, 1, 9, stride=stride, desc=True)
    assert np.array_equal(host(d2), host(pk2)[:, 4:12].copy().view(np.int64).reshape(-1))
    # per-slot overflow bits in the flags byte, and batches split into packet ranges
    ovf = dev((rng.random(-(-n // V)) < 0.5).astype(np.uint8))
    try:
        for chunks in (2**31 - 1, 3 * (stride // 16) + 1):
            o.set_tuning(launch_chunks=chunks)
            pk3, d3 = o.pack_nga(vals, V, 5, 3, 2, 4_000_000_000, num_slots=1000, stride=stride,
                                 overflow=ovf, desc=True)
            assert np.array_equal(host(d3), host(pk3)[:, 4:12].copy().view(np.int64).reshape(-1)), chunks
    finally:
        o.set_tuning(launch_chunks=2**31 - 1)


@pytest.mark.parametrize("write_dropped", [True, False])
@pytest.mark.parametrize("ack_fast", [True, False])
@pytest.mark.parametrize("W,ack", [(1, 0.5), (1, 1.0), (2, 0.4), (5, 0.3)])
def test_switch_lone_acks_vs_oracle(W, ack, ack_fast, write_dropped):
    """Radix-path batches (> 2,048 packets) full of short segments: a PS ack alone in its
    slot's segment takes the run kernel's lane-parallel path (its bit rides through the
    slot sort in the key), everything else the per-segment state machine; bit-exact
    against the oracle either way, with the switch state carried across batches."""
    rng = np.random.default_rng(7 * W + int(ack * 10) + ack_fast)
    o = ops()
    V, num_slots = 32, 8192
    stride = o.nga_stride(V)
    o.set_tuning(switch_ack_fast=ack_fast)
    try:
        sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
        sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
        for rnd in range(3):
            stream = make_stream(rng, V, 3000 // W + 1, W, num_slots, collide=0.05,
                                 ack=ack if rnd else 0.0, other=0.05, stride=stride)
            assert stream.shape[0] > 2048
            want_pk, want_act = sw_orc.run(stream, stride=stride)
            d = dev(stream)
            act = sw_dev.process(d)
            assert np.array_equal(host(act), want_act), rnd
            got = host(d)
            if write_dropped:
                assert np.array_equal(got, want_pk), rnd
            else:                 # forwarded packets exact; dropped ones left as they arrived
                fwd = want_act != orc.ACT_DROP
                assert np.array_equal(got[fwd], want_pk[fwd]), rnd
                assert np.array_equal(got[~fwd], stream[~fwd]), rnd
        cnt, frag, regs = sw_orc.registers()
        assert np.array_equal(host(sw_dev.count), cnt)
        assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
        assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)
    finally:
        o.set_tuning(switch_ack_fast=True)


@pytest.mark.parametrize("seed", range(6))
def test_switch_small_batch_paths_agree(seed):
    """Batches of <= 4096 packets through the three paths -- ONE launch of one workgroup
    (k_switch_tiny: LDS sort then the run kernel's work), the one-workgroup sort + run
    kernel (two launches), and the multi-launch slot sort -- give identical actions,
    packets and registers, all equal to the P4 restatement."""
    rng = np.random.default_rng(70_000 + seed)
    o = ops()
    V = int(rng.choice([32, 256, 33]))
    num_slots = int(rng.choice([3, 64, 16384, 1 << 17]))
    W = int(rng.integers(1, 17))
    used = int(rng.integers(1, 4096 // W + 1))
    stream = make_stream(rng, V, used, W, num_slots, stride=o.nga_stride(V))
    assert stream.shape[0] <= 4096
    want_pk, want_act = orc.Switch(V, num_slots=num_slots, switch_id=1).run(stream, stride=o.nga_stride(V))
    outs = []
    for small, tiny in ((2048, 2048), (2048, 0), (False, 0)):
        sw = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=True)
        d = dev(stream)
        try:
            o.set_tuning(switch_small_sort=small, switch_tiny_max=tiny)
            act = sw.process(d)
        finally:
            o.set_tuning(switch_small_sort=True, switch_tiny_max=128)
        outs.append((host(act), host(d), host(sw.regs)))
    for act, pk, regs in outs:
        assert np.array_equal(act, want_act) and np.array_equal(pk, want_pk)
    assert np.array_equal(outs[0][2], outs[1][2]) and np.array_equal(outs[0][2], outs[2][2])


@pytest.mark.parametrize("num_slots", [16384, 1 << 17])
def test_switch_state_across_batch_paths(num_slots):
    """One switch, one register state, a sequence of batches whose sizes walk across the
    default path thresholds (<= 128 packets: one launch; 129..768: one-workgroup sort +
    run kernel; above: the bucket sort) and back: every batch's actions and packets and
    the final registers equal the P4 restatement fed the same sequence."""
    rng = np.random.default_rng(num_slots)
    o = ops()
    V, W = 32, 8
    stride = o.nga_stride(V)
    sw_dev = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=True)
    sw_orc = orc.Switch(V, num_slots=num_slots, switch_id=1)
    for used in (10, 50, 500, 16, 17, 96, 97, 3000, 1, 200):     # x W = 8 packets per slot
        stream = make_stream(rng, V, used, W, num_slots, stride=stride, idx_hi=2 * 4096)
        assert stream.shape[0] == used * W
        want_pk, want_act = sw_orc.run(stream, stride=stride)
        d = dev(stream)
        act = sw_dev.process(d)
        assert np.array_equal(host(act), want_act), used
        assert np.array_equal(host(d), want_pk), used
    cnt, frag, regs = sw_orc.registers()
    assert np.array_equal(host(sw_dev.count), cnt)
    assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
    assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


def test_switch_collision_free_equals_bulk_reduce():
    """Stateful device switch over a full W-worker stream == the bulk sum-reduce."""
    rng = np.random.default_rng(77)
    o = ops()
    V, W, n = 256, 8, 256 * 500 + 17
    bufs = [rand_i32(rng, n) for _ in range(W)]
    sw = o.Switch(V, num_slots=16384, switch_id=1, device=DEV)
    stream = torch.cat([o.pack_nga(dev(b), V, w + 1, W, 1, 1) for w, b in enumerate(bufs)])
    act = host(sw.process(stream))
    npk = -(-n // V)
    done = np.nonzero(act == orc.ACT_FWD_AGG)[0]
    assert len(done) == npk and (done >= (W - 1) * npk).all()
    f, vals = o.unpack_nga(stream[torch.from_numpy(done).to(DEV)], V)
    order = np.argsort(host(f["frag_id"]))
    got = host(vals).reshape(npk, V)[order].reshape(-1)[:n]
    assert np.array_equal(got, host(o.sum_reduce([dev(b) for b in bufs])))


@pytest.mark.parametrize("V,n,pool", [(256, 26_214_400, 1 << 17), (32, 1_280_000, 1 << 16),
                                      (64, 1_600_000, 1 << 15)])
def test_switch_config3_full_size_equals_bulk_reduce(V, n, pool):
    """Config 3 at full size through the packet path: 8 workers x 26,214,400 int32 ->
    819,200 NGA-256 packets -> device switch (2^17-slot pool, multi-pass radix sort,
    windowed run kernel) -> the 102,400 completed packets, unpacked and ordered by frag id,
    equal the bulk W-way sum-reduce bit for bit (full-range values, so the sums wrap).
    The smaller cases take the sort's other chunk geometries (320,000 and 200,000 packets)."""
    o = ops()
    W = 8
    g = torch.Generator(device=DEV).manual_seed(31)
    bufs = [torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device=DEV, generator=g)
            for _ in range(W)]
    want = o.sum_reduce(bufs)
    # anchored to the oracle directly too: 4,099 slots' values summed on the host
    idx = np.unique(np.concatenate([np.arange(0, n // V, 97), [n // V - 1]]))
    cols = (idx[:, None] * V + np.arange(V)).ravel()
    tcols = torch.from_numpy(cols).to(DEV)
    host_want = orc.sum_reduce_i32([host(b[tcols]) for b in bufs])
    packed = [o.pack_nga(b, V, w + 1, W, 1, 1, num_slots=pool, desc=True) for w, b in enumerate(bufs)]
    stream = torch.cat([p for p, _ in packed])
    desc = torch.cat([d for _, d in packed])
    del bufs, packed
    sw = o.Switch(V, num_slots=pool, switch_id=1, device=DEV)
    act = sw.process(stream, desc=desc)
    npk = n // V
    done = torch.nonzero(act == orc.ACT_FWD_AGG).flatten()
    assert done.numel() == npk and bool((done >= (W - 1) * npk).all())
    f, vals = o.unpack_nga(stream[done], V)
    order = torch.argsort(f["frag_id"].to(torch.int64))
    got = vals.view(npk, V)[order].reshape(-1)
    assert torch.equal(got, want)
    assert np.array_equal(host(got[tcols]), host_want)


def test_switch_config3_full_size_shuffled_arrival():
    """Config 3 at full size in a random arrival order (as a NIC interleaves W workers):
    every slot completes, the completed sums equal the bulk W-way reduce bit for bit, and
    the packet that completes each slot is that slot's LAST arrival -- the slot sort
    (bucket + local) kept arrival order inside every slot across 819,200 packets."""
    o = ops()
    W, V, n, pool = 8, 256, 26_214_400, 1 << 17
    g = torch.Generator(device=DEV).manual_seed(37)
    bufs = [torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device=DEV, generator=g)
            for _ in range(W)]
    want = o.sum_reduce(bufs)
    cols = torch.arange(0, n, 9973, device=DEV)                      # oracle anchor: a strided sample
    host_want = orc.sum_reduce_i32([host(b[cols]) for b in bufs])
    packed = [o.pack_nga(b, V, w + 1, W, 1, 1, num_slots=pool, desc=True) for w, b in enumerate(bufs)]
    del bufs
    npk = n // V
    perm = torch.randperm(W * npk, device=DEV, generator=g)
    stream = torch.cat([p for p, _ in packed])[perm]
    desc = torch.cat([d for _, d in packed])[perm]
    del packed
    sw = o.Switch(V, num_slots=pool, switch_id=1, device=DEV)
    act = sw.process(stream, desc=desc)
    done = torch.nonzero(act == orc.ACT_FWD_AGG).flatten()
    assert done.numel() == npk
    slot_of = perm % npk                                  # original packet i: slot i mod npk
    last = torch.full((npk,), -1, dtype=torch.int64, device=DEV)
    last.scatter_reduce_(0, slot_of, torch.arange(W * npk, device=DEV), reduce="amax")
    assert torch.equal(torch.sort(done).values, torch.sort(last).values)
    f, vals = o.unpack_nga(stream[done], V)
    order = torch.argsort(f["frag_id"].to(torch.int64))
    got = vals.view(npk, V)[order].reshape(-1)
    assert torch.equal(got, want)
    assert np.array_equal(host(got[cols]), host_want)


@pytest.mark.parametrize("extra", [0, 1])
def test_switch_bucket_rows_limit_equals_digit_passes(extra):
    """The chunk + bucket sort takes batches of up to 2,048 chunks (8,388,608 packets at
    4,096-packet chunks; its bucket kernel's LDS rows), larger batches the LSD digit
    passes.  At the limit and one packet past it, V = 4 packets of 8 workers into a 2^17-
    slot pool (slots reused across the batch: collisions and in-batch completions): the
    default sort and the digit passes (tuning key 12 = 3, itself oracle-tested above) give
    identical actions, packets and registers."""
    o = ops()
    W, V, pool = 8, 4, 1 << 17
    npk = 2048 * 4096 + extra
    per = -(-npk // W)
    g = torch.Generator(device=DEV).manual_seed(5 + extra)
    vals = torch.randint(-(1 << 31), (1 << 31) - 1, (W, per * V), dtype=torch.int32, device=DEV, generator=g)
    stream = torch.cat([o.pack_nga(vals[w], V, w + 1, W, 1, 1, num_slots=pool) for w in range(W)])[:npk]
    del vals
    res = []
    for sort in (0, 3):
        o.set_tuning(switch_sort=sort)
        try:
            sw = o.Switch(V, num_slots=pool, switch_id=1, device=DEV, write_dropped=True)
            pk = stream.clone()
            act = sw.process(pk)
            torch.cuda.synchronize()
            res.append((act, pk, sw.count, sw.frag, sw.regs))
        finally:
            o.set_tuning(switch_sort=0)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    assert int((res[0][0] == orc.ACT_FWD_AGG).sum()) > 0


@pytest.mark.parametrize("keep", [True, False])
@pytest.mark.parametrize("V,W,per,tail", [(32, 4, 60, 11), (256, 8, 700, 0), (32, 3, 3000, 5),
                                          (64, 16, 200, 37), (32, 2, 30, 3), (256, 3, 30, 0)])   # last two: <= 128-packet batches (one launch)
def test_switch_process_apply_equals_two_steps(V, W, per, tail, keep):
    """ina_switch with a PS step (the PS on the switch's GPU) == ina_switch_process then
    ina_apply_completed_nga: same actions, switch registers, parameter update (bit for bit)
    and PS ack rows, over two steps with the acks riding in front of the second step's
    packets; keep_forwarded=False leaves completed packets as they arrived."""
    rng = np.random.default_rng(V * W + per + keep)
    o = ops()
    n = V * per - tail
    npk = -(-n // V)
    stride = o.nga_stride(V)
    local = dev(rng.standard_normal(n).astype(np.float32))
    res = {}
    for fused in (False, True):
        big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=DEV)
        acks, rows = big[:npk], big[npk:].view(W, npk, stride)
        sw = o.Switch(V, num_slots=1 << 13, switch_id=1, device=DEV)
        g = np.random.default_rng(5)
        outs = []
        for step in range(2):
            for w in range(W):
                o.pack_nga(dev(rand_i32(g, n, full=False)), V, w + 1, W, 1, 7, num_slots=1 << 13,
                           out=rows[w])
            before = host(big).copy()
            out = torch.full_like(local, float("nan"))
            if fused:
                act, _ = sw.process_apply(big, 7, local, 16, 0.25, out=out, acks=acks, keep_forwarded=keep)
            else:
                act = sw.process(big)
                o.apply_completed(big, act, V, 7, local, 16, 0.25, out=out, acks=acks)
            a = host(act)
            pk = host(big)
            if fused and not keep:
                done = a == orc.ACT_FWD_AGG
                assert done.sum() > 0 and np.array_equal(pk[done], before[done])
            outs.append((a, pk[:npk].copy(), host(out).view(np.uint32), pk if keep or not fused else None))
        res[fused] = (outs, host(sw.count), host(sw.frag), host(sw.regs))
    (o0, c0, f0, r0), (o1, c1, f1, r1) = res[False], res[True]
    for (a0, k0, u0, p0), (a1, k1, u1, p1) in zip(o0, o1):
        assert np.array_equal(a0, a1)
        assert np.array_equal(k0, k1)                 # PS ack rows
        assert np.array_equal(u0, u1)                 # parameter update, bit for bit
        if p1 is not None:
            assert np.array_equal(p0, p1)
    assert np.array_equal(c0, c1) and np.array_equal(f0, f1) and np.array_equal(r0, r1)


@pytest.mark.parametrize("sort_mode", [0, 3])
@pytest.mark.parametrize("V,W,per,order", [(256, 8, 700, "worker"), (256, 8, 700, "round_robin"),
                                           (32, 4, 3000, "shuffled"), (256, 3, 30, "worker"),
                                           (32, 4, 150, "worker"), (64, 16, 200, "shuffled")])
def test_switch_two_phase_equals_one_call(V, W, per, order, sort_mode):
    """ina_switch (INA_SWITCH_SORT) queued on a side stream from descriptors made from the header
    fields alone (ina_nga_make_descriptors + the ack rows' descriptors), BEFORE the packets'
    payload is packed on the main stream, then ina_switch (INA_SWITCH_RUN + PS step) after both ==
    ina_switch (descriptors + PS step) on the packed batch: same actions, PS update (bit for bit),
    ack rows and switch state over two steady-state steps.  Covers the bucket sort, the
    digit passes (sort_mode 3), presorted batches and the one-workgroup small-batch paths
    (<= 768 and <= 128 packets, which sort inside the run call)."""
    rng = np.random.default_rng(V * W + per)
    o = ops()
    n = V * per - 5
    npk = -(-n // V)
    stride = o.nga_stride(V)
    slots = 1 << 13
    xs = [dev((rng.standard_normal(n) * 1e-2).astype(np.float32)) for _ in range(W)]
    glob0 = rng.standard_normal(n).astype(np.float32) * 1e-2
    perm = None
    if order == "round_robin":
        perm = torch.arange(W * npk, device=DEV).view(W, npk).t().reshape(-1)
    elif order == "shuffled":
        perm = torch.randperm(W * npk, device=DEV)
    res = {}
    side = torch.cuda.Stream(DEV)
    try:
        o.set_tuning(switch_sort=sort_mode)
        for two in (False, True):
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
            for step in range(2):
                if two:
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        o.make_descriptors(npk, W, W, 1, 1, num_slots=slots, outs=list(wdesc.unbind(0)),
                                           device=DEV)
                        o.nga_descriptors(acks, out=desc[:npk])
                        desc[npk:] = wdesc.reshape(-1) if perm is None else wdesc.reshape(-1)[perm]
                        sw.sort(big, desc, actions=acts)
                    o.quantize_pack_nga_multi(xs, 16, V, list(range(1, W + 1)), W, 1, 1, base=glob,
                                              num_slots=slots, outs=list(wrows.unbind(0)))
                    rows.view(W * npk, stride)[:] = wrows.view(W * npk, stride) if perm is None \
                        else wrows.view(W * npk, stride)[perm]
                    torch.cuda.current_stream().wait_stream(side)
                    sw.run_apply(big, acts, 1, glob, 16, 1.0 / (W + 1), out=upd, acks=acks,
                                 keep_forwarded=False)
                else:
                    o.quantize_pack_nga_multi(xs, 16, V, list(range(1, W + 1)), W, 1, 1, base=glob,
                                              num_slots=slots, outs=list(wrows.unbind(0)),
                                              descs=list(wdesc.unbind(0)))
                    rows.view(W * npk, stride)[:] = wrows.view(W * npk, stride) if perm is None \
                        else wrows.view(W * npk, stride)[perm]
                    o.nga_descriptors(acks, out=desc[:npk])
                    desc[npk:] = wdesc.reshape(-1) if perm is None else wdesc.reshape(-1)[perm]
                    sw.process_apply(big, 1, glob, 16, 1.0 / (W + 1), out=upd, acks=acks,
                                     keep_forwarded=False, actions=acts, desc=desc)
                steps.append((host(acts).copy(), host(upd).view(np.uint32).copy(), host(acks).copy()))
                glob.copy_(upd)
            res[two] = (steps, host(sw.count), host(sw.frag), host(sw.regs))
    finally:
        o.set_tuning(switch_sort=0)
    (s0, c0, f0, r0), (s1, c1, f1, r1) = res[False], res[True]
    for (a0, u0, k0), (a1, u1, k1) in zip(s0, s1):
        assert np.array_equal(a0, a1)
        assert np.array_equal(u0, u1)
        assert np.array_equal(k0, k1)
    assert int((s1[1][0] == orc.ACT_FWD_AGG).sum()) == npk        # every slot completed
    assert np.array_equal(c0, c1) and np.array_equal(f0, f1) and np.array_equal(r0, r1)


def test_switch_run_requires_its_sort():
    """run() reads the scratch its sort() left: without that sort, for another batch, or
    after a one-call process() reused the scratch, it refuses before any launch."""
    o = ops()
    V, W, n = 32, 4, 32 * 3000
    pk = [o.pack_nga(dev(rand_i32(np.random.default_rng(w), n, full=False)), V, w + 1, W, 1, 1,
                     num_slots=4096, desc=True) for w in range(W)]
    batch = torch.cat([p for p, _ in pk])
    desc = torch.cat([d for _, d in pk])
    sw = o.Switch(V, num_slots=4096, switch_id=1, device=DEV)
    acts = torch.empty(batch.shape[0], dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError):
        sw.run(batch, acts)
    sw.sort(batch, desc, actions=acts)
    with pytest.raises(ValueError):
        sw.run(batch[:-1], acts)
    sw.process(batch[:10].clone())
    with pytest.raises(ValueError):
        sw.run(batch, acts)
    sw.sort(batch, desc, actions=acts)
    sw.run(batch, acts)
    assert int((acts == orc.ACT_FWD_AGG).sum()) == n // V


def test_make_descriptors_equal_pack_descriptors():
    """Descriptors from the header fields alone == the ones the pack kernel writes."""
    o = ops()
    rng = np.random.default_rng(3)
    V, W, n = 256, 11, 256 * 40 + 9
    xs = [dev(mixed_floats(rng, n)) for _ in range(W)]
    seqs = [int(s) for s in rng.integers(0, 2**32 - 64, W)]
    _, d_pack = o.quantize_pack_nga_multi(xs, 16, V, list(range(W)), 5, 2, seqs, num_slots=777,
                                          flags=0x10, descs=True)
    d_made = o.make_descriptors(-(-n // V), W, 5, 2, seqs, flags=0x10, num_slots=777, device=DEV)
    for a, b in zip(d_pack, d_made):
        assert torch.equal(a, b)


@pytest.mark.parametrize("V,W,per", [(32, 4, 300), (256, 8, 70)])
def test_process_apply_packets_outside_the_bucket_are_forwarded(V, W, per):
    """keep_forwarded=False consumes only the completed packets the PS takes (frag_id -
    seq0 inside the bucket); a completed packet outside it is forwarded with its slot sum
    exactly as ina_switch_process forwards it (the fused kernel used to leave
    such packets as they arrived)."""
    o = ops()
    n = V * per
    stride = o.nga_stride(V)
    g = np.random.default_rng(V + W)
    q = [rand_i32(g, n, full=False) for _ in range(W)]
    half = per // 2
    seq_apply = 7 + half                    # packets 0..half-1 fall before the bucket
    local = dev(np.random.default_rng(1).standard_normal(n).astype(np.float32))
    res = {}
    for fused in (False, True):
        rows = torch.cat([o.pack_nga(dev(b), V, w + 1, W, 1, 7, num_slots=1 << 13) for w, b in enumerate(q)])
        before = host(rows).copy()
        sw = o.Switch(V, num_slots=1 << 13, switch_id=1, device=DEV)
        out = torch.full_like(local, float("nan"))
        if fused:
            act, _ = sw.process_apply(rows, seq_apply, local, 16, 0.25, out=out, keep_forwarded=False)
        else:
            act = sw.process(rows)
            o.apply_completed(rows, act, V, seq_apply, local, 16, 0.25, out=out)
        res[fused] = (host(act), host(rows).copy(), host(out).view(np.uint32), before)
    (a0, p0, u0, _), (a1, p1, u1, b1) = res[False], res[True]
    assert np.array_equal(a0, a1) and np.array_equal(u0, u1)
    done = np.nonzero(a1 == orc.ACT_FWD_AGG)[0]
    assert done.size == per
    frag = np.array([int.from_bytes(bytes(b1[p, 11:15]), "big") for p in done])
    inside = frag - seq_apply >= 0
    assert inside.sum() == per - half and (~inside).sum() == half
    assert np.array_equal(p1[done[inside]], b1[done[inside]])     # consumed: as they arrived
    assert np.array_equal(p1[done[~inside]], p0[done[~inside]])   # forwarded: slot sums
    assert not np.array_equal(p0[done[~inside]], b1[done[~inside]])


@pytest.mark.parametrize("V,W,per", [(32, 4, 3000), (256, 8, 700)])
def test_steady_state_acks_ride_with_next_step(V, W, per):
    """Steady-state packet path: step t's PS acks sit in front of step t+1's worker packets
    in ONE switch batch (the bench's steady-state row).  Every step the device switch
    equals the oracle's P4 restatement on the same bytes (actions, packets, registers):
    the acks free the slots (FWD_ACK) and the new packets complete them (FWD_AGG)."""
    rng = np.random.default_rng(V + W)
    o = ops()
    n = V * per
    stride = o.nga_stride(V)
    big = torch.zeros(((W + 1) * per, stride), dtype=torch.uint8, device=DEV)
    ack_rows, rows_w = big[:per], big[per:].view(W, per, stride)
    sw_dev = o.Switch(V, num_slots=1 << 13, switch_id=1, device=DEV, write_dropped=True)
    sw_orc = orc.Switch(V, num_slots=1 << 13, switch_id=1)
    local = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(DEV)
    for step in range(3):
        q = [dev(rand_i32(rng, n)) for _ in range(W)]
        for w in range(W):
            o.pack_nga(q[w], V, w + 1, W, 1, 1, num_slots=1 << 13, out=rows_w[w])
        stream = host(big).copy()
        want_pk, want_act = sw_orc.run(stream, stride=stride)
        act = sw_dev.process(big)
        assert np.array_equal(host(act), want_act), step
        assert np.array_equal(host(big), want_pk), step
        assert int((want_act[per:] == orc.ACT_FWD_AGG).sum()) == per
        assert (want_act[:per] == (orc.ACT_FWD_ACK if step else orc.ACT_FWD_OTHER)).all()
        o.apply_completed(big, act, V, 1, local, 16, 0.2, acks=ack_rows)
    cnt, frag, regs = sw_orc.registers()
    assert np.array_equal(host(sw_dev.count), cnt)
    assert np.array_equal(host(sw_dev.frag).view(np.uint32), frag)
    assert np.array_equal(host(sw_dev.regs).view(np.uint32), regs)


@pytest.mark.parametrize("V", [32, 256, 33, 100, 4])
@pytest.mark.parametrize("with_base", [False, True])
@pytest.mark.parametrize("padded", [True, False])
def test_quantize_pack_fused_matches_oracle(V, with_base, padded):
    """Worker side in one pass: packets of quantize(x - base) == oracle quantize then pack."""
    o = ops()
    rng = np.random.default_rng(V + 2 * with_base + padded)
    n = 77 * V + 5
    x = mixed_floats(rng, n)
    base = (rng.standard_normal(n) * 0.1).astype(np.float32) if with_base else None
    stride = o.nga_stride(V) if padded else 15 + 4 * V
    got = host(o.quantize_pack_nga(dev(x), 16, V, bitmap=3, count=4, switch_id=1, seq0=42,
                                   base=dev(base) if with_base else None, stride=stride))
    d = (x - base).astype(np.float32) if with_base else x
    want = orc.pack_nga(orc.quantize_i32(d, 16), V, 3, 4, 1, 42, stride=stride)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("V,W,with_base,padded", [
    (256, 8, True, True), (256, 8, False, True), (32, 3, True, True), (256, 13, True, True),
    (256, 1, True, True), (4, 5, True, True), (100, 2, True, True), (256, 17, True, True),
    (32, 4, True, False), (256, 2, False, False), (256, 3, True, "wide"), (256, 9, True, "wide")])
def test_quantize_pack_multi_matches_oracle(V, W, with_base, padded):
    """W workers' quantise + pack in one launch (groups of 8, per-worker bitmaps and
    sequence starts, descriptors) == the oracle's quantize then pack worker by worker;
    V = 256 takes the wave-per-packet kernel (wide strides: zeroed padding chunks), other
    V the flat chunk stream, unpadded strides the per-worker byte path; same bytes."""
    o = ops()
    rng = np.random.default_rng(1000 * V + W + 2 * with_base + (padded is True))
    n = 61 * V + 7                                  # ragged last packet
    xs = [mixed_floats(rng, n) for _ in range(W)]
    base = (rng.standard_normal(n) * 0.1).astype(np.float32) if with_base else None
    stride = {True: o.nga_stride(V), False: 15 + 4 * V, "wide": o.nga_stride(V) + 48}[padded]
    seqs = [int(s) for s in rng.integers(0, 2**32 - 100, W)]
    seqs[0] = 2**32 - 30                            # sequence numbers wrap inside the bucket
    outs, descs = o.quantize_pack_nga_multi([dev(x) for x in xs], 16, V, [w + 1 for w in range(W)],
                                            W, 1, seqs, base=dev(base) if with_base else None,
                                            num_slots=1000, stride=stride, descs=True)
    for w, x in enumerate(xs):
        d = (x - base).astype(np.float32) if with_base else x
        want = orc.pack_nga(orc.quantize_i32(d, 16), V, w + 1, W, 1, seqs[w], stride=stride,
                            num_slots=1000)
        got = host(outs[w])
        assert np.array_equal(got, want), w
        dw = host(descs[w]).view(np.uint8).reshape(-1, 8)
        assert np.array_equal(dw, want.reshape(-1, stride)[:, 4:12]), w


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257])
def test_quantize_pack_multi_tiny_buckets(n):
    """Empty and sub-packet buckets at the 64-worker maximum: zero packets, or one ragged
    packet per worker, byte-equal to the oracle."""
    o = ops()
    rng = np.random.default_rng(n + 1)
    V, W = 256, 64
    xs = [mixed_floats(rng, n) for _ in range(W)]
    outs = o.quantize_pack_nga_multi([dev(x) for x in xs], 16, V, list(range(W)), W, 3, 77)
    for w, x in enumerate(xs):
        got = host(outs[w])
        want = orc.pack_nga(orc.quantize_i32(x, 16), V, w, W, 3, 77, stride=o.nga_stride(V))
        assert got.size == want.size and np.array_equal(got.reshape(-1), want.reshape(-1)), w


def test_quantize_pack_multi_split_launches():
    """Packet ranges (a small launch_chunks forces them) carry every worker's sequence."""
    o = ops()
    rng = np.random.default_rng(7)
    V, W, n = 256, 9, 256 * 23 + 100
    xs = [mixed_floats(rng, n) for _ in range(W)]
    base = (rng.standard_normal(n) * 0.1).astype(np.float32)
    try:
        o.set_tuning(launch_chunks=65 * 5)
        outs = o.quantize_pack_nga_multi([dev(x) for x in xs], 12, V, [7] * W, 8, 2,
                                         [100 * w for w in range(W)], base=dev(base))
    finally:
        o.set_tuning(launch_chunks=2**31 - 1)
    for w, x in enumerate(xs):
        want = orc.pack_nga(orc.quantize_i32((x - base).astype(np.float32), 12), V, 7, 8, 2,
                            100 * w, stride=o.nga_stride(V))
        assert np.array_equal(host(outs[w]), want), w


@pytest.mark.parametrize("V,W", [(256, 8), (32, 3), (128, 4), (100, 5), (4, 2)])
def test_switch_then_fused_apply_matches_oracle(V, W):
    """PS side: device switch over W worker streams, then one fused kernel places,
    dequantises and applies the completed slots; its ack rows free every slot."""
    o = ops()
    rng = np.random.default_rng(V * W)
    n, k, seq0 = 60 * V + 11, 16, 5000
    local = rng.standard_normal(n).astype(np.float32)
    q = [rand_i32(rng, n, full=False) for _ in range(W)]
    stream = torch.cat([o.pack_nga(dev(b), V, w + 1, W, 1, seq0) for w, b in enumerate(q)])
    stream = stream[torch.randperm(stream.shape[0], device=stream.device)]
    sw = o.Switch(V, num_slots=16384, switch_id=1, device=DEV)
    act = sw.process(stream)
    npk = -(-n // V)
    acks = torch.zeros((npk, stream.shape[1]), dtype=torch.uint8, device=DEV)
    out = host(o.apply_completed(stream, act, V, seq0, dev(local), k, 1.0 / (W + 1), acks=acks))
    S = orc.sum_reduce_i32(q)
    want = (local + (orc.dequantize_i32(S, k) * np.float32(1.0 / (W + 1))).astype(np.float32)).astype(np.float32)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))
    assert (host(sw.frag)[(seq0 + np.arange(npk)) % 16384] != 0).all()
    ack_act = host(sw.process(acks))
    assert (ack_act == orc.ACT_FWD_ACK).all()
    assert not host(sw.frag).any()


def test_apply_wrappers_refuse_short_buffers():
    """Buffer sizes the C ABI cannot see are checked by the Python wrappers (a short ack
    table or action array would otherwise be an out-of-bounds device write)."""
    o = ops()
    V, n = 32, 32 * 10
    pk = torch.zeros((40, o.nga_stride(V)), dtype=torch.uint8, device=DEV)
    act = torch.zeros(40, dtype=torch.uint8, device=DEV)
    local = torch.zeros(n, device=DEV)
    with pytest.raises(ValueError, match="one row per slot"):
        o.apply_completed(pk, act, V, 1, local, 16, 0.5,
                          acks=torch.zeros((9, o.nga_stride(V)), dtype=torch.uint8, device=DEV))
    with pytest.raises(ValueError, match="one byte per packet"):
        o.apply_completed(pk, act[:39], V, 1, local, 16, 0.5)
    with pytest.raises(ValueError, match="local's size|needs"):
        o.apply_completed(pk, act, V, 1, local, 16, 0.5, out=torch.zeros(n - 1, device=DEV))
    sw = o.Switch(V, num_slots=64, switch_id=1, device=DEV)
    with pytest.raises(ValueError, match="one byte per packet"):
        sw.process(pk, act[:39])
    with pytest.raises(ValueError, match="one row per slot"):
        sw.process_apply(pk, 1, local, 16, 0.5,
                         acks=torch.zeros((9, o.nga_stride(V)), dtype=torch.uint8, device=DEV))


def test_sum_reduce_host_concurrent_threads():
    """ina_sum_reduce_host_i32 from several host threads at once (thread-local copy
    streams and ring events, one scratch per caller): every result exact."""
    import threading
    o = ops()
    rng = np.random.default_rng(21)
    jobs = []
    for t in range(3):
        W, n = 3 + t, 1_000_003 + 17 * t
        bufs = [torch.from_numpy(rand_i32(rng, n)).pin_memory() for _ in range(W)]
        jobs.append((bufs, orc.sum_reduce_i32([b.numpy() for b in bufs])))
    results, errors = [None] * len(jobs), []

    def work(i):
        try:
            results[i] = o.sum_reduce_host(jobs[i][0], chunk=1 << 18).numpy().copy()
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append(e)
    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(60)
    assert not errors, errors
    for (bufs, want), got in zip(jobs, results):
        assert got is not None and np.array_equal(got, want)
