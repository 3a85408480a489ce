"""Oracle quantiser (build-defined; the reference's float_to_int/int_to_float are
missing -- parity unpinned) checked against an independent numpy statement of
the same definition: q = saturate(round_half_even(x * 2^k)), NaN -> 0."""
import numpy as np
import pytest

from oracle import oracle as orc


def np_q32(x, k):
    with np.errstate(invalid="ignore", over="ignore"):
        y = np.rint(x.astype(np.float32) * np.float32(2.0 ** k)).astype(np.float64)
    y = np.where(np.isnan(y), 0, y)
    return np.clip(y, -2**31, 2**31 - 1).astype(np.int64).astype(np.int32)


def np_q16(x, k):
    with np.errstate(invalid="ignore", over="ignore"):
        y = np.rint(x.astype(np.float32) * np.float32(2.0 ** k)).astype(np.float64)
    sat = np.isnan(y) | (y > 32767) | (y < -32768)
    y = np.where(np.isnan(y), 0, y)
    return np.clip(y, -32768, 32767).astype(np.int16), sat


EDGE = np.array([0.0, -0.0, 0.5, 1.5, 2.5, -0.5, -1.5, 1e-45, -1e-45, 1e-38,
                 np.inf, -np.inf, np.nan, 3e38, -3e38, 32767.5, -32768.5, 32766.5,
                 2147483520.0, 2147483648.0, -2147483648.0, -2147483904.0], np.float32)


@pytest.mark.parametrize("k", [0, 1, 16, 20, -3])
def test_quantize_i32_matches_numpy(k):
    rng = np.random.default_rng(k + 50)
    x = np.concatenate([EDGE, (rng.standard_normal(10000) * 10.0 ** rng.integers(-6, 6, 10000))
                        .astype(np.float32), EDGE / np.float32(2.0 ** k)])
    assert np.array_equal(orc.quantize_i32(x, k), np_q32(x, k))


@pytest.mark.parametrize("V", [32, 256])
def test_quantize_i16_matches_numpy_and_flags(V):
    rng = np.random.default_rng(V)
    k = 10
    x = (rng.standard_normal(3 * V + 5) * 8).astype(np.float32)
    x[:len(EDGE)] = EDGE
    q, ovf = orc.quantize_i16_sat(x, k, V)
    qn, sat = np_q16(x, k)
    assert np.array_equal(q, qn)
    want = np.zeros(len(ovf), bool)
    for i in np.nonzero(sat)[0]:
        want[i // V] = True
    assert np.array_equal(ovf.astype(bool), want)


def test_dequantize_exact_power_of_two():
    s = np.array([0, 1, -1, 2**31 - 1, -2**31, 12345678, 2**24 + 1], np.int32)
    for k in (0, 16, 30):
        y = orc.dequantize_i32(s, k)
        want = (s.astype(np.float32) * np.float32(2.0 ** -k)).astype(np.float32)
        assert np.array_equal(y.view(np.uint32), want.view(np.uint32))


def test_round_trip_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(10000) * 0.01).astype(np.float32)
    k = 16
    y = orc.dequantize_i32(orc.quantize_i32(x, k), k)
    assert np.abs(y - x).max() <= 2.0 ** -(k + 1) * (1 + 1e-6)


def test_bad_k_rejected():
    with pytest.raises(ValueError):
        orc.quantize_i32(np.zeros(4, np.float32), 200)


def test_fused_quant_reduce_equals_composition():
    rng = np.random.default_rng(9)
    bufs = [(rng.standard_normal(4099) * 50).astype(np.float32) for _ in range(5)]
    k = 8
    want = orc.sum_reduce_i32([orc.quantize_i32(b, k) for b in bufs])
    assert np.array_equal(orc.quantize_reduce_i32(bufs, k), want)
    V = 128
    q16 = [orc.quantize_i16_sat(b, k, V) for b in bufs]
    s16, ovf_sum = orc.sum_reduce_i16_sat([q for q, _ in q16], V)
    f16, ovf = orc.quantize_reduce_i16_sat(bufs, k, V)
    assert np.array_equal(f16, s16)
    anyq = np.any([o for _, o in q16], axis=0)
    assert np.array_equal(ovf.astype(bool), anyq | ovf_sum.astype(bool))


@pytest.mark.parametrize("k", [0, 13, 16, -3])
def test_bench_spot_check_quantisers_match_oracle(k):
    """bench.py's C2 / C4 parity spot checks restate the quantiser in numpy; they must
    agree with the oracle on the edge values and random magnitudes."""
    import bench
    rng = np.random.default_rng(k + 70)
    x = np.concatenate([EDGE, (rng.standard_normal(5000) * 10.0 ** rng.integers(-6, 6, 5000))
                        .astype(np.float32), EDGE / np.float32(2.0 ** k)])
    assert np.array_equal(bench._np_q32(x, k), orc.quantize_i32(x, k).astype(np.int64))
    q, sat = bench._np_q16(x, k)
    qo, _ = orc.quantize_i16_sat(x, k, 1)
    assert np.array_equal(q, qo.astype(np.int64))
    assert np.array_equal(sat, np_q16(x, k)[1])
