"""stream_store's contract at the addresses that broke it (csrc/ina_device.h): every kernel
that writes through the sc1 buffer store (the reduce, the quantisers, the dequantisers, the
fused quantise + reduce, the PS updates, the int16 wire and its finish) writes its output into
views of one 7 GiB allocation placed (a) across a 4 GiB boundary (the high address word changes
inside a wave), (b) across the low word's bit 31 (where round 4's readfirstlane sign extension
dropped stores) and (c) wholly above it (every lane's low word has bit 31 set).  Each output
must equal the same call into an ordinary allocation bit for bit, and the bytes around the view
must stay untouched.  Under the checked build (INA_LIBRARY=libina_storecheck.so) the conftest
hook also asserts that no lane stored outside its wave's resource."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GiB = 1 << 30
N = 1 << 16                                     # elements per output
GUARD = 4096                                    # bytes checked on either side of a view


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd import ops  # noqa: F401  (fails loudly if libina.so is missing)


@pytest.fixture(scope="module")
def arena():
    buf = torch.empty(7 * GiB, dtype=torch.uint8, device=DEV)
    base = buf.data_ptr()
    b4 = ((base >> 32) + 1) << 32                # the first 4 GiB boundary past the start
    assert b4 + (1 << 31) + 64 * (1 << 20) < base + buf.numel()
    yield buf, base, b4
    del buf
    torch.cuda.empty_cache()


def _places(b4, nbytes):
    """Start addresses: across the 4 GiB boundary, across the low word's bit 31, above it.
    +48: a wave's 1 KiB run of 16-byte stores then always straddles the crossing point."""
    half = (nbytes // 2) & ~1023
    return {"straddle_4gib": b4 - half + 48,
            "straddle_bit31": b4 + (1 << 31) - half + 48,
            "bit31_set": b4 + (1 << 31) + (1 << 20) + 48}


def _view(arena, addr, dtype, n):
    buf, base, _ = arena
    off = addr - base
    esz = torch.empty(0, dtype=dtype).element_size()
    assert off % esz == 0 and off >= GUARD
    return buf[off:off + n * esz].view(dtype)


def _guard_bytes(arena, addr, nbytes):
    buf, base, _ = arena
    off = addr - base
    return torch.cat([buf[off - GUARD:off], buf[off + nbytes:off + nbytes + GUARD]]).clone()


def _cases():
    """name -> (output dtype, fn(out) -> None writing N elements into out)."""
    from ina_amd import _lib, ops
    g = torch.Generator(device=DEV).manual_seed(31)
    xs = [torch.randn(N, device=DEV, generator=g) * 1e-2 for _ in range(4)]
    xs16 = [torch.randn(N, device=DEV, generator=g) * 2.0 for _ in range(4)]   # some saturate
    i32 = [torch.randint(-(1 << 30), 1 << 30, (N,), dtype=torch.int32, device=DEV, generator=g) for _ in range(8)]
    i16 = [torch.randint(-(1 << 14), 1 << 14, (N,), dtype=torch.int16, device=DEV, generator=g) for _ in range(4)]
    local = torch.randn(N, device=DEV, generator=g) * 1e-2
    q = ops.quantize(xs[0], 16)
    q16, _ = ops.quantize_i16(xs16[0], 13, 32)
    wire = ops.quantize_i16_wire(xs16[1], 11)

    def ps_ina(out):
        arr = _lib.ptr_array([x.data_ptr() for x in xs])
        _lib.check(_lib.load().ina_ps_combine_ina_f32(local.data_ptr(), arr, len(xs), 16, 0.2, out.data_ptr(), N,
                                                     torch.cuda.current_stream().cuda_stream), "ps_combine_ina")

    return {
        "sum_reduce_i32_w8": (torch.int32, lambda o: ops.sum_reduce(i32, out=o)),
        "sum_reduce_i32_w3": (torch.int32, lambda o: ops.sum_reduce(i32[:3], out=o)),
        "sum_reduce_i16_sat": (torch.int16, lambda o: ops.sum_reduce_i16(i16, 32, out=o)),
        "quantize_i32": (torch.int32, lambda o: ops.quantize(xs[1], 16, out=o)),
        "quantize_i16_sat": (torch.int16, lambda o: ops.quantize_i16(xs16[2], 13, 32, out=o)),
        "dequantize_i32": (torch.float32, lambda o: ops.dequantize(q, 16, out=o)),
        "dequantize_i16": (torch.float32, lambda o: ops.dequantize(q16, 13, out=o)),
        "quantize_reduce_i32": (torch.int32, lambda o: ops.quantize_reduce(xs, 16, out=o)),
        "quantize_reduce_i16": (torch.int16, lambda o: ops.quantize_reduce_i16(xs16, 13, 32, out=o)),
        "ps_combine_f32": (torch.float32, lambda o: ops.ps_combine(local, xs, 0.2, out=o)),
        "ps_apply_i32": (torch.float32, lambda o: ops.ps_apply(local, q, 16, 0.2, out=o)),
        "ps_combine_ina_f32": (torch.float32, ps_ina),
        "i16_wire": (torch.int32, lambda o: ops.quantize_i16_wire(xs16[3], 11, out=o)),
        "i16_wire_finish_out16": (torch.int16, lambda o: ops.i16_wire_finish(wire, 11, 32, out16=o, want_y=False)),
        "i16_wire_finish_y": (torch.float32, lambda o: ops.i16_wire_finish(wire, 11, 32, y=o, want_out16=False)),
    }


CASES = ["sum_reduce_i32_w8", "sum_reduce_i32_w3", "sum_reduce_i16_sat", "quantize_i32", "quantize_i16_sat",
         "dequantize_i32", "dequantize_i16", "quantize_reduce_i32", "quantize_reduce_i16", "ps_combine_f32",
         "ps_apply_i32", "ps_combine_ina_f32", "i16_wire", "i16_wire_finish_out16", "i16_wire_finish_y"]


@pytest.mark.parametrize("place", ["straddle_4gib", "straddle_bit31", "bit31_set"])
@pytest.mark.parametrize("case", CASES)
def test_stream_store_views(arena, case, place):
    dtype, fn = _cases()[case]
    ref = torch.empty(N, dtype=dtype, device=DEV)
    fn(ref)
    esz = ref.element_size()
    addr = _places(arena[2], N * esz)[place]
    lo, hi = addr & 0xFFFFFFFF, (addr + N * esz - 1) & 0xFFFFFFFF
    if place == "straddle_4gib":
        assert (addr >> 32) != ((addr + N * esz - 1) >> 32)
    elif place == "straddle_bit31":
        assert lo < (1 << 31) <= hi
    else:
        assert lo >= (1 << 31)
    view = _view(arena, addr, dtype, N)
    view.fill_(0x55 if dtype != torch.float32 else float("nan"))
    before = _guard_bytes(arena, addr, N * esz)
    fn(view)
    torch.cuda.synchronize()
    got, want = view.cpu().numpy(), ref.cpu().numpy()
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (case, place)
    assert torch.equal(_guard_bytes(arena, addr, N * esz), before), (case, place)


def test_checked_build_counts_nothing_here():
    """Under the checked build, the library's own counter is readable and zero after the
    views above (the plain build has no counter: nothing to read)."""
    from ina_amd import _lib
    lib = _lib.load()
    if not hasattr(lib, "ina_store_check_violations"):
        pytest.skip("plain build (INA_STORE_CHECK=0)")
    n = ctypes.c_ulonglong(7)
    assert lib.ina_store_check_violations(ctypes.byref(n)) == 0
    assert n.value == 0
