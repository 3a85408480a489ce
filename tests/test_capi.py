"""C-ABI boundary checks that need no GPU: libina.so loads, exports every
function include/ina.h declares, and the Python layer rejects bad input before
any device call (no CPU fallback exists)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "ina.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", src, flags=re.M)
    return sorted({n for n in names if not n.startswith("INA_") and n not in ("defined",)})


def test_header_declares_expected_surface():
    fns = declared_functions()
    for must in ("ina_sum_reduce_i32", "ina_quantize_f32_i32", "ina_pack_nga", "ina_unpack_nga",
                 "ina_pack_c128", "ina_switch_process", "send_gradients", "ina_ps_combine_f32"):
        assert must in fns
    assert len(fns) >= 20


def test_library_exports_every_declared_symbol():
    from ina_amd import _lib
    lib = _lib.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # and the Python binding knows every one of them
    assert not [f for f in declared_functions() if f not in _lib.SIGNATURES]


def test_legacy_symbol_is_unmangled_c():
    """communicator.py:15-24 binds `send_gradients` by its C name."""
    from ina_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    assert lib.send_gradients is not None
    assert _lib.load().ina_version().decode().startswith("ina-mi355x")


def test_error_codes_without_device_work():
    from ina_amd import _lib
    lib = _lib.load()
    assert lib.ina_quantize_f32_i32(None, None, 10, 500, None) == _lib.INA_EINVAL
    assert b"k out of range" in lib.ina_last_error_string()
    assert lib.ina_sum_reduce_i32(None, 0, None, 10, None) == _lib.INA_EINVAL
    assert lib.ina_sum_reduce_i32(None, 3, None, 0, None) == 0     # n == 0 is a no-op
    assert lib.ina_pack_c128(None, -1, 1, 0, 0, None, None) == _lib.INA_EINVAL
    prm = _lib.NgaParams(1, 2, 0, 1, 0, 1, 16384, 32)
    assert lib.ina_pack_nga(None, 64, ctypes.byref(prm), None, None, 100, None) == _lib.INA_EINVAL
    st = _lib.SwitchState(16384, 512, 1, 0, None, None, None)
    assert lib.ina_switch_process(ctypes.byref(st), None, 1, 2064, None, None, None) == _lib.INA_EINVAL


def test_ops_refuse_cpu_tensors():
    from ina_amd import ops
    x = torch.zeros(16, dtype=torch.float32)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.quantize(x, 16)
    with pytest.raises(ValueError):
        ops.sum_reduce([torch.zeros(8, dtype=torch.int32)])


def test_nga_stride():
    from ina_amd import ops
    assert ops.nga_stride(32) == 144 and ops.nga_stride(256) == 1040 and ops.nga_stride(128) == 528


@pytest.mark.parametrize("bits", [32, 16])
@pytest.mark.parametrize("W", [1, 2, 8, 16, 64])
def test_scale_for_is_the_largest_non_saturating_k(W, bits):
    """ina_scale_for (host-only): W * (amax * 2^k + 1/2) fits the width at k and not at
    k + 1 (unless k is already 127); checked in exact rational arithmetic."""
    from fractions import Fraction
    from ina_amd import ops
    lim = Fraction(2**(bits - 1) - 1, W) - Fraction(1, 2)
    if lim <= 0:
        return
    rng = np.random.default_rng(W * bits)
    amaxes = np.concatenate([rng.uniform(0, 1, 50), 10.0 ** rng.uniform(-30, 30, 50),
                             [1e-38, 1.0, 0.5, 2.0, 3.0e38]]).astype(np.float32)
    for a in amaxes:
        k = ops.scale_for(float(a), W, bits)
        af = Fraction(float(a))
        scaled = lambda kk: af * (Fraction(2) ** kk)                     # noqa: E731
        assert -126 <= k <= 127
        if k > -126:
            assert scaled(k) <= lim, (a, k)
        if k < 127:
            assert scaled(k + 1) > lim, (a, k)


def test_scale_for_edges():
    from ina_amd import _lib, ops
    assert ops.scale_for(0.0, 8) == 127
    for bad in (-1.0, float("nan"), float("inf")):
        with pytest.raises(_lib.InaError):
            ops.scale_for(bad, 8)
    with pytest.raises(_lib.InaError):
        ops.scale_for(1.0, 0)
    with pytest.raises(_lib.InaError):
        ops.scale_for(1.0, 8, bits=8)
    with pytest.raises(_lib.InaError):
        ops.scale_for(1.0, 70000, bits=16)      # W/2 alone exceeds 32767


def _einval_cases():
    from ina_amd import _lib
    P = _lib.ptr_array
    prm = _lib.NgaParams(1, 2, 0, 1, 0, 1, 16384, 32)
    st = _lib.SwitchState(16384, 32, 1, 0, None, None, None)
    return {
        "ina_quantize_f32_i32": (None, None, 64, 16, None),
        "ina_quantize_f32_i16_sat": (None, None, 64, 8, 32, None, None),
        "ina_dequantize_i32_f32": (None, None, 64, 16, None),
        "ina_quantize_f32_i16_wire": (None, None, 64, 11, None),
        "ina_i16_wire_finish": (None, 64, 11, 256, None, None, None, None),
        "ina_dequantize_i16_f32": (None, None, 64, 16, None),
        "ina_sum_reduce_i32": (P([None, None]), 2, None, 64, None),
        "ina_sum_reduce_i16_sat": (P([None, None]), 2, None, 64, 32, None, None),
        "ina_quantize_reduce_f32_i32": (P([None, None]), 2, None, 64, 16, None),
        "ina_quantize_reduce_f32_i16_sat": (P([None, None]), 2, None, 64, 8, 32, None, None),
        "ina_ps_combine_f32": (None, P([None, None]), 2, 0.5, None, 64, None),
        "ina_ps_apply_i32": (None, None, 16, 0.5, None, 64, None),
        "ina_ps_combine_ina_f32": (None, P([None, None]), 2, 16, 0.5, None, 64, None),
        "ina_pack_nga": (None, 64, ctypes.byref(prm), None, None, 144, None),
        "ina_quantize_pack_nga": (None, None, 64, 16, ctypes.byref(prm), None, 144, None),
        "ina_unpack_nga": (None, 2, 32, 144, None, None, None),
        "ina_pack_c128": (None, 2, 1, 0, 0, None, None),
        "ina_apply_completed_nga": (None, 2, 32, 144, None, 1, None, 16, 0.5, None, 64, None, 144,
                                    None),
        "ina_switch_process": (ctypes.byref(st), None, 2, 144, None, None, None),
        "ina_switch": (ctypes.byref(st), ctypes.byref(_lib.SwitchBatch(None, None, 2, 144, None, None, None)),
                       None, _lib.INA_SWITCH_ALL, None),
        "ina_pack_nga_desc": (None, 64, ctypes.byref(prm), None, None, 144, None, None),
        "ina_quantize_pack_nga_desc": (None, None, 64, 16, ctypes.byref(prm), None, 144, None, None),
        "ina_nga_descriptors": (None, 2, 144, None, None),
        "ina_nga_make_descriptors": ((_lib.NgaParams * 2)(prm, prm), 2, 64, P([None, None]), None),
        "ina_quantize_pack_nga_multi": (P([None, None]), 2, None, 64, 16,
                                        (_lib.NgaParams * 2)(prm, prm), P([None, None]), 144, None, None),
        "ina_route_ipv4": (None, None, 0, 4, None, None, 1, None, None),
        "ina_checksum_i32": (None, 64, None, None),
        "ina_absmax_f32": (None, None, 64, None, None),
        "ina_absmax_multi_f32": (P([None, None]), 2, None, 64, None, None),
        "ina_sum_reduce_host_i32": (P([None, None]), 2, None, 64, 0, None, None),
        "ina_switch_batch_path": (None, 2048, 16384, None),
        "ina_pack_nga_split": (None, 64, ctypes.byref(prm), None, None, None, None, None),
        "ina_quantize_pack_nga_multi_split": (P([None, None]), 2, None, 64, 16,
                                              (_lib.NgaParams * 2)(prm, prm), P([None, None]),
                                              P([None, None]), None, None),
        "ina_unpack_nga_split": (None, None, 2, 32, None, None, None),
    }


def test_every_device_entry_point_rejects_null_buffers():
    """Null buffers with n > 0 come back as INA_EINVAL with a message, before any HIP
    call (the reference's send_gradients would exit(-1), communicator.cc:11-12)."""
    from ina_amd import _lib
    lib = _lib.load()
    cases = _einval_cases()
    device_fns = {n for n in _lib.SIGNATURES if n.startswith("ina_")} - {
        "ina_version", "ina_last_error_string", "ina_set_tuning", "ina_switch_scratch_bytes",
        "ina_host_reduce_scratch_bytes", "ina_scale_for", "ina_send_gradients_fd",
        "ina_send_packets_fd", "ina_recv_packets_fd", "ina_send_packets_split_fd",
        "ina_recv_packets_split_fd"}
    assert device_fns == set(cases)
    for name, args in cases.items():
        rc = getattr(lib, name)(*args)
        assert rc == _lib.INA_EINVAL, (name, rc, lib.ina_last_error_string())
        assert lib.ina_last_error_string(), name


def test_socket_entry_points_reject_bad_descriptors():
    from ina_amd import _lib
    lib = _lib.load()
    assert lib.ina_send_packets_fd(-1, None, 2, 144, 144, 0) < 0
    assert lib.ina_recv_packets_fd(-1, None, 2, 144, 0, 0, None) < 0
    assert lib.ina_send_gradients_fd(-1, None, 1, 0, 1, 0, 0) < 0
    assert lib.ina_send_packets_split_fd(-1, None, None, 2, 32, 0) < 0
    assert lib.ina_recv_packets_split_fd(-1, None, None, 2, 32, 0, 0, None) < 0


def test_set_tuning_rejects_unknown_keys_and_values():
    """Launch-geometry knobs (include/ina.h ina_set_tuning): bad keys/values are refused
    and leave the defaults alone; no device work is involved."""
    from ina_amd import _lib
    lib = _lib.load()
    assert lib.ina_set_tuning(99, 1) == _lib.INA_EINVAL
    assert lib.ina_set_tuning(-1, 1) == _lib.INA_EINVAL
    assert lib.ina_set_tuning(1, 3) == _lib.INA_EINVAL          # reduce chunks: 1, 2 or 4
    assert lib.ina_set_tuning(7, 3) == _lib.INA_EINVAL          # H2D streams: 1 or 2
    for lab_key in (4, 5, 6, 10, 14):                           # grid-cap sweeps: lab builds only
        assert lib.ina_set_tuning(lab_key, 1) == _lib.INA_EINVAL
    assert lib.ina_set_tuning(11, 1) == _lib.INA_OK
    assert lib.ina_set_tuning(21, -1) == _lib.INA_EINVAL       # decision delay: 0..100000 us
    assert lib.ina_set_tuning(21, 0) == _lib.INA_OK
    assert lib.ina_set_tuning(12, 4) == _lib.INA_EINVAL        # sort: 0 auto, 3 digit passes
    assert lib.ina_set_tuning(12, 1) == _lib.INA_EINVAL        # one-sweep: moved to tools/lab
    assert lib.ina_set_tuning(12, 2) == _lib.INA_EINVAL
    assert lib.ina_set_tuning(12, 3) == _lib.INA_OK
    assert lib.ina_set_tuning(15, 4096) == _lib.INA_EINVAL      # tiny path: 0..2048 packets
    assert lib.ina_set_tuning(15, 512) == _lib.INA_OK
    assert lib.ina_set_tuning(13, 5) == _lib.INA_EINVAL        # one-sweep rounds: 0, 4, 8, 16
    assert lib.ina_set_tuning(12, 0) == _lib.INA_OK and lib.ina_set_tuning(13, 0) == _lib.INA_OK
    assert lib.ina_set_tuning(16, 2) == _lib.INA_EINVAL        # host zero copy: 0 / 1
    assert lib.ina_set_tuning(16, 0) == _lib.INA_OK and lib.ina_set_tuning(16, 1) == _lib.INA_OK
    assert lib.ina_set_tuning(17, 5) == _lib.INA_EINVAL        # bucket tile: 0 auto / 4 / 8
    for v in (4, 8, 0):
        assert lib.ina_set_tuning(17, v) == _lib.INA_OK


def test_switch_scratch_bytes_monotonic():
    """One scratch buffer sized for the largest batch must serve every smaller one, across
    the sort's chunk tiers (include/ina.h, ina_switch_scratch_bytes)."""
    from ina_amd import _lib
    lib = _lib.load()
    for slots in (1, 64, 16384, 1 << 17, (1 << 31) - 1):
        prev = 0
        for npk in list(range(1, 5000, 37)) + list(range(250_000, 560_000, 1_013)) + [819_200]:
            b = lib.ina_switch_scratch_bytes(npk, slots)
            assert b >= prev, (slots, npk)
            assert b >= 16 * npk
            prev = b


def test_process_apply_refuses_misaligned_registers():
    """ina_switch with a PS step takes only layouts its fused kernel handles, so
    keep_forwarded=0 always holds: misaligned slot registers are refused
    before any device work (the pointers are never dereferenced)."""
    from ina_amd import _lib
    lib = _lib.load()
    fake = 1 << 20                                   # aligned, never touched
    st = _lib.SwitchState(64, 32, 1, 0, fake, fake, fake + 8)
    b = _lib.SwitchBatch(fake, None, 4, 144, None, fake, fake)
    ps = _lib.SwitchPs(1, 16, 0.5, fake, fake, 64, None, 144, None, 0)
    rc = lib.ina_switch(ctypes.byref(st), ctypes.byref(b), ctypes.byref(ps), _lib.INA_SWITCH_ALL, None)
    assert rc == _lib.INA_EINVAL
    assert b"registers" in lib.ina_last_error_string()


def test_switch_call_validates_before_device_work():
    """ina_switch (include/ina.h): an unknown phase, a null batch, a split PS step whose ack
    rows are not header rows, and a run alone over a scratch no sort of that batch filled are
    refused with a message -- no pointer is dereferenced."""
    from ina_amd import _lib
    lib = _lib.load()
    fake = 1 << 20
    st = _lib.SwitchState(1 << 13, 32, 1, 0, fake, fake, fake)
    b = _lib.SwitchBatch(fake, None, 4096, 144, fake, fake, fake + 4096)
    assert lib.ina_switch(ctypes.byref(st), ctypes.byref(b), None, 3, None) == _lib.INA_EINVAL
    assert b"phase" in lib.ina_last_error_string()
    assert lib.ina_switch(ctypes.byref(st), None, None, _lib.INA_SWITCH_ALL, None) == _lib.INA_EINVAL
    split = _lib.SwitchBatch(fake, fake, 4096, 0, fake, fake, fake + 4096)
    ps = _lib.SwitchPs(1, 16, 0.5, fake, fake, 64, fake, 144, None, 0)
    assert lib.ina_switch(ctypes.byref(st), ctypes.byref(split), ctypes.byref(ps), _lib.INA_SWITCH_ALL,
                          None) == _lib.INA_EINVAL
    assert b"header rows" in lib.ina_last_error_string()
    # never sorted into this scratch: refused (it used to read stale packet ids)
    assert lib.ina_switch(ctypes.byref(st), ctypes.byref(b), None, _lib.INA_SWITCH_RUN, None) == _lib.INA_EINVAL
    assert b"no sort of this batch" in lib.ina_last_error_string()
    # a sort alone needs the descriptors
    nodesc = _lib.SwitchBatch(fake, None, 4096, 144, None, fake, fake + 4096)
    assert lib.ina_switch(ctypes.byref(st), ctypes.byref(nodesc), None, _lib.INA_SWITCH_SORT,
                          None) == _lib.INA_EINVAL
