"""ctypes binding of libina.so (the C ABI in include/ina.h).

The library is built in-tree by distributed-training-ina_amd/csrc/Makefile (or
__graft_entry__.build()).  There is no fallback: if libina.so is missing or does
not load, every op raises -- the device path is the product.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# INA_LIBRARY=<name>.so beside libina.so: a variant build of the same sources (the checked
# stream_store build, libina_storecheck.so), for test runs only
LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("INA_LIBRARY", "libina.so")))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

INA_OK, INA_EINVAL, INA_EHIP, INA_ESOCK, INA_ENOMEM = 0, -1, -2, -3, -4
MAX_WORKERS = 64
NGA_HDR_BYTES = 15
NUM_REGISTER = 16384
C128_VALUES = 128
C128_BYTES = 524
FLAG_OVERFLOW, FLAG_ACK, FLAG_COLLISION, FLAG_RESEND = 0x80, 0x40, 0x20, 0x10
ACT_DROP, ACT_FWD_AGG, ACT_FWD_COLLISION, ACT_FWD_ACK, ACT_FWD_OTHER = range(5)
ROUTE_MAX = 256                    # ipRoute size, ngaa.p4:59
PORT_DROP, PORT_NONE = -1, -2
I16_WIRE_SHIFT, I16_WIRE_MAX_RANKS = 22, 64      # include/ina.h


class InaError(RuntimeError):
    pass


class NgaParams(C.Structure):
    _fields_ = [("bitmap", C.c_uint32), ("count", C.c_uint8), ("flags", C.c_uint8),
                ("switch_id", C.c_uint8), ("pad", C.c_uint8), ("seq0", C.c_uint32),
                ("num_slots", C.c_uint32), ("V", C.c_int32)]


class NgaFields(C.Structure):
    _fields_ = [("bitmap", C.c_void_p), ("count", C.c_void_p), ("flags", C.c_void_p),
                ("index", C.c_void_p), ("switch_id", C.c_void_p), ("frag_id", C.c_void_p)]


class SwitchState(C.Structure):
    _fields_ = [("num_slots", C.c_uint32), ("V", C.c_int32), ("switch_id", C.c_int32),
                ("write_dropped", C.c_int32),
                ("count", C.c_void_p), ("frag", C.c_void_p), ("regs", C.c_void_p)]


class SwitchBatch(C.Structure):          # include/ina.h ina_switch_batch_t
    _fields_ = [("rows", C.c_void_p), ("pay", C.c_void_p), ("npkts", C.c_size_t), ("stride", C.c_size_t),
                ("desc", C.c_void_p), ("actions", C.c_void_p), ("scratch", C.c_void_p)]


class SwitchPs(C.Structure):             # include/ina.h ina_switch_ps_t
    _fields_ = [("seq0", C.c_uint32), ("k", C.c_int), ("weight_step", C.c_double), ("local", C.c_void_p),
                ("out", C.c_void_p), ("n", C.c_size_t), ("acks", C.c_void_p), ("ack_stride", C.c_size_t),
                ("ack_desc", C.c_void_p), ("keep_forwarded", C.c_int)]


INA_SWITCH_ALL, INA_SWITCH_SORT, INA_SWITCH_RUN = 0, 1, 2


# exported symbol -> argtypes (restype int unless listed in _RESTYPE)
_vp, _sz, _i, _u32, _d = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32, C.c_double
SIGNATURES = {
    "ina_version": [],
    "ina_last_error_string": [],
    "ina_set_tuning": [_i, _i],
    "ina_quantize_f32_i32": [_vp, _vp, _sz, _i, _vp],
    "ina_quantize_f32_i16_sat": [_vp, _vp, _sz, _i, _i, _vp, _vp],
    "ina_dequantize_i32_f32": [_vp, _vp, _sz, _i, _vp],
    "ina_dequantize_i16_f32": [_vp, _vp, _sz, _i, _vp],
    "ina_sum_reduce_i32": [_vp, _i, _vp, _sz, _vp],
    "ina_quantize_f32_i16_wire": [_vp, _vp, _sz, _i, _vp],
    "ina_i16_wire_finish": [_vp, _sz, _i, _i, _vp, _vp, _vp, _vp],
    "ina_sum_reduce_i16_sat": [_vp, _i, _vp, _sz, _i, _vp, _vp],
    "ina_quantize_reduce_f32_i32": [_vp, _i, _vp, _sz, _i, _vp],
    "ina_quantize_reduce_f32_i16_sat": [_vp, _i, _vp, _sz, _i, _i, _vp, _vp],
    "ina_ps_combine_f32": [_vp, _vp, _i, _d, _vp, _sz, _vp],
    "ina_ps_apply_i32": [_vp, _vp, _i, _d, _vp, _sz, _vp],
    "ina_ps_combine_ina_f32": [_vp, _vp, _i, _i, _d, _vp, _sz, _vp],
    "ina_pack_nga": [_vp, _sz, C.POINTER(NgaParams), _vp, _vp, _sz, _vp],
    "ina_quantize_pack_nga": [_vp, _vp, _sz, _i, C.POINTER(NgaParams), _vp, _sz, _vp],
    "ina_pack_nga_desc": [_vp, _sz, C.POINTER(NgaParams), _vp, _vp, _sz, _vp, _vp],
    "ina_quantize_pack_nga_desc": [_vp, _vp, _sz, _i, C.POINTER(NgaParams), _vp, _sz, _vp, _vp],
    "ina_nga_descriptors": [_vp, _sz, _sz, _vp, _vp],
    "ina_quantize_pack_nga_multi": [_vp, _i, _vp, _sz, _i, _vp, _vp, _sz, _vp, _vp],
    "ina_nga_make_descriptors": [_vp, _i, _sz, _vp, _vp],
    "ina_unpack_nga": [_vp, _sz, _i, _sz, C.POINTER(NgaFields), _vp, _vp],
    "ina_pack_c128": [_vp, _i, _i, _u32, _i, _vp, _vp],
    "ina_apply_completed_nga": [_vp, _sz, _i, _sz, _vp, _u32, _vp, _i, _d, _vp, _sz, _vp, _sz, _vp],
    "ina_pack_nga_split": [_vp, _sz, C.POINTER(NgaParams), _vp, _vp, _vp, _vp, _vp],
    "ina_quantize_pack_nga_multi_split": [_vp, _i, _vp, _sz, _i, _vp, _vp, _vp, _vp, _vp],
    "ina_unpack_nga_split": [_vp, _vp, _sz, _i, C.POINTER(NgaFields), _vp, _vp],
    "ina_send_packets_split_fd": [_i, _vp, _vp, _sz, _i, _u32],
    "ina_recv_packets_split_fd": [_i, _vp, _vp, _sz, _i, _sz, _i, _vp],
    "ina_switch_scratch_bytes": [_sz, _u32],
    "ina_switch_batch_path": [_vp, _sz, _u32, C.POINTER(C.c_int)],
    "ina_switch_process": [C.POINTER(SwitchState), _vp, _sz, _sz, _vp, _vp, _vp],
    "ina_switch": [C.POINTER(SwitchState), C.POINTER(SwitchBatch), C.POINTER(SwitchPs), _i, _vp],
    "ina_route_ipv4": [_vp, _vp, _u32, _sz, _vp, _vp, _i, _vp, _vp],
    "ina_checksum_i32": [_vp, _sz, _vp, _vp],
    "ina_absmax_f32": [_vp, _vp, _sz, _vp, _vp],
    "ina_absmax_multi_f32": [_vp, _i, _vp, _sz, _vp, _vp],
    "ina_scale_for": [C.c_float, _i, _i, C.POINTER(C.c_int)],
    "ina_host_reduce_scratch_bytes": [_i, _sz],
    "ina_sum_reduce_host_i32": [_vp, _i, _vp, _sz, _sz, _vp, _vp],
    "send_gradients": [C.POINTER(C.c_uint32), _i, _u32, _i, _u32, _i],
    "ina_send_gradients_fd": [_i, _vp, _i, _u32, _i, _u32, _i],
    "ina_send_packets_fd": [_i, _vp, _sz, _sz, _sz, _u32],
    "ina_recv_packets_fd": [_i, _vp, _sz, _sz, _sz, _i, _vp],
}
_RESTYPE = {"ina_version": C.c_char_p, "ina_last_error_string": C.c_char_p,
            "ina_switch_scratch_bytes": C.c_size_t, "ina_host_reduce_scratch_bytes": C.c_size_t,
            "send_gradients": None}

_lib = None
_lock = threading.Lock()


def open_library(path: str) -> C.CDLL:
    """A libina.so build at `path` with the ABI's signatures set (the A/B labs load a second
    build beside the in-tree one and swap it in as `_lib._lib`)."""
    if not os.path.exists(path):
        raise InaError(f"libina.so not built at {path}; run `make -C {CSRC}` or __graft_entry__.build()")
    lib = C.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, C.c_int)
    return lib


def load() -> C.CDLL:
    """Load libina.so (raises InaError if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = open_library(LIB_PATH)
    return _lib


def check(rc: int, what: str = "ina call") -> int:
    if rc < 0:
        msg = load().ina_last_error_string().decode(errors="replace")
        raise InaError(f"{what} failed (rc={rc}): {msg}")
    return rc


def ptr_array(ptrs):
    return (C.c_void_p * len(ptrs))(*ptrs)
