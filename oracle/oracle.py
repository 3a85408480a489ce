"""oracle.py -- numpy/ctypes front end of the CPU oracle (libina_oracle.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package (ina_amd).  Every
function restates the reference (Fangjin98/distributed-training-INA); the
file:line each one follows is cited in ina_oracle.c.

Quantiser parity is UNPINNED: the reference's float_to_int / int_to_float are
missing from its repository (DataManager.py:9, NGAPacket.py:5); the definition
used here (scale 2^k, round-half-to-even, saturate) is the build's own, see
DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libina_oracle.so")

NGA_HDR = 15
NUM_REGISTER = 16384
C128_V = 128
C128_BYTES = 524
FLAG_OVERFLOW, FLAG_ACK, FLAG_COLLISION, FLAG_RESEND = 0x80, 0x40, 0x20, 0x10
ACT_DROP, ACT_FWD_AGG, ACT_FWD_COLLISION, ACT_FWD_ACK, ACT_FWD_OTHER = range(5)


class NgaParams(C.Structure):
    _fields_ = [("bitmap", C.c_uint32), ("count", C.c_uint8), ("flags", C.c_uint8),
                ("switch_id", C.c_uint8), ("pad", C.c_uint8), ("seq0", C.c_uint32),
                ("num_slots", C.c_uint32), ("V", C.c_int32)]


class NgaFields(C.Structure):
    _fields_ = [("bitmap", C.c_void_p), ("count", C.c_void_p), ("flags", C.c_void_p),
                ("index", C.c_void_p), ("switch_id", C.c_void_p), ("frag_id", C.c_void_p)]


class SwitchState(C.Structure):
    _fields_ = [("num_slots", C.c_uint32), ("V", C.c_int), ("switch_id", C.c_int),
                ("count", C.c_void_p), ("frag", C.c_void_p), ("regs", C.c_void_p)]


def build() -> str:
    """Compile libina_oracle.so (gcc) if missing or stale."""
    src = os.path.join(_HERE, "ina_oracle.c")
    if (not os.path.exists(_LIB_PATH)
            or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
        subprocess.run(["make", "-C", _HERE, "libina_oracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        L = _lib
        vp, sz, i, u32 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32
        sig = {
            "orc_quantize_f32_i32": [vp, vp, sz, i],
            "orc_quantize_f32_i16_sat": [vp, vp, sz, i, i, vp],
            "orc_dequantize_i32_f32": [vp, vp, sz, i],
            "orc_dequantize_i16_f32": [vp, vp, sz, i],
            "orc_sum_reduce_i32": [vp, i, vp, sz],
            "orc_sum_reduce_i16_sat": [vp, i, vp, sz, i, vp],
            "orc_quantize_reduce_f32_i32": [vp, i, vp, sz, i],
            "orc_quantize_reduce_f32_i16_sat": [vp, i, vp, sz, i, i, vp],
            "orc_quantize_f32_i16_wire": [vp, vp, sz, i],
            "orc_i16_wire_finish": [vp, sz, i, i, vp, vp, vp],
            "orc_ps_combine_f32": [vp, vp, i, C.c_double, vp, sz],
            "orc_ps_combine_ina_f32": [vp, vp, i, i, C.c_double, vp, sz],
            "orc_pack_nga": [vp, sz, C.POINTER(NgaParams), vp, vp, sz],
            "orc_unpack_nga": [vp, sz, i, sz, C.POINTER(NgaFields), vp],
            "orc_pack_c128": [vp, i, i, u32, i, vp],
            "orc_switch_init": [C.POINTER(SwitchState), u32, i, i],
            "orc_switch_free": [C.POINTER(SwitchState)],
            "orc_switch_run": [C.POINTER(SwitchState), vp, sz, sz, vp],
            "orc_cpu_packetise_aggregate": [vp, i, sz, i, i, vp, C.POINTER(C.c_double)],
            "orc_checksum_i32": [vp, sz],
            "orc_c128_bitmap": [i],
            "orc_route_ipv4": [vp, vp, u32, sz, vp, vp, i, vp],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = C.c_int
        L.orc_checksum_i32.restype = C.c_uint32
        L.orc_c128_bitmap.restype = C.c_uint32
        L.orc_switch_free.restype = None
        L.orc_route_ipv4.restype = None
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def _ptr_array(bufs):
    arr = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    return arr


def _chk(rc):
    if rc != 0:
        raise ValueError(f"oracle call failed rc={rc}")


# -- a1/a2 quantise / dequantise ------------------------------------------------
def quantize_i32(x: np.ndarray, k: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    q = np.empty(x.shape, np.int32)
    _chk(lib().orc_quantize_f32_i32(_p(x), _p(q), x.size, k))
    return q


def quantize_i16_sat(x: np.ndarray, k: int, V: int):
    x = np.ascontiguousarray(x, np.float32)
    q = np.empty(x.shape, np.int16)
    ovf = np.zeros((x.size + V - 1) // V, np.uint8)
    _chk(lib().orc_quantize_f32_i16_sat(_p(x), _p(q), x.size, k, V, _p(ovf)))
    return q, ovf


def dequantize_i32(s: np.ndarray, k: int) -> np.ndarray:
    s = np.ascontiguousarray(s, np.int32)
    y = np.empty(s.shape, np.float32)
    _chk(lib().orc_dequantize_i32_f32(_p(s), _p(y), s.size, k))
    return y


def dequantize_i16(s: np.ndarray, k: int) -> np.ndarray:
    s = np.ascontiguousarray(s, np.int16)
    y = np.empty(s.shape, np.float32)
    _chk(lib().orc_dequantize_i16_f32(_p(s), _p(y), s.size, k))
    return y


# -- a10 bulk sum ----------------------------------------------------------------
def sum_reduce_i32(bufs) -> np.ndarray:
    bufs = [np.ascontiguousarray(b, np.int32) for b in bufs]
    n = bufs[0].size
    out = np.empty(n, np.int32)
    _chk(lib().orc_sum_reduce_i32(_ptr_array(bufs), len(bufs), _p(out), n))
    return out


def sum_reduce_i16_sat(bufs, V: int):
    bufs = [np.ascontiguousarray(b, np.int16) for b in bufs]
    n = bufs[0].size
    out = np.empty(n, np.int16)
    ovf = np.zeros((n + V - 1) // V, np.uint8)
    _chk(lib().orc_sum_reduce_i16_sat(_ptr_array(bufs), len(bufs), _p(out), n, V, _p(ovf)))
    return out, ovf


def quantize_reduce_i32(bufs, k: int) -> np.ndarray:
    bufs = [np.ascontiguousarray(b, np.float32) for b in bufs]
    n = bufs[0].size
    out = np.empty(n, np.int32)
    _chk(lib().orc_quantize_reduce_f32_i32(_ptr_array(bufs), len(bufs), _p(out), n, k))
    return out


def quantize_reduce_i16_sat(bufs, k: int, V: int):
    bufs = [np.ascontiguousarray(b, np.float32) for b in bufs]
    n = bufs[0].size
    out = np.empty(n, np.int16)
    ovf = np.zeros((n + V - 1) // V, np.uint8)
    _chk(lib().orc_quantize_reduce_f32_i16_sat(_ptr_array(bufs), len(bufs), _p(out), n, k, V,
                                               _p(ovf)))
    return out, ovf


# -- int16 wire under sharding (build-defined; include/ina.h) -----------
def quantize_i16_wire(x: np.ndarray, k: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    w = np.empty(x.shape, np.int32)
    _chk(lib().orc_quantize_f32_i16_wire(_p(x), _p(w), x.size, k))
    return w


def i16_wire_finish(wsum: np.ndarray, k: int, V: int):
    """summed wire -> (int16, fp32 dequantised, per-slot overflow flags)"""
    wsum = np.ascontiguousarray(wsum, np.int32)
    n = wsum.size
    out16 = np.empty(n, np.int16)
    y = np.empty(n, np.float32)
    ovf = np.zeros((n + V - 1) // V, np.uint8)
    _chk(lib().orc_i16_wire_finish(_p(wsum), n, k, V, _p(out16), _p(y), _p(ovf)))
    return out16, y, ovf


# -- a13 PS float combine ---------------------------------------------------------
def ps_combine_f32(local: np.ndarray, paras, weight_step: float) -> np.ndarray:
    local = np.ascontiguousarray(local, np.float32)
    paras = [np.ascontiguousarray(p, np.float32) for p in paras]
    out = np.empty_like(local)
    _chk(lib().orc_ps_combine_f32(_p(local), _ptr_array(paras), len(paras), float(weight_step),
                                  _p(out), local.size))
    return out


def ps_combine_ina_f32(local: np.ndarray, paras, k: int, weight_step: float) -> np.ndarray:
    local = np.ascontiguousarray(local, np.float32)
    paras = [np.ascontiguousarray(p, np.float32) for p in paras]
    out = np.empty_like(local)
    _chk(lib().orc_ps_combine_ina_f32(_p(local), _ptr_array(paras), len(paras), k,
                                      float(weight_step), _p(out), local.size))
    return out


# -- a3/a12 NGA-V pack / unpack -----------------------------------------------------
def nga_packet_bytes(V: int) -> int:
    return NGA_HDR + 4 * V


def pack_nga(vals: np.ndarray, V: int, bitmap: int, count: int, switch_id: int, seq0: int,
             flags: int = 0, num_slots: int = NUM_REGISTER, stride: int | None = None,
             ovf: np.ndarray | None = None) -> np.ndarray:
    vals = np.ascontiguousarray(vals, np.int32)
    stride = stride or nga_packet_bytes(V)
    npk = (vals.size + V - 1) // V
    out = np.empty(npk * stride, np.uint8)
    prm = NgaParams(bitmap & 0xFFFFFFFF, count & 0xFF, flags & 0xFF, switch_id & 0xFF, 0,
                    seq0 & 0xFFFFFFFF, num_slots, V)
    op = None if ovf is None else _p(np.ascontiguousarray(ovf, np.uint8))
    _chk(lib().orc_pack_nga(_p(vals), vals.size, C.byref(prm), op, _p(out), stride))
    return out.reshape(npk, stride)


def unpack_nga(pkts: np.ndarray, V: int, stride: int | None = None):
    pkts = np.ascontiguousarray(pkts, np.uint8)
    stride = stride or nga_packet_bytes(V)
    npk = pkts.size // stride
    f = {"bitmap": np.empty(npk, np.uint32), "count": np.empty(npk, np.uint8),
         "flags": np.empty(npk, np.uint8), "index": np.empty(npk, np.uint32),
         "switch_id": np.empty(npk, np.uint8), "frag_id": np.empty(npk, np.uint32)}
    fs = NgaFields(*[f[k].ctypes.data for k in
                     ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
    vals = np.empty(npk * V, np.int32)
    _chk(lib().orc_unpack_nga(_p(pkts), npk, V, stride, C.byref(fs), _p(vals)))
    return f, vals


# -- a5 C-128 -------------------------------------------------------------------------
def c128_bitmap(worker_id: int) -> int:
    return lib().orc_c128_bitmap(worker_id)


def pack_c128(g: np.ndarray, packet_num: int, worker_id: int, aggregator_index: int,
              tensor_index: int) -> np.ndarray:
    g = np.ascontiguousarray(g).view(np.uint32)
    assert g.size >= packet_num * C128_V
    out = np.empty(packet_num * C128_BYTES, np.uint8)
    _chk(lib().orc_pack_c128(_p(g), packet_num, worker_id, aggregator_index & 0xFFFFFFFF,
                             tensor_index, _p(out)))
    return out


# -- a8-a11 stateful switch -------------------------------------------------------------
class Switch:
    """The P4 aggregator (ngaa.p4 Ingress) restated; registers persist across run()."""

    def __init__(self, V: int = 32, num_slots: int = NUM_REGISTER, switch_id: int = 1):
        self._st = SwitchState()
        self.V, self.num_slots = V, num_slots
        _chk(lib().orc_switch_init(C.byref(self._st), num_slots, V, switch_id))

    def run(self, pkts: np.ndarray, stride: int | None = None):
        """Process packets in arrival order; returns (rewritten packets, actions)."""
        stride = stride or nga_packet_bytes(self.V)
        buf = np.array(pkts, np.uint8, copy=True).reshape(-1)
        npk = buf.size // stride
        act = np.empty(npk, np.uint8)
        _chk(lib().orc_switch_run(C.byref(self._st), _p(buf), npk, stride, _p(act)))
        return buf.reshape(npk, stride), act

    def registers(self):
        st = self._st
        cnt = np.ctypeslib.as_array(C.cast(st.count, C.POINTER(C.c_uint8)), (self.num_slots,))
        frag = np.ctypeslib.as_array(C.cast(st.frag, C.POINTER(C.c_uint32)), (self.num_slots,))
        regs = np.ctypeslib.as_array(C.cast(st.regs, C.POINTER(C.c_uint32)),
                                     (self.num_slots, self.V))
        return cnt.copy(), frag.copy(), regs.copy()

    def __del__(self):
        try:
            lib().orc_switch_free(C.byref(self._st))
        except Exception:
            pass


# -- CPU baseline ------------------------------------------------------------------------
def cpu_packetise_aggregate(bufs, V: int, threads: int = 1):
    """Returns (aggregate int32[n], seconds)."""
    bufs = [np.ascontiguousarray(b, np.int32) for b in bufs]
    n = bufs[0].size
    out = np.empty(n, np.int32)
    secs = C.c_double(0.0)
    _chk(lib().orc_cpu_packetise_aggregate(_ptr_array(bufs), len(bufs), n, V, threads, _p(out),
                                           C.byref(secs)))
    return out, secs.value


def checksum_i32(x: np.ndarray) -> int:
    x = np.ascontiguousarray(x, np.int32)
    return int(lib().orc_checksum_i32(_p(x), x.size))


PORT_DROP, PORT_NONE = -1, -2


def route_ipv4(actions: np.ndarray, table, dst_ip=None, dst_default: int = 0) -> np.ndarray:
    """ipRoute (ngaa.p4:39-61) over a batch: table = [(ipv4 int, port | PORT_DROP |
    PORT_NONE), ...]; returns egress int32[np] (PORT_DROP for dropped packets)."""
    actions = np.ascontiguousarray(actions, np.uint8)
    keys = np.ascontiguousarray([k for k, _ in table] or [0], np.uint32)
    ports = np.ascontiguousarray([v for _, v in table] or [0], np.int32)
    dst = None if dst_ip is None else np.ascontiguousarray(dst_ip, np.uint32)
    egress = np.empty(actions.size, np.int32)
    lib().orc_route_ipv4(_p(actions), None if dst is None else _p(dst), dst_default & 0xFFFFFFFF,
                         actions.size, _p(keys), _p(ports), len(table), _p(egress))
    return egress
