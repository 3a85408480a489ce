"""torch-facing wrappers over libina.so's device entry points.

Tensors must be CUDA (HIP) tensors on one device, contiguous, of the stated
dtype.  Every call is asynchronous on torch's current stream of that device.
These are the kernels that replace the reference's CPU / switch arithmetic:

  quantize / dequantize      float_to_int / int_to_float (absent; DataManager.py:9,
                             NGAPacket.py:5) -- build-defined, see DESIGN.md
  sum_reduce                 the switch's per-slot Processor add (processor.p4:14-24)
  sum_reduce_host            the same from/to host memory across PCIe (PS ingest)
  quantize_reduce            worker quantise fused with the aggregator sum
  pack_nga / unpack_nga      DataManager._send_data (DataManager.py:111-165) and the
                             PS-side parse (NGAPacket.py:62-143), headers.p4 layout
  pack_c128                  send_gradients' packet loop (communicator.cc:23-37)
  ps_combine                 aggregate() (launch.py:42-52)
  absmax / scale_for         per-bucket dynamic scale for the quantiser (build-defined)
"""
from __future__ import annotations

import ctypes as C
import numbers

import torch

from . import _lib
from ._lib import NGA_HDR_BYTES, NUM_REGISTER, check, load, ptr_array


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _req(t: torch.Tensor, dtype, name: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor; the INA path has no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _fits(out: torch.Tensor, numel: int, name: str = "out"):
    """A caller-supplied output must hold what the kernel writes (the C ABI sees only a
    pointer, so a short buffer would be an out-of-bounds device write)."""
    if not isinstance(out, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if out.numel() < int(numel):
        raise ValueError(f"{name} holds {out.numel()} elements, needs {int(numel)}")


def _same_device(*ts):
    d = ts[0].device
    for t in ts[1:]:
        if t.device != d:
            raise ValueError("all tensors must be on the same device")


def nga_stride(V: int) -> int:
    """Recommended device packet stride: 15 + 4V rounded up to 16 bytes."""
    return (NGA_HDR_BYTES + 4 * V + 15) // 16 * 16


# -- quantise / dequantise -------------------------------------------------------------
def quantize(x: torch.Tensor, k: int, out: torch.Tensor | None = None) -> torch.Tensor:
    _req(x, torch.float32, "x")
    out = torch.empty(x.shape, dtype=torch.int32, device=x.device) if out is None else out
    _fits(out, x.numel())
    _req(out, torch.int32, "out")
    check(load().ina_quantize_f32_i32(x.data_ptr(), out.data_ptr(), x.numel(), k, _stream(x)),
          "quantize")
    return out


def quantize_i16(x: torch.Tensor, k: int, V: int, out=None, overflow=None):
    _req(x, torch.float32, "x")
    out = torch.empty(x.shape, dtype=torch.int16, device=x.device) if out is None else out
    _fits(out, x.numel())
    nslot = (x.numel() + V - 1) // V
    overflow = torch.empty(nslot, dtype=torch.uint8, device=x.device) if overflow is None else overflow
    _fits(overflow, nslot, "overflow")
    _req(out, torch.int16, "out")
    _req(overflow, torch.uint8, "overflow")
    check(load().ina_quantize_f32_i16_sat(x.data_ptr(), out.data_ptr(), x.numel(), k, V,
                                          overflow.data_ptr(), _stream(x)), "quantize_i16")
    return out, overflow


def quantize_i16_wire(x: torch.Tensor, k: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 -> int32 wire words q16(x) + (saturated << 22) (include/ina.h): the int16
    quantisation widened so an int32 SUM collective carries the sum and the saturation
    count together (the sharded int16 path, dist.ShardedAggregator(wire="i16"))."""
    _req(x, torch.float32, "x")
    out = torch.empty(x.shape, dtype=torch.int32, device=x.device) if out is None else out
    _fits(out, x.numel())
    _req(out, torch.int32, "out")
    _same_device(x, out)
    check(load().ina_quantize_f32_i16_wire(x.data_ptr(), out.data_ptr(), x.numel(), k, _stream(x)),
          "quantize_i16_wire")
    return out


def i16_wire_finish(wire_sum: torch.Tensor, k: int, V: int, out16=None, y=None, overflow=None,
                    want_out16: bool = True, want_y: bool = True):
    """Summed int32 wire shard -> (int16 saturated sum, fp32 dequantised, u8 per-slot
    overflow flags); a result is None when neither given nor wanted."""
    _req(wire_sum, torch.int32, "wire_sum")
    n, dev = wire_sum.numel(), wire_sum.device
    if V <= 0:
        raise ValueError("V must be > 0")
    nslot = (n + V - 1) // V
    if out16 is None and want_out16:
        out16 = torch.empty(n, dtype=torch.int16, device=dev)
    if y is None and want_y:
        y = torch.empty(n, dtype=torch.float32, device=dev)
    overflow = torch.empty(nslot, dtype=torch.uint8, device=dev) if overflow is None else overflow
    for t, dt, cnt, name in ((out16, torch.int16, n, "out16"), (y, torch.float32, n, "y"),
                             (overflow, torch.uint8, nslot, "overflow")):
        if t is not None:
            _fits(t, cnt, name)
            _req(t, dt, name)
            _same_device(wire_sum, t)
    check(load().ina_i16_wire_finish(wire_sum.data_ptr(), n, k, V,
                                     out16.data_ptr() if out16 is not None else None,
                                     y.data_ptr() if y is not None else None, overflow.data_ptr(),
                                     _stream(wire_sum)), "i16_wire_finish")
    return out16, y, overflow


def dequantize(s: torch.Tensor, k: int, out: torch.Tensor | None = None) -> torch.Tensor:
    out = torch.empty(s.shape, dtype=torch.float32, device=s.device) if out is None else out
    _fits(out, s.numel())
    _req(out, torch.float32, "out")
    if s.dtype == torch.int16:
        _req(s, torch.int16, "s")
        rc = load().ina_dequantize_i16_f32(s.data_ptr(), out.data_ptr(), s.numel(), k, _stream(s))
    else:
        _req(s, torch.int32, "s")
        rc = load().ina_dequantize_i32_f32(s.data_ptr(), out.data_ptr(), s.numel(), k, _stream(s))
    check(rc, "dequantize")
    return out


# -- aggregator --------------------------------------------------------------------------
def _bufs(bufs, dtype, name="bufs"):
    if isinstance(bufs, torch.Tensor):       # [W, n] stacked
        bufs = list(bufs.unbind(0)) if bufs.dim() > 1 else [bufs]
    bufs = list(bufs)
    if not 1 <= len(bufs) <= _lib.MAX_WORKERS:
        raise ValueError(f"need 1..{_lib.MAX_WORKERS} worker buffers, got {len(bufs)}")
    n = bufs[0].numel()
    for i, b in enumerate(bufs):
        _req(b, dtype, f"{name}[{i}]")
        if b.numel() != n:
            raise ValueError("worker buffers differ in length")
    _same_device(*bufs)
    return bufs, n


def sum_reduce(bufs, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = sum_w bufs[w][i] mod 2^32 (int32), the switch's slot sum."""
    bufs, n = _bufs(bufs, torch.int32)
    out = torch.empty(n, dtype=torch.int32, device=bufs[0].device) if out is None else out
    _fits(out, n)
    _req(out, torch.int32, "out")
    arr = ptr_array([b.data_ptr() for b in bufs])
    check(load().ina_sum_reduce_i32(arr, len(bufs), out.data_ptr(), n, _stream(out)), "sum_reduce")
    return out


def sum_reduce_host(bufs, out: torch.Tensor | None = None, chunk: int = 0,
                    device: torch.device | str | None = None, scratch: torch.Tensor | None = None):
    """PCIe-inclusive aggregation at the PS: W int32 buckets in HOST memory (what the worker
    sockets deliver) -> the same W-way sum-reduce -> the aggregate back in host memory
    (`out`, pinned CPU int32 by default).  Pinned inputs and output: one reduce launch reads
    them across PCIe in place (zero copy); otherwise chunked and pipelined over H2D /
    reduce / D2H (ina_sum_reduce_host_i32).  Returns when `out` is complete."""
    if isinstance(bufs, torch.Tensor):
        bufs = list(bufs.unbind(0)) if bufs.dim() > 1 else [bufs]
    bufs = list(bufs)
    if not 1 <= len(bufs) <= _lib.MAX_WORKERS:
        raise ValueError(f"need 1..{_lib.MAX_WORKERS} worker buffers, got {len(bufs)}")
    n = bufs[0].numel()
    for i, b in enumerate(bufs):
        if b.is_cuda or b.dtype != torch.int32 or not b.is_contiguous() or b.numel() != n:
            raise ValueError(f"bufs[{i}] must be a contiguous host int32 tensor of {n} values")
    out = torch.empty(n, dtype=torch.int32).pin_memory() if out is None else out
    _fits(out, n)
    if out.is_cuda or out.dtype != torch.int32 or not out.is_contiguous() or out.numel() != n:
        raise ValueError("out must be a contiguous host int32 tensor")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    lib = load()
    need = lib.ina_host_reduce_scratch_bytes(len(bufs), chunk)
    if scratch is None or scratch.numel() < need:
        scratch = torch.empty(need, dtype=torch.uint8, device=dev)
    arr = ptr_array([b.data_ptr() for b in bufs])
    with torch.cuda.device(dev):
        check(lib.ina_sum_reduce_host_i32(arr, len(bufs), out.data_ptr(), n, chunk,
                                          scratch.data_ptr(), torch.cuda.current_stream(dev).cuda_stream),
              "sum_reduce_host")
    return out


def sum_reduce_i16(bufs, V: int, out=None, overflow=None):
    bufs, n = _bufs(bufs, torch.int16)
    dev = bufs[0].device
    out = torch.empty(n, dtype=torch.int16, device=dev) if out is None else out
    _fits(out, n)
    overflow = (torch.empty((n + V - 1) // V, dtype=torch.uint8, device=dev)
                if overflow is None else overflow)
    _req(out, torch.int16, "out")
    _req(overflow, torch.uint8, "overflow")
    _fits(overflow, (n + V - 1) // V, "overflow")
    arr = ptr_array([b.data_ptr() for b in bufs])
    check(load().ina_sum_reduce_i16_sat(arr, len(bufs), out.data_ptr(), n, V, overflow.data_ptr(),
                                        _stream(out)), "sum_reduce_i16")
    return out, overflow


def quantize_reduce(bufs, k: int, out: torch.Tensor | None = None) -> torch.Tensor:
    bufs, n = _bufs(bufs, torch.float32)
    out = torch.empty(n, dtype=torch.int32, device=bufs[0].device) if out is None else out
    _fits(out, n)
    _req(out, torch.int32, "out")
    arr = ptr_array([b.data_ptr() for b in bufs])
    check(load().ina_quantize_reduce_f32_i32(arr, len(bufs), out.data_ptr(), n, k, _stream(out)),
          "quantize_reduce")
    return out


def quantize_reduce_i16(bufs, k: int, V: int, out=None, overflow=None):
    bufs, n = _bufs(bufs, torch.float32)
    dev = bufs[0].device
    out = torch.empty(n, dtype=torch.int16, device=dev) if out is None else out
    _fits(out, n)
    overflow = (torch.empty((n + V - 1) // V, dtype=torch.uint8, device=dev)
                if overflow is None else overflow)
    _req(out, torch.int16, "out")
    _req(overflow, torch.uint8, "overflow")
    _fits(overflow, (n + V - 1) // V, "overflow")
    arr = ptr_array([b.data_ptr() for b in bufs])
    check(load().ina_quantize_reduce_f32_i16_sat(arr, len(bufs), out.data_ptr(), n, k, V,
                                                 overflow.data_ptr(), _stream(out)),
          "quantize_reduce_i16")
    return out, overflow


# -- PS combine ----------------------------------------------------------------------------
def ps_combine(local: torch.Tensor, paras, weight_step: float, out=None) -> torch.Tensor:
    """launch.py:42-52: local + float(weight_step) * sum_w (paras[w] - local), bit-exact."""
    _req(local, torch.float32, "local")
    paras, n = _bufs(paras, torch.float32, "paras")
    if n != local.numel():
        raise ValueError("local and paras differ in length")
    out = torch.empty_like(local) if out is None else out
    _fits(out, local.numel())
    arr = ptr_array([p.data_ptr() for p in paras])
    check(load().ina_ps_combine_f32(local.data_ptr(), arr, len(paras), float(weight_step),
                                    out.data_ptr(), n, _stream(local)), "ps_combine")
    return out


def ps_apply(local: torch.Tensor, sum_int: torch.Tensor, k: int, weight_step: float, out=None):
    """INA update: local + float(weight_step) * dequantize(sum_int, k)."""
    _req(local, torch.float32, "local")
    _req(sum_int, torch.int32, "sum_int")
    out = torch.empty_like(local) if out is None else out
    _fits(out, local.numel())
    check(load().ina_ps_apply_i32(local.data_ptr(), sum_int.data_ptr(), k, float(weight_step),
                                  out.data_ptr(), local.numel(), _stream(local)), "ps_apply")
    return out


# -- packets -----------------------------------------------------------------------------------
def _ack_desc_arg(ack_desc, acks):
    """The ack rows' descriptor output of process_apply / run_apply: a device pointer or None."""
    if ack_desc is None:
        return None
    if acks is None:
        raise ValueError("ack_desc needs acks")
    _req(ack_desc, torch.int64, "ack_desc")
    _fits(ack_desc, acks.shape[0], "ack_desc")
    if not ack_desc.is_contiguous():
        raise ValueError("ack_desc must be contiguous (one int64 per ack row)")
    _same_device(acks, ack_desc)
    return ack_desc.data_ptr()


def _desc_arg(desc, npk, dev):
    """Descriptor output/input: True -> a new int64 [npk] tensor; a tensor -> checked."""
    if desc is None or desc is False:
        return None
    if desc is True:
        return torch.empty(npk, dtype=torch.int64, device=dev)
    _req(desc, torch.int64, "desc")
    _fits(desc, npk, "desc")
    if desc.device != torch.device(dev):
        raise ValueError("all tensors must be on the same device")
    return desc


def pack_nga(vals: torch.Tensor, V: int, bitmap: int, count: int, switch_id: int, seq0: int,
             flags: int = 0, num_slots: int = NUM_REGISTER, stride: int | None = None,
             overflow: torch.Tensor | None = None, out: torch.Tensor | None = None,
             desc=None):
    """Returns uint8 [npkts, stride] device packets (first 15 + 4V bytes of each row on the
    wire).  desc=True (or an int64 [npkts] tensor) also writes each packet's descriptor
    (header bytes 4..11, include/ina.h) and returns (packets, descriptors)."""
    _req(vals, torch.int32, "vals")
    stride = stride or nga_stride(V)
    npk = (vals.numel() + V - 1) // V
    out = torch.empty((npk, stride), dtype=torch.uint8, device=vals.device) if out is None else out
    _fits(out, npk * stride)
    prm = _lib.NgaParams(bitmap & 0xFFFFFFFF, count & 0xFF, flags & 0xFF, switch_id & 0xFF, 0,
                         seq0 & 0xFFFFFFFF, num_slots, V)
    ovp = None
    if overflow is not None:
        _req(overflow, torch.uint8, "overflow")
        _fits(overflow, npk, "overflow")
        ovp = overflow.data_ptr()
    d = _desc_arg(desc, npk, vals.device)
    check(load().ina_pack_nga_desc(vals.data_ptr(), vals.numel(), C.byref(prm), ovp, out.data_ptr(),
                                   stride, d.data_ptr() if d is not None else None, _stream(vals)),
          "pack_nga")
    return (out, d) if d is not None else out


def nga_descriptors(pkts: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """int64 [npkts] descriptors (header bytes 4..11) gathered from uint8 [npkts, stride]."""
    _req(pkts, torch.uint8, "pkts")
    npk, stride = pkts.shape
    d = _desc_arg(True if out is None else out, npk, pkts.device)
    check(load().ina_nga_descriptors(pkts.data_ptr(), npk, stride, d.data_ptr(), _stream(pkts)),
          "nga_descriptors")
    return d


def quantize_pack_nga(x: torch.Tensor, k: int, V: int, bitmap: int, count: int, switch_id: int,
                      seq0: int, base: torch.Tensor | None = None, flags: int = 0,
                      num_slots: int = NUM_REGISTER, stride: int | None = None,
                      out: torch.Tensor | None = None, desc=None):
    """Fused worker side: NGA-V packets of quantize(x - base, k) in one pass (same bytes as
    quantize() then pack_nga()); desc as in pack_nga."""
    _req(x, torch.float32, "x")
    if base is not None:
        _req(base, torch.float32, "base")
        if base.numel() != x.numel():
            raise ValueError("base and x differ in length")
        _same_device(x, base)
    stride = stride or nga_stride(V)
    npk = (x.numel() + V - 1) // V
    out = torch.empty((npk, stride), dtype=torch.uint8, device=x.device) if out is None else out
    _fits(out, npk * stride)
    prm = _lib.NgaParams(bitmap & 0xFFFFFFFF, count & 0xFF, flags & 0xFF, switch_id & 0xFF, 0,
                         seq0 & 0xFFFFFFFF, num_slots, V)
    d = _desc_arg(desc, npk, x.device)
    check(load().ina_quantize_pack_nga_desc(x.data_ptr(), base.data_ptr() if base is not None else None,
                                            x.numel(), k, C.byref(prm), out.data_ptr(), stride,
                                            d.data_ptr() if d is not None else None, _stream(x)),
          "quantize_pack_nga")
    return (out, d) if d is not None else out


def quantize_pack_nga_multi(xs, k: int, V: int, bitmaps, count: int, switch_id: int, seq0,
                            base: torch.Tensor | None = None, flags: int = 0,
                            num_slots: int = NUM_REGISTER, stride: int | None = None,
                            outs=None, descs=None):
    """W workers' quantize_pack_nga in ONE launch (ina_quantize_pack_nga_multi): worker w's
    packets of quantize(xs[w] - base, k) with header word bitmaps[w] and sequence start
    seq0 (an int for all workers or one per worker); the shared base is read once for
    every 8 workers.  Same bytes as W quantize_pack_nga calls.  outs / descs: W tensors
    each (descs=True allocates them); returns outs, or (outs, descs)."""
    xs, n = _bufs(xs, torch.float32, "xs")
    W, dev = len(xs), xs[0].device
    if base is not None:
        _req(base, torch.float32, "base")
        if base.numel() != n:
            raise ValueError("base and xs differ in length")
        _same_device(xs[0], base)
    bitmaps = list(bitmaps)
    seqs = [int(seq0)] * W if isinstance(seq0, numbers.Integral) else list(seq0)
    if len(bitmaps) != W or len(seqs) != W:
        raise ValueError("one bitmap and one seq0 per worker")
    stride = stride or nga_stride(V)
    npk = (n + V - 1) // V
    if outs is None:
        outs = [torch.empty((npk, stride), dtype=torch.uint8, device=dev) for _ in range(W)]
    outs = list(outs)
    if len(outs) != W:
        raise ValueError("one output per worker")
    for o in outs:
        _fits(o, npk * stride)
        _req(o, torch.uint8, "outs")
        _same_device(xs[0], o)
    ds = None
    if descs is not None and descs is not False:
        if descs is not True and (len(descs) != W or any(d is None for d in descs)):
            raise ValueError("descs: True, or one int64 tensor per worker")
        ds = [_desc_arg(True if descs is True else descs[w], npk, dev) for w in range(W)]
    prm = (_lib.NgaParams * W)(*[_lib.NgaParams(bitmaps[w] & 0xFFFFFFFF, count & 0xFF, flags & 0xFF,
                                                switch_id & 0xFF, 0, seqs[w] & 0xFFFFFFFF, num_slots, V)
                                 for w in range(W)])
    check(load().ina_quantize_pack_nga_multi(
        ptr_array([x.data_ptr() for x in xs]), W, base.data_ptr() if base is not None else None, n, k,
        prm, ptr_array([o.data_ptr() for o in outs]), stride,
        ptr_array([d.data_ptr() for d in ds]) if ds is not None else None, _stream(xs[0])),
        "quantize_pack_nga_multi")
    return (outs, ds) if ds is not None else outs


# ---- split NGA rows (include/ina.h): 16-byte header rows + 4V-byte payload rows -------------
def _split_rows(npk, V, dev, hdr=None, pay=None):
    if V % 4 or not 4 <= V <= 256:
        raise ValueError("split rows need V a multiple of 4 in [4, 256]")
    hdr = torch.zeros((npk, 16), dtype=torch.uint8, device=dev) if hdr is None else hdr
    pay = torch.empty((npk, 4 * V), dtype=torch.uint8, device=dev) if pay is None else pay
    for t, name, row in ((hdr, "hdr", 16), (pay, "pay", 4 * V)):
        _req(t, torch.uint8, name)
        if t.dim() != 2 or t.shape[1] != row or t.shape[0] < npk or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous uint8 [>= {npk}, {row}] tensor")
        if t.data_ptr() % 16:
            raise ValueError(f"{name} rows must be 16-byte aligned")
    return hdr, pay


def pack_nga_split(vals: torch.Tensor, V: int, bitmap: int, count: int, switch_id: int, seq0: int,
                   flags: int = 0, num_slots: int = NUM_REGISTER, overflow: torch.Tensor | None = None,
                   hdr: torch.Tensor | None = None, pay: torch.Tensor | None = None, desc=None):
    """pack_nga into split rows (ina_pack_nga_split): returns (hdr uint8 [npkts, 16], pay uint8
    [npkts, 4V]) -- hdr[p, :15] || pay[p] is packet p's datagram, byte for byte the packed
    row's first 15 + 4V bytes -- or (hdr, pay, desc) with desc as in pack_nga."""
    _req(vals, torch.int32, "vals")
    npk = (vals.numel() + V - 1) // V
    hdr, pay = _split_rows(npk, V, vals.device, hdr, pay)
    prm = _lib.NgaParams(bitmap & 0xFFFFFFFF, count & 0xFF, flags & 0xFF, switch_id & 0xFF, 0,
                         seq0 & 0xFFFFFFFF, num_slots, V)
    ovp = None
    if overflow is not None:
        _req(overflow, torch.uint8, "overflow")
        _fits(overflow, npk, "overflow")
        ovp = overflow.data_ptr()
    d = _desc_arg(desc, npk, vals.device)
    check(load().ina_pack_nga_split(vals.data_ptr(), vals.numel(), C.byref(prm), ovp, hdr.data_ptr(),
                                    pay.data_ptr(), d.data_ptr() if d is not None else None, _stream(vals)),
          "pack_nga_split")
    return (hdr, pay, d) if d is not None else (hdr, pay)


def quantize_pack_nga_multi_split(xs, k: int, V: int, bitmaps, count: int, switch_id: int, seq0,
                                  base: torch.Tensor | None = None, flags: int = 0,
                                  num_slots: int = NUM_REGISTER, hdrs=None, pays=None, descs=None):
    """quantize_pack_nga_multi into split rows (ina_quantize_pack_nga_multi_split): W
    workers' quantize(xs[w] - base, k) as header rows hdrs[w] + payload rows pays[w], the
    base read once per 8 workers.  Returns (hdrs, pays) or (hdrs, pays, descs)."""
    xs, n = _bufs(xs, torch.float32, "xs")
    W, dev = len(xs), xs[0].device
    if base is not None:
        _req(base, torch.float32, "base")
        if base.numel() != n:
            raise ValueError("base and xs differ in length")
        _same_device(xs[0], base)
    bitmaps = list(bitmaps)
    seqs = [int(seq0)] * W if isinstance(seq0, numbers.Integral) else list(seq0)
    if len(bitmaps) != W or len(seqs) != W:
        raise ValueError("one bitmap and one seq0 per worker")
    npk = (n + V - 1) // V
    hdrs = [None] * W if hdrs is None else list(hdrs)
    pays = [None] * W if pays is None else list(pays)
    if len(hdrs) != W or len(pays) != W:
        raise ValueError("one header and one payload array per worker")
    rows = [_split_rows(npk, V, dev, h, p) for h, p in zip(hdrs, pays)]
    hdrs, pays = [r[0] for r in rows], [r[1] for r in rows]
    ds = None
    if descs is not None and descs is not False:
        if descs is not True and (len(descs) != W or any(d is None for d in descs)):
            raise ValueError("descs: True, or one int64 tensor per worker")
        ds = [_desc_arg(True if descs is True else descs[w], npk, dev) for w in range(W)]
    prm = (_lib.NgaParams * W)(*[_lib.NgaParams(bitmaps[w] & 0xFFFFFFFF, count & 0xFF, flags & 0xFF,
                                                switch_id & 0xFF, 0, seqs[w] & 0xFFFFFFFF, num_slots, V)
                                 for w in range(W)])
    check(load().ina_quantize_pack_nga_multi_split(
        ptr_array([x.data_ptr() for x in xs]), W, base.data_ptr() if base is not None else None, n, k,
        prm, ptr_array([h.data_ptr() for h in hdrs]), ptr_array([p.data_ptr() for p in pays]),
        ptr_array([d.data_ptr() for d in ds]) if ds is not None else None, _stream(xs[0])),
        "quantize_pack_nga_multi_split")
    return (hdrs, pays, ds) if ds is not None else (hdrs, pays)


def unpack_nga_split(hdr: torch.Tensor, pay: torch.Tensor, V: int, with_values: bool = True):
    """The PS parse of split rows: (fields dict of device tensors, int32 values [npkts*V] or
    None) -- what unpack_nga returns for the packed rows."""
    npk = hdr.shape[0]
    hdr, pay = _split_rows(npk, V, hdr.device, hdr, pay)
    dev = hdr.device
    f = {"bitmap": torch.empty(npk, dtype=torch.int32, device=dev),
         "count": torch.empty(npk, dtype=torch.uint8, device=dev),
         "flags": torch.empty(npk, dtype=torch.uint8, device=dev),
         "index": torch.empty(npk, dtype=torch.int32, device=dev),
         "switch_id": torch.empty(npk, dtype=torch.uint8, device=dev),
         "frag_id": torch.empty(npk, dtype=torch.int32, device=dev)}
    fs = _lib.NgaFields(*[f[k].data_ptr() for k in ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
    vals = torch.empty(npk * V, dtype=torch.int32, device=dev) if with_values else None
    check(load().ina_unpack_nga_split(hdr.data_ptr(), pay.data_ptr(), npk, V, C.byref(fs),
                                      vals.data_ptr() if vals is not None else None, _stream(hdr)),
          "unpack_nga_split")
    return f, vals


def make_descriptors(n_packets: int, W: int, count: int, switch_id: int, seq0,
                     flags: int = 0, num_slots: int = NUM_REGISTER, outs=None,
                     device: str | torch.device = "cuda", stream: torch.cuda.Stream | None = None):
    """Packet descriptors from the header fields alone (ina_nga_make_descriptors): W
    workers x n_packets int64 entries, what pack_nga(desc=True) writes beside each packet
    (no overflow bits) -- a switch's sort() can take them before the payload exists.
    seq0: one int for every worker or one per worker.  Returns the W tensors."""
    W = int(W)
    seqs = [int(seq0)] * W if isinstance(seq0, numbers.Integral) else list(seq0)
    if len(seqs) != W or not 1 <= W <= _lib.MAX_WORKERS:
        raise ValueError("one seq0 per worker, 1..64 workers")
    if outs is None:
        outs = [torch.empty(n_packets, dtype=torch.int64, device=device) for _ in range(W)]
    outs = [_desc_arg(o, n_packets, outs[0].device) for o in outs]
    if len(outs) != W:
        raise ValueError("one output per worker")
    prm = (_lib.NgaParams * W)(*[_lib.NgaParams(0, count & 0xFF, flags & 0xFF, switch_id & 0xFF, 0,
                                                seqs[w] & 0xFFFFFFFF, num_slots, 1) for w in range(W)])
    st = stream.cuda_stream if stream is not None else _stream(outs[0])
    check(load().ina_nga_make_descriptors(prm, W, n_packets, ptr_array([o.data_ptr() for o in outs]), st),
          "nga_make_descriptors")
    return outs


def unpack_nga(pkts: torch.Tensor, V: int, stride: int | None = None, with_values: bool = True):
    """Returns (fields dict of device tensors, int32 values [npkts*V] or None)."""
    _req(pkts, torch.uint8, "pkts")
    stride = stride or (pkts.shape[1] if pkts.dim() == 2 else nga_stride(V))
    npk = pkts.numel() // stride
    dev = pkts.device
    f = {"bitmap": torch.empty(npk, dtype=torch.int32, device=dev),
         "count": torch.empty(npk, dtype=torch.uint8, device=dev),
         "flags": torch.empty(npk, dtype=torch.uint8, device=dev),
         "index": torch.empty(npk, dtype=torch.int32, device=dev),
         "switch_id": torch.empty(npk, dtype=torch.uint8, device=dev),
         "frag_id": torch.empty(npk, dtype=torch.int32, device=dev)}
    fs = _lib.NgaFields(*[f[k].data_ptr() for k in
                          ("bitmap", "count", "flags", "index", "switch_id", "frag_id")])
    vals = torch.empty(npk * V, dtype=torch.int32, device=dev) if with_values else None
    check(load().ina_unpack_nga(pkts.data_ptr(), npk, V, stride, C.byref(fs),
                                vals.data_ptr() if vals is not None else None, _stream(pkts)),
          "unpack_nga")
    return f, vals


def _check_apply(pkts, actions, V, local, out, acks):
    """Sizes the C ABI cannot see (raw pointers): checked here so a short buffer is a
    Python error, not an out-of-bounds device write."""
    if pkts.dim() != 2:
        raise ValueError("pkts must be [npkts, stride]")
    if actions.numel() < pkts.shape[0]:
        raise ValueError("actions must hold one byte per packet")
    _req(out, torch.float32, "out")
    if out.numel() != local.numel():
        raise ValueError("out must have local's size")
    tensors = [pkts, actions, local, out]
    if acks is not None:
        _req(acks, torch.uint8, "acks")
        if acks.dim() != 2 or acks.shape[1] < 16:
            raise ValueError("acks must be [rows, stride >= 16] (16-byte ack headers)")
        if acks.shape[0] < -(-local.numel() // V):
            raise ValueError("acks needs one row per slot: ceil(local.numel() / V) rows")
        tensors.append(acks)
    _same_device(*tensors)


def apply_completed(pkts: torch.Tensor, actions: torch.Tensor, V: int, seq0: int,
                    local: torch.Tensor, k: int, weight_step: float, out=None, acks=None):
    """PS side after Switch.process: completed slots (actions == ACT_FWD_AGG) are decoded,
    dequantised and applied: out[slot*V + j] = local + weight_step * sum * 2^-k, slot =
    frag_id - seq0.  With acks ([nslots, stride] uint8), row `slot` gets the PS ack header."""
    _req(pkts, torch.uint8, "pkts")
    _req(actions, torch.uint8, "actions")
    _req(local, torch.float32, "local")
    npk, stride = pkts.shape
    out = torch.empty_like(local) if out is None else out
    _fits(out, local.numel())
    _check_apply(pkts, actions, V, local, out, acks)
    ack_ptr, ack_stride = None, 0
    if acks is not None:
        ack_ptr, ack_stride = acks.data_ptr(), acks.shape[1]
    check(load().ina_apply_completed_nga(pkts.data_ptr(), npk, V, stride, actions.data_ptr(),
                                         seq0 & 0xFFFFFFFF, local.data_ptr(), k, float(weight_step),
                                         out.data_ptr(), local.numel(), ack_ptr, ack_stride,
                                         _stream(pkts)), "apply_completed")
    return out


def pack_c128(gradient: torch.Tensor, packet_num: int, worker_id: int, aggregator_index: int,
              tensor_index: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """communicator.cc's packet_t x packet_num as uint8 [packet_num, 524] (device)."""
    if gradient.dtype not in (torch.int32, torch.uint32):
        raise TypeError("gradient must be int32/uint32")
    if not gradient.is_cuda or not gradient.is_contiguous():
        raise ValueError("gradient must be a contiguous device tensor")
    if gradient.numel() < packet_num * 128:
        raise ValueError("gradient shorter than packet_num * 128")
    out = (torch.empty((packet_num, _lib.C128_BYTES), dtype=torch.uint8, device=gradient.device)
           if out is None else out)
    _req(out, torch.uint8, "out")
    _fits(out, packet_num * _lib.C128_BYTES)
    check(load().ina_pack_c128(gradient.data_ptr(), packet_num, worker_id,
                               aggregator_index & 0xFFFFFFFF, tensor_index, out.data_ptr(),
                               _stream(gradient)), "pack_c128")
    return out


# -- integrity --------------------------------------------------------------------------------
def checksum(x: torch.Tensor) -> torch.Tensor:
    """Device u32 (as int64 tensor view) of sum_i x[i]*(2i+1) mod 2^32."""
    _req(x, torch.int32, "x")
    out = torch.empty(1, dtype=torch.int32, device=x.device)
    check(load().ina_checksum_i32(x.data_ptr(), x.numel(), out.data_ptr(), _stream(x)), "checksum")
    return out


# -- dynamic scale ---------------------------------------------------------------------------
def absmax(x: torch.Tensor, base: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """Device float32 [1] = max_i |x[i] - base[i]| (base optional; NaN ignored)."""
    _req(x, torch.float32, "x")
    if base is not None:
        _req(base, torch.float32, "base")
        if base.numel() != x.numel():
            raise ValueError("base and x differ in length")
        _same_device(x, base)
    out = torch.empty(1, dtype=torch.float32, device=x.device) if out is None else out
    _fits(out, 1)
    _req(out, torch.float32, "out")
    check(load().ina_absmax_f32(x.data_ptr(), base.data_ptr() if base is not None else None,
                                x.numel(), out.data_ptr(), _stream(x)), "absmax")
    return out


def scale_for(amax: float, W: int, bits: int = 32) -> int:
    """Largest k in [-126, 127] such that no worker value and no W-way sum of 2^k fixed
    point values with |x| <= amax saturates at `bits` (32, or 16 for the int16 wire)."""
    k = C.c_int(0)
    check(load().ina_scale_for(float(amax), int(W), int(bits), C.byref(k)), "scale_for")
    return k.value


def absmax_multi(xs, base: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """Device float32 [1] = max_w,i |xs[w][i] - base[i]| over W buckets in ONE pass
    (ina_absmax_multi_f32: each base chunk is read once for all W workers)."""
    xs, n = _bufs(xs, torch.float32, "xs")
    if base is not None:
        _req(base, torch.float32, "base")
        if base.numel() != n:
            raise ValueError("base and xs differ in length")
        _same_device(xs[0], base)
    out = torch.empty(1, dtype=torch.float32, device=xs[0].device) if out is None else out
    _fits(out, 1)
    _req(out, torch.float32, "out")
    arr = ptr_array([x.data_ptr() for x in xs])
    check(load().ina_absmax_multi_f32(arr, len(xs), base.data_ptr() if base is not None else None,
                                      n, out.data_ptr(), _stream(xs[0])), "absmax_multi")
    return out


def scale_for_workers(xs, base: torch.Tensor | None = None, bits: int = 32) -> int:
    """k for W device buckets (deltas against `base` when given): one absmax_multi pass over
    all W buckets, one host read of the maximum."""
    xs = list(xs)
    m = absmax_multi(xs, base)
    return scale_for(float(m.item()), len(xs), bits)


# -- device packet-stream switch ---------------------------------------------------------------
class Switch:
    """ngaa.p4's aggregator with its registers in HBM (count u8, frag u32, V x u32 per slot)."""

    def __init__(self, V: int = 32, num_slots: int = NUM_REGISTER, switch_id: int = 1,
                 device: str | torch.device = "cuda", write_dropped: bool = False):
        """write_dropped=True also rewrites dropped packets with their running sums (what
        the P4 deparser emits before the drop); the default skips those unobservable writes."""
        self.V, self.num_slots, self.switch_id = V, num_slots, switch_id
        self.count = torch.zeros(num_slots, dtype=torch.uint8, device=device)
        self.frag = torch.zeros(num_slots, dtype=torch.int32, device=device)
        self.regs = torch.zeros((num_slots, V), dtype=torch.int32, device=device)
        self._state = _lib.SwitchState(num_slots, V, switch_id, int(write_dropped),
                                       self.count.data_ptr(), self.frag.data_ptr(),
                                       self.regs.data_ptr())
        self._scratch = None
        self._sorted = None        # (batch, scratch) of a sort() awaiting its run()
        # the scratch (key / id arrays, epochs, run table) is reused by every call: an event
        # recorded after each call, waited on by the next call's stream when that stream
        # differs, so a sort queued on a side stream never overwrites what a run on the main
        # stream still reads (and a run never starts before its side-stream sort)
        self._done = None
        self._done_stream = None
        self._sorted_desc = None

    def _begin(self, ts: torch.cuda.Stream) -> int:
        """Orders this call after the previous call on the scratch; returns ts's handle."""
        if self._done is not None and self._done_stream != ts.cuda_stream:
            ts.wait_event(self._done)
        return ts.cuda_stream

    def _end(self, ts: torch.cuda.Stream) -> None:
        if self._done is None:
            self._done = torch.cuda.Event()
        self._done.record(ts)
        self._done_stream = ts.cuda_stream

    def _call(self, ts, rows, pay, npk, stride, d, actions, scratch, phase, ps=None, what="switch"):
        """One ina_switch call (include/ina.h): the batch struct, the PS step (or None), the
        phase -- ordered after the previous call on this switch's scratch."""
        b = _lib.SwitchBatch(rows.data_ptr(), pay.data_ptr() if pay is not None else None, npk, stride,
                             d.data_ptr() if d is not None else None, actions.data_ptr(), scratch.data_ptr())
        st = self._begin(ts)
        check(load().ina_switch(C.byref(self._state), C.byref(b), C.byref(ps) if ps is not None else None,
                                phase, st), what)
        self._end(ts)

    @staticmethod
    def _ps(seq0, local, k, weight_step, out, ack_ptr, ack_stride, ack_desc_ptr, keep_forwarded):
        return _lib.SwitchPs(seq0 & 0xFFFFFFFF, k, weight_step, local.data_ptr(), out.data_ptr(), local.numel(),
                             ack_ptr, ack_stride, ack_desc_ptr, int(keep_forwarded))

    def process(self, pkts: torch.Tensor, actions: torch.Tensor | None = None,
                desc: torch.Tensor | None = None) -> torch.Tensor:
        """Runs packets (uint8 [npkts, stride], arrival order) through the switch in place;
        returns the uint8 action per packet (ACT_*).  desc: the batch's descriptors
        (int64 [npkts], pack_nga(desc=True) / nga_descriptors) -- the slot sort then reads
        them instead of the packet headers; results identical."""
        _req(pkts, torch.uint8, "pkts")
        npk, stride = pkts.shape
        d = _desc_arg(desc, npk, pkts.device)
        actions = torch.empty(npk, dtype=torch.uint8, device=pkts.device) if actions is None else actions
        _req(actions, torch.uint8, "actions")
        if actions.numel() < npk:
            raise ValueError("actions must hold one byte per packet")
        _same_device(pkts, actions)
        need = load().ina_switch_scratch_bytes(npk, self.num_slots)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=pkts.device)
        self._sorted = None                       # the scratch is reused below
        self._call(torch.cuda.current_stream(pkts.device), pkts, None, npk, stride, d, actions, self._scratch,
                   _lib.INA_SWITCH_ALL, what="switch_process")
        return actions

    def batch_path(self, npk: int) -> str:
        """Which slot-sort path the last call over this switch's scratch took for its batch of
        npk packets (batches past the one-workgroup small-batch paths): "in_order" (no sort),
        "runs" (dense ascending runs, no sort), "local" (near-sorted: per-slot lists, no sort)
        or "sorted" (the bucket sort or the LSD digit passes).  Synchronises the device (a diagnostic)."""
        if self._scratch is None:
            raise ValueError("no batch has run on this switch")
        torch.cuda.synchronize(self._scratch.device)
        p = C.c_int(0)
        check(load().ina_switch_batch_path(self._scratch.data_ptr(), npk, self.num_slots, C.byref(p)),
              "switch_batch_path")
        return {1: "in_order", 2: "runs", 3: "sorted", 4: "local"}[p.value]

    def _scratch_for(self, npk, dev):
        need = load().ina_switch_scratch_bytes(npk, self.num_slots)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=dev)
        return self._scratch

    def sort(self, pkts: torch.Tensor, desc: torch.Tensor, actions: torch.Tensor | None = None,
             stream: torch.cuda.Stream | None = None) -> torch.Tensor:
        """The slot sort of process(pkts, desc=desc) alone (ina_switch, INA_SWITCH_SORT): it reads
        only the descriptors, so it may be queued before -- or on `stream`, beside -- the
        kernels still filling pkts' payload; run() / run_apply() finish the batch over the
        same scratch (the scratch is this switch's, one batch at a time).  Every call on this
        switch records an event that the next call's stream waits on when the streams
        differ, so a sort on a side stream starts after the previous run and run() after its
        sort without the caller ordering them.  Returns the actions tensor to hand to run()."""
        _req(pkts, torch.uint8, "pkts")
        npk, stride = pkts.shape
        d = _desc_arg(desc, npk, pkts.device)
        if d is None:
            raise ValueError("sort() needs the batch's descriptors")
        actions = torch.empty(npk, dtype=torch.uint8, device=pkts.device) if actions is None else actions
        _req(actions, torch.uint8, "actions")
        _fits(actions, npk, "actions")
        _same_device(pkts, actions)
        scratch = self._scratch_for(npk, pkts.device)
        ts = stream if stream is not None else torch.cuda.current_stream(pkts.device)
        if stream is not None:
            scratch.record_stream(stream)        # in use there until run() joins it
        self._call(ts, pkts, None, npk, stride, d, actions, scratch, _lib.INA_SWITCH_SORT, what="switch_sort")
        self._sorted = (pkts.data_ptr(), npk, stride, actions.data_ptr(), scratch.data_ptr())
        self._sorted_desc = d
        return actions

    def check_sorted_desc(self, pkts: torch.Tensor) -> None:
        """Optional guard for the two-phase switch: the descriptors sort() ordered the batch
        by (typically made from the header parameters by make_descriptors) must equal the
        packed headers' bytes 4..11 (nga_descriptors).  A mismatch (wrong seq0, num_slots,
        count or switch id) would aggregate into the wrong slots silently, so it raises
        ValueError.  Call between sort() and run(); synchronises the device."""
        if self._sorted is None:
            raise ValueError("check_sorted_desc() needs a sort() awaiting its run()")
        got = nga_descriptors(pkts)
        if not torch.equal(got, self._sorted_desc[: got.numel()]):
            bad = int((got != self._sorted_desc[: got.numel()]).nonzero()[0])
            raise ValueError(f"sort() descriptors disagree with the packed headers (first at packet {bad})")

    def _take_sorted(self, pkts, actions):
        # the run reads the sort's scratch as it stands: a run without its own sort (or for
        # another batch) would read stale packet ids, so the pairing is enforced here
        npk, stride = pkts.shape
        want = (pkts.data_ptr(), npk, stride, actions.data_ptr(),
                self._scratch.data_ptr() if self._scratch is not None else None)
        if self._sorted != want:
            raise ValueError("run() / run_apply() must follow sort() of the same batch and actions")
        self._sorted = None
        return self._scratch

    def run(self, pkts: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
        """Second phase of process(): the batch sort() sorted, run over its scratch."""
        _req(pkts, torch.uint8, "pkts")
        _req(actions, torch.uint8, "actions")
        npk, stride = pkts.shape
        _fits(actions, npk, "actions")
        _same_device(pkts, actions)
        scratch = self._take_sorted(pkts, actions)
        self._call(torch.cuda.current_stream(pkts.device), pkts, None, npk, stride, None, actions, scratch,
                   _lib.INA_SWITCH_RUN, what="switch_run")
        return actions

    def run_apply(self, pkts: torch.Tensor, actions: torch.Tensor, seq0: int, local: torch.Tensor,
                  k: int, weight_step: float, out: torch.Tensor | None = None,
                  acks: torch.Tensor | None = None, keep_forwarded: bool = True,
                  ack_desc: torch.Tensor | None = None):
        """Second phase of process_apply() after sort().  Returns (actions, out)."""
        _req(pkts, torch.uint8, "pkts")
        _req(local, torch.float32, "local")
        npk, stride = pkts.shape
        _req(actions, torch.uint8, "actions")
        out = torch.empty_like(local) if out is None else out
        _fits(out, local.numel())
        _check_apply(pkts, actions, self.V, local, out, acks)
        ack_ptr, ack_stride = (acks.data_ptr(), acks.shape[1]) if acks is not None else (None, 0)
        ad = _ack_desc_arg(ack_desc, acks)
        scratch = self._take_sorted(pkts, actions)
        self._call(torch.cuda.current_stream(pkts.device), pkts, None, npk, stride, None, actions, scratch,
                   _lib.INA_SWITCH_RUN, self._ps(seq0, local, k, weight_step, out, ack_ptr, ack_stride, ad,
                                                 keep_forwarded), what="switch_run_apply")
        return actions, out

    def process_apply(self, pkts: torch.Tensor, seq0: int, local: torch.Tensor, k: int,
                      weight_step: float, out: torch.Tensor | None = None,
                      acks: torch.Tensor | None = None, keep_forwarded: bool = True,
                      actions: torch.Tensor | None = None, desc: torch.Tensor | None = None,
                      ack_desc: torch.Tensor | None = None):
        """process() + apply_completed() in one pass (the PS on the switch's GPU): completed
        slots update out = local + weight_step * sum * 2^-k and write their PS ack rows.
        keep_forwarded=False leaves completed packets as they arrived (consumed here).
        ack_desc (int64 [ack rows]): also written beside every ack row -- its descriptor, as
        nga_descriptors(acks) would give -- for the next batch's sort.  Returns (actions, out)."""
        _req(pkts, torch.uint8, "pkts")
        _req(local, torch.float32, "local")
        npk, stride = pkts.shape
        actions = torch.empty(npk, dtype=torch.uint8, device=pkts.device) if actions is None else actions
        _req(actions, torch.uint8, "actions")
        out = torch.empty_like(local) if out is None else out
        _fits(out, local.numel())
        _check_apply(pkts, actions, self.V, local, out, acks)
        d = _desc_arg(desc, npk, pkts.device)
        ack_ptr, ack_stride = None, 0
        if acks is not None:
            ack_ptr, ack_stride = acks.data_ptr(), acks.shape[1]
        need = load().ina_switch_scratch_bytes(npk, self.num_slots)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=pkts.device)
        self._sorted = None
        ad = _ack_desc_arg(ack_desc, acks)
        self._call(torch.cuda.current_stream(pkts.device), pkts, None, npk, stride, d, actions, self._scratch,
                   _lib.INA_SWITCH_ALL, self._ps(seq0, local, k, weight_step, out, ack_ptr, ack_stride, ad,
                                                 keep_forwarded), what="switch_process_apply")
        return actions, out


    def process_split(self, hdr: torch.Tensor, pay: torch.Tensor, actions: torch.Tensor | None = None,
                      desc: torch.Tensor | None = None) -> torch.Tensor:
        """process() over split rows (ina_switch, batch.pay set): header rows uint8 [npkts, 16]
        and payload rows uint8 [npkts, 4V]; same actions, registers and forwarded bytes."""
        npk = hdr.shape[0]
        hdr, pay = _split_rows(npk, self.V, hdr.device, hdr, pay)
        d = _desc_arg(desc, npk, hdr.device)
        actions = torch.empty(npk, dtype=torch.uint8, device=hdr.device) if actions is None else actions
        _req(actions, torch.uint8, "actions")
        _fits(actions, npk, "actions")
        _same_device(hdr, pay, actions)
        scratch = self._scratch_for(npk, hdr.device)
        self._sorted = None
        self._call(torch.cuda.current_stream(hdr.device), hdr, pay, npk, 16, d, actions, scratch,
                   _lib.INA_SWITCH_ALL, what="switch_process_split")
        return actions

    def process_apply_split(self, hdr: torch.Tensor, pay: torch.Tensor, seq0: int, local: torch.Tensor,
                            k: int, weight_step: float, out: torch.Tensor | None = None,
                            ack_hdr: torch.Tensor | None = None, ack_desc: torch.Tensor | None = None,
                            keep_forwarded: bool = True, actions: torch.Tensor | None = None,
                            desc: torch.Tensor | None = None):
        """process_apply() over split rows (ina_switch with batch.pay and a PS step): the PS ack rows are
        header rows (uint8 [slots, 16]) with their descriptors in ack_desc.  Returns (actions, out)."""
        _req(local, torch.float32, "local")
        npk = hdr.shape[0]
        hdr, pay = _split_rows(npk, self.V, hdr.device, hdr, pay)
        actions = torch.empty(npk, dtype=torch.uint8, device=hdr.device) if actions is None else actions
        _req(actions, torch.uint8, "actions")
        _fits(actions, npk, "actions")
        out = torch.empty_like(local) if out is None else out
        _req(out, torch.float32, "out")
        if out.numel() != local.numel():
            raise ValueError("out must have local's size")
        if ack_hdr is not None:
            _req(ack_hdr, torch.uint8, "ack_hdr")
            if ack_hdr.dim() != 2 or ack_hdr.shape[1] != 16 or ack_hdr.shape[0] < -(-local.numel() // self.V):
                raise ValueError("ack_hdr must be uint8 [>= ceil(local.numel() / V), 16] header rows")
        d = _desc_arg(desc, npk, hdr.device)
        ad = _ack_desc_arg(ack_desc, ack_hdr)
        _same_device(hdr, pay, actions, local, out, *([ack_hdr] if ack_hdr is not None else []))
        scratch = self._scratch_for(npk, hdr.device)
        self._sorted = None
        self._call(torch.cuda.current_stream(hdr.device), hdr, pay, npk, 16, d, actions, scratch,
                   _lib.INA_SWITCH_ALL,
                   self._ps(seq0, local, k, weight_step, out, ack_hdr.data_ptr() if ack_hdr is not None else None,
                            16, ad, keep_forwarded), what="switch_process_apply_split")
        return actions, out


def route_ipv4(actions: torch.Tensor, keys: torch.Tensor, ports: torch.Tensor,
               dst_ip: torch.Tensor | None = None, dst_default: int = 0,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """ipRoute (ngaa.p4:39-61) for a switched batch: int32 egress port per packet
    (PORT_DROP for ingress drops, drop rows and table misses; PORT_NONE for NoAction).
    keys uint32-valued int32/int64 IPv4 addresses and ports int32 (<= 256 rows, on the
    device); dst_ip per packet (int32 view of the u32 address) or None for dst_default."""
    _req(actions, torch.uint8, "actions")
    _req(keys, torch.int32, "keys")
    _req(ports, torch.int32, "ports")
    if keys.numel() != ports.numel() or keys.numel() > _lib.ROUTE_MAX:
        raise ValueError(f"route table: keys/ports must match and hold <= {_lib.ROUTE_MAX} rows")
    if dst_ip is not None:
        _req(dst_ip, torch.int32, "dst_ip")
        if dst_ip.numel() != actions.numel():
            raise ValueError("dst_ip must hold one address per packet")
    out = torch.empty(actions.numel(), dtype=torch.int32, device=actions.device) if out is None else out
    _fits(out, actions.numel())
    _req(out, torch.int32, "out")
    _same_device(actions, keys, ports, out, *([dst_ip] if dst_ip is not None else []))
    check(load().ina_route_ipv4(actions.data_ptr(), None if dst_ip is None else dst_ip.data_ptr(),
                                dst_default & 0xFFFFFFFF, actions.numel(), keys.data_ptr(),
                                ports.data_ptr(), keys.numel(), out.data_ptr(), _stream(actions)),
          "route_ipv4")
    return out


def set_tuning(max_blocks: int | None = None, unroll: int | None = None,
               nontemporal: bool | None = None, reduce_blocks: int | None = None,
               stream_blocks: int | None = None, combine_blocks: int | None = None,
               combine_ina_blocks: int | None = None, h2d_streams: int | None = None,
               launch_chunks: int | None = None, switch_small_sort: bool | int | None = None,
               switch_window: int | None = None, switch_ack_fast: bool | None = None,
               switch_sort: int | None = None, switch_sort_rounds: int | None = None,
               ew_blocks: int | None = None, switch_tiny_max: int | None = None,
               host_zero_copy: bool | None = None, switch_bucket_tile: int | None = None,
               switch_runs: bool | None = None, switch_pre_all: bool | None = None,
               switch_local: bool | None = None, switch_decide_delay_us: int | None = None):
    """Launch-geometry knobs (results never change, only speed): max_blocks caps the
    grid of the elementwise kernels, reduce_blocks that of the sum-reduce (0 = the
    measured 64*W rule), stream_blocks the chunk-loop kernels, combine_blocks the fp32
    PS combine, combine_ina_blocks the INA-semantics combine, h2d_streams the host-ingest
    pipeline's H2D copy streams (1 or 2), launch_chunks the 16-byte chunks one flat packet
    kernel launch covers (default 2^31 - 1; smaller values only split launches),
    switch_small_sort the one-workgroup key+sort path for small switch batches (False or 0:
    off; True or 1: the default threshold, 768 packets -- 1 is the C ABI's sentinel for
    the default, not "batches of one packet"; an int 2..2048: up to that many),
    switch_window the sorted positions one wave of the switch run kernel owns (0 = auto,
    1..64), switch_ack_fast the lane-parallel path for PS acks alone in their slot's
    segment, switch_sort the slot sort (0 auto = chunk + bucket sort where the keys have
    one or two digits, 3 the LSD digit passes for every batch), switch_sort_rounds the
    sort chunk (64-item rounds per wave: 0 auto, 4, 8, 16), ew_blocks the grid cap of the
    one-in one-out elementwise kernels (default 2^24: one 16-byte chunk per thread),
    switch_tiny_max the largest batch the switch sorts and runs in ONE launch of one
    workgroup (0 = off, at most 2048) -- only batches that take the small-sort path at all
    reach it, so it is capped by switch_small_sort's threshold; host_zero_copy lets
    sum_reduce_host reduce pinned, device-mapped host buffers in place over PCIe (True,
    the default) instead of through the chunked copy pipeline; switch_bucket_tile the slot
    sort's bucket tile in 64-item rounds per wave (0 = auto: 8 when the average bucket
    exceeds 3,584 packets, else 4; or 4, 8); switch_runs lets batches of at most 64 runs of
    consecutive slots (worker-major arrival, PS acks in front) skip the slot sort (True, the
    default; False always sorts); switch_pre_all splits the sort's first pass into detection,
    decision and digits for every key width (True, the default; False: keys of 19-22 bits only);
    switch_local lets near-sorted batches (V <= 32, local disorder) run from per-slot lists
    without a sort (True, the default); switch_decide_delay_us (tests) delays the near-sorted
    decision so the digit pass's bounded wait for it runs out (0, the default); unroll is the sum-reduce's 16-byte chunks per worker
    per thread.  Each switch batch reads the switch keys once (a run() follows what its sort()
    recorded).  stream_blocks, combine_blocks, combine_ina_blocks, ew_blocks and switch_window
    are grid-cap sweeps that only lab builds of the library accept (make EXTRA=-DINA_LAB_KEYS=1);
    the product library refuses them (RuntimeError)."""
    lib = load()
    if reduce_blocks is not None:
        check(lib.ina_set_tuning(3, int(reduce_blocks)), "set_tuning")
    if stream_blocks is not None:
        check(lib.ina_set_tuning(4, int(stream_blocks)), "set_tuning")
    if combine_blocks is not None:
        check(lib.ina_set_tuning(5, int(combine_blocks)), "set_tuning")
    if combine_ina_blocks is not None:
        check(lib.ina_set_tuning(6, int(combine_ina_blocks)), "set_tuning")
    if h2d_streams is not None:
        check(lib.ina_set_tuning(7, int(h2d_streams)), "set_tuning")
    if launch_chunks is not None:
        check(lib.ina_set_tuning(8, int(launch_chunks)), "set_tuning")
    if switch_small_sort is not None:
        check(lib.ina_set_tuning(9, int(switch_small_sort)), "set_tuning")   # True -> 1: the default
    if switch_window is not None:
        check(lib.ina_set_tuning(10, int(switch_window)), "set_tuning")
    if switch_ack_fast is not None:
        check(lib.ina_set_tuning(11, int(bool(switch_ack_fast))), "set_tuning")
    if switch_sort is not None:
        check(lib.ina_set_tuning(12, int(switch_sort)), "set_tuning")
    if switch_sort_rounds is not None:
        check(lib.ina_set_tuning(13, int(switch_sort_rounds)), "set_tuning")
    if ew_blocks is not None:
        check(lib.ina_set_tuning(14, int(ew_blocks)), "set_tuning")
    if switch_tiny_max is not None:
        check(lib.ina_set_tuning(15, int(switch_tiny_max)), "set_tuning")
    if host_zero_copy is not None:
        check(lib.ina_set_tuning(16, int(bool(host_zero_copy))), "set_tuning")
    if switch_bucket_tile is not None:
        check(lib.ina_set_tuning(17, int(switch_bucket_tile)), "set_tuning")
    if switch_runs is not None:
        check(lib.ina_set_tuning(18, int(bool(switch_runs))), "set_tuning")
    if switch_pre_all is not None:
        check(lib.ina_set_tuning(19, int(bool(switch_pre_all))), "set_tuning")
    if switch_local is not None:
        check(lib.ina_set_tuning(20, int(bool(switch_local))), "set_tuning")
    if switch_decide_delay_us is not None:
        check(lib.ina_set_tuning(21, int(switch_decide_delay_us)), "set_tuning")
    if max_blocks is not None:
        check(lib.ina_set_tuning(0, int(max_blocks)), "set_tuning")
    if unroll is not None:
        check(lib.ina_set_tuning(1, int(unroll)), "set_tuning")
    if nontemporal is not None:
        check(lib.ina_set_tuning(2, int(bool(nontemporal))), "set_tuning")


def version() -> str:
    return load().ina_version().decode()
