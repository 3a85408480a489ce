"""Multi-GPU aggregation of one bucket that outgrows a GPU (BASELINE config 5).

Layout A of SURVEY.md 8e (ShardedAggregator): every rank is one worker holding its full fp32
gradient bucket.  Each rank quantises its bucket on its GPU, RCCL reduce-scatters
the integers with SUM over xGMI, the owner of each shard decodes it, and an
all-gather returns the full aggregate to every rank (the PS broadcast).  The
switch aggregates every slot independently (ngaa.p4:87-168), so contiguous slot
ranges can live on different GPUs.

Two wires:
  "i32"  int32 fixed point (2^k).  Integer addition mod 2^32 is associative and
         commutative, so the shard each rank receives is bit-identical to the
         switch's per-slot sum (processor.p4:14-24) in any ring or tree order.
  "i16"  config 4's int16 saturating quantiser.  Saturation is not associative,
         so int16 values never go through the collective: each rank sends the
         int32 wire q16 + (saturated << 22) (ina_quantize_f32_i16_wire), the SUM
         carries the exact int16 sum and the count of saturating ranks together,
         and the owner saturates once and sets the per-slot overflow flag (the
         ngaa_h overflow bit, headers.p4:30) -- bit-identical to the single-GPU
         ina_quantize_reduce_f32_i16_sat over the same W buckets.  The all-gather
         then moves the saturated int16 sums (2 bytes a value, half of fp32's xGMI
         bytes) and the flags, and every rank dequantises the gathered int16 vector
         (an HBM pass of 6 bytes a value, cheap next to the xGMI bytes it saves).

Layout B (RangeAggregator): the workers' buckets arrive already split by range -- rank
r holds every worker's slice of slot range r -- so each rank reduces its W slices
locally with the fused quantise + reduce kernel (no reduce-scatter), decodes, and one
all-gather returns the full aggregate; the xGMI traffic is that all-gather alone (fp32
on the i32 wire; the int16 sums + flags, decoded after the gather, on the i16 wire).

Shards are contiguous slot ranges padded to `align` values (default 1024 values =
4 KiB, rounded up to a whole number of V-value slots), so no slot straddles two
ranks.  The collective plumbing (ShardPlan, reduce_scatter_sum, all_gather_shards)
is device-agnostic and covered on CPU with gloo; with a gloo group and device
tensors the collectives stage through host memory (a test harness for several
ranks on one GPU, never the RCCL path).  Quantise and decode are the device
kernels (no CPU path).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import _lib, ops


class ShardPlan:
    def __init__(self, n: int, world: int, align: int = 1024):
        if n < 0 or world < 1 or align < 1:
            raise ValueError("bad shard plan")
        self.n, self.world, self.align = n, world, align
        per = -(-n // world) if n else 0
        self.shard = -(-per // align) * align
        self.padded = self.shard * world

    def range_of(self, rank: int):
        lo = min(rank * self.shard, self.n)
        return lo, min(lo + self.shard, self.n)


def _host_staged(group) -> bool:
    return dist.get_backend(group) == "gloo"


def reduce_scatter_sum(x_padded: torch.Tensor, plan: ShardPlan, group=None, out=None,
                       async_op: bool = False):
    """int32 [padded] -> this rank's [shard] of the element-wise sum over ranks.  With
    async_op the RCCL work handle is returned as well ((out, work); work is None when
    the call completed synchronously): the collective runs on RCCL's stream and the
    caller's stream waits for it only at work.wait()."""
    if x_padded.numel() != plan.padded:
        raise ValueError("input must be padded to plan.padded")
    out = torch.empty(plan.shard, dtype=x_padded.dtype, device=x_padded.device) if out is None else out
    work = None
    if plan.world == 1:
        out.copy_(x_padded)
    elif x_padded.is_cuda and _host_staged(group):
        h = torch.empty(plan.shard, dtype=x_padded.dtype)
        dist.reduce_scatter_tensor(h, x_padded.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(h)
    else:
        work = dist.reduce_scatter_tensor(out, x_padded, op=dist.ReduceOp.SUM, group=group,
                                          async_op=async_op)
    return (out, work) if async_op else out


def reduce_scatter_a2a(x_padded: torch.Tensor, plan: ShardPlan, group=None, out=None, recv=None):
    """int32 [padded] -> this rank's [shard] of the element-wise sum over ranks, as ONE
    all-to-all (rank r's slice j goes straight to rank j: on a fully connected xGMI mesh
    every pair of GPUs has its own link, so all 7 links carry (G-1)/G x S at once instead
    of a ring's hops) followed by the device W-way wrapping sum of the G received slices
    (ina_sum_reduce_i32, HBM-bound) -- the same bits as the RCCL SUM (mod-2^32 adds in any
    order).  recv: a [padded] int32 scratch (allocated when None)."""
    if x_padded.numel() != plan.padded:
        raise ValueError("input must be padded to plan.padded")
    out = torch.empty(plan.shard, dtype=torch.int32, device=x_padded.device) if out is None else out
    if plan.world == 1:
        out.copy_(x_padded)
        return out
    recv = torch.empty(plan.padded, dtype=torch.int32, device=x_padded.device) if recv is None else recv
    if x_padded.is_cuda and _host_staged(group):
        h = torch.empty(plan.padded, dtype=torch.int32)
        dist.all_to_all_single(h, x_padded.cpu(), group=group)
        recv.copy_(h)
    else:
        dist.all_to_all_single(recv, x_padded, group=group)
    parts = [recv[r * plan.shard:(r + 1) * plan.shard] for r in range(plan.world)]
    if out.is_cuda:
        ops.sum_reduce(parts, out=out)
    else:                                       # CPU tensors (the gloo tests): the same sum
        acc = parts[0].to(torch.int64)
        for q in parts[1:]:
            acc += q
        out.copy_(((acc + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32))
    return out


def all_reduce_sum(x: torch.Tensor, group=None):
    """int32 in place -> the element-wise sum over ranks (RCCL all-reduce; host-staged
    with gloo and device tensors)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    if x.is_cuda and _host_staged(group):
        h = x.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        x.copy_(h)
        return x
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    return x


def all_gather_shards(shard: torch.Tensor, plan: ShardPlan, group=None, out=None,
                      async_op: bool = False):
    """[count] per rank -> [world * count] (count = plan.shard values, or its slot flags).
    async_op: returns (out, work) as reduce_scatter_sum does."""
    out = torch.empty(plan.world * shard.numel(), dtype=shard.dtype, device=shard.device) \
        if out is None else out
    work = None
    if plan.world == 1:
        out.copy_(shard)
    elif _host_staged(group):
        # gloo gathers bytes: an all-gather only moves data, so any dtype (gloo has no
        # int16) goes through as its uint8 view, bit for bit
        h = torch.empty(out.numel() * out.element_size(), dtype=torch.uint8)
        dist.all_gather_into_tensor(h, shard.contiguous().cpu().view(torch.uint8), group=group)
        out.copy_(h.view(out.dtype).view(out.shape))
    elif shard.dtype == torch.int16:
        # RCCL has no int16 type; a gather only moves bytes, so int16 goes as its uint8 view
        work = dist.all_gather_into_tensor(out.view(torch.uint8), shard.contiguous().view(torch.uint8),
                                           group=group, async_op=async_op)
    else:
        work = dist.all_gather_into_tensor(out, shard, group=group, async_op=async_op)
    return (out, work) if async_op else out


def _wait(work):
    if work is not None:
        work.wait()          # the caller's stream waits for RCCL's; the host does not block


class ShardedAggregator:
    """Reusable buffers for repeated sharded aggregation of same-sized buckets.

    wire="i32": __call__ returns the dequantised fp32 sum over ranks.
    wire="i16": the same from the int16 saturating path; `overflow` then holds the
    per-slot flags (ceil(n / V) bytes) of the last call.
    collective="rs_ag" (default): reduce-scatter the integer wire, the owner decodes its
    shard, all-gather.  collective="a2a": the reduce-scatter as one all-to-all of the wire
    slices plus the device sum of the G received slices (reduce_scatter_a2a), then the
    same decode and all-gather.  collective="allreduce": one RCCL all-reduce of the
    integer wire (the same (G-1)/G bytes each way per rank inside one collective) and
    every rank decodes the whole bucket.  All give the same bits; which one xGMI runs
    faster is measured by bench.py at N > 1 (sharded_c5 / .a2a / .allreduce).
    chunks=C > 1 (rs_ag, world > 1): the bucket is cut into C contiguous chunks, each
    reduce-scattered and all-gathered on its own (async RCCL work), so chunk c+1's
    quantise runs under chunk c's reduce-scatter and the decodes under the later
    collectives; same bits (integer sums are order-free, the decode is elementwise).
    """

    def __init__(self, n: int, k: int = 16, group=None, device=None, align: int = 1024,
                 wire: str = "i32", V: int = 256, collective: str = "rs_ag", chunks: int = 1):
        if wire not in ("i32", "i16"):
            raise ValueError("wire must be 'i32' or 'i16'")
        if collective not in ("rs_ag", "a2a", "allreduce"):
            raise ValueError("collective must be 'rs_ag', 'a2a' or 'allreduce'")
        if chunks < 1 or (chunks > 1 and collective != "rs_ag"):
            raise ValueError("chunks must be >= 1, and > 1 only with collective='rs_ag'")
        self.collective = collective
        if V <= 0:
            raise ValueError("V must be > 0")
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if wire == "i16" and self.world > _lib.I16_WIRE_MAX_RANKS:
            raise ValueError(f"the int16 wire sums at most {_lib.I16_WIRE_MAX_RANKS} ranks")
        if wire == "i16":
            align = align * V // math.gcd(align, V)        # shards hold whole slots
        self.plan = ShardPlan(n, self.world, align)
        self.k, self.group, self.wire, self.V = k, group, wire, V
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.chunks = chunks if self.world > 1 else 1
        tot = self.plan.padded
        if self.chunks > 1:
            # chunk c = values [c*L, (c+1)*L), L = world * Sc; rank r owns [c*L + r*Sc, +Sc)
            sc = -(-n // (self.world * self.chunks)) if n else 0
            self.sc = max(-(-sc // align) * align, align)
            self.cplan = ShardPlan(self.world * self.sc, self.world, align=self.sc)
            self.cpad = self.chunks * self.cplan.padded
            tot = max(tot, self.cpad)
        # one allocation backs both the whole-bucket and the chunked views; pad stays 0
        self._qbuf = torch.zeros(tot, dtype=torch.int32, device=dev)
        self._fbuf = torch.empty(tot, dtype=torch.float32, device=dev)
        self.q, self.full = self._qbuf[: self.plan.padded], self._fbuf[: self.plan.padded]
        # whole-bucket shard buffers (sum_shard, f_shard, s16_shard): used by the unchunked
        # step, aggregate_int and the phase_* methods; the pipelined step (chunks > 1) has
        # its own per-chunk buffers, so there they are allocated on first use only
        self._dev = dev
        self._shard_bufs = {}
        if self.chunks == 1:                     # allocate now, outside any timed step
            self._shard_buf("sum", torch.int32)
            self._shard_buf("f", torch.float32)
        if wire == "i16":
            self.slots_per_shard = self.plan.shard // V
            self.ovf_shard = torch.empty(self.slots_per_shard, dtype=torch.uint8, device=dev)
            self._obuf = torch.zeros(tot // V, dtype=torch.uint8, device=dev)
            self.ovf_full = self._obuf[: self.slots_per_shard * self.world]
            if self.world > 1 and collective != "allreduce":   # gather int16 sums, decode after
                if self.chunks == 1:
                    self._shard_buf("s16", torch.int16)
                self._s16buf = torch.empty(tot, dtype=torch.int16, device=dev)
                self.s16_full = self._s16buf[: self.plan.padded]
        # the all-to-all's receive buffer (world slices of one shard each)
        self._recv = (torch.empty(self.plan.padded, dtype=torch.int32, device=dev)
                      if collective == "a2a" and self.world > 1 else None)
        if self.chunks > 1:
            m = self.chunks * self.sc
            self.sum_c = torch.empty(m, dtype=torch.int32, device=dev)
            if wire == "i32":
                self.f_c = torch.empty(m, dtype=torch.float32, device=dev)
            else:
                self.s16_c = torch.empty(m, dtype=torch.int16, device=dev)
                self.ovf_c = torch.empty(m // V, dtype=torch.uint8, device=dev)

    def _shard_buf(self, name, dtype):
        b = self._shard_bufs.get(name)
        if b is None:
            b = self._shard_bufs[name] = torch.empty(self.plan.shard, dtype=dtype, device=self._dev)
        return b

    @property
    def sum_shard(self) -> torch.Tensor:
        """This rank's int32 shard of the summed wire (whole-bucket step)."""
        return self._shard_buf("sum", torch.int32)

    @property
    def f_shard(self) -> torch.Tensor:
        return self._shard_buf("f", torch.float32)

    @property
    def s16_shard(self) -> torch.Tensor:
        return self._shard_buf("s16", torch.int16)

    @property
    def overflow(self) -> torch.Tensor:
        """Per-slot overflow flags of the last i16 aggregation (ceil(n / V) bytes)."""
        if self.wire != "i16":
            raise AttributeError("overflow flags exist only on the i16 wire")
        return self._obuf[: -(-self.plan.n // self.V)]

    @property
    def gather_bytes(self) -> int:
        """Bytes one all-gather step brings to each rank over xGMI (values + flags);
        with collective="allreduce" the all-reduce's gather half (int32 wire words)."""
        if self.world == 1:
            return 0
        shard = self.chunks * self.sc if self.chunks > 1 else self.plan.shard
        if self.collective == "allreduce":
            return (self.world - 1) * shard * 4
        per = shard * (2 if self.wire == "i16" else 4)
        if self.wire == "i16":
            per += shard // self.V
        return (self.world - 1) * per

    # The step's phases, in order (bench.py times each one between HIP events).
    def phase_quantize(self, grad: torch.Tensor):
        self._quantize(grad)

    def phase_reduce_scatter(self):
        """The integer collective: reduce-scatter, or the whole all-reduce."""
        if self.world == 1:
            return
        if self.collective == "allreduce":
            all_reduce_sum(self.q, self.group)
        elif self.collective == "a2a":
            reduce_scatter_a2a(self.q, self.plan, self.group, out=self.sum_shard, recv=self._recv)
        else:
            reduce_scatter_sum(self.q, self.plan, self.group, out=self.sum_shard)

    def phase_decode(self):
        """The owner's decode of its shard (one rank, or after an all-reduce: the whole
        bucket on every rank)."""
        if self.world == 1 or self.collective == "allreduce":
            self._decode(self.q, self.full, self.ovf_full if self.wire == "i16" else None)
        elif self.wire == "i32":
            ops.dequantize(self.sum_shard, self.k, out=self.f_shard)
        else:
            ops.i16_wire_finish(self.sum_shard, self.k, self.V, out16=self.s16_shard,
                                overflow=self.ovf_shard, want_y=False)

    def phase_all_gather(self):
        if self.world == 1 or self.collective == "allreduce":
            return
        if self.wire == "i32":
            all_gather_shards(self.f_shard, self.plan, self.group, out=self.full)
        else:
            all_gather_shards(self.s16_shard, self.plan, self.group, out=self.s16_full)
            all_gather_shards(self.ovf_shard, self.plan, self.group, out=self.ovf_full)

    def phase_expand(self):
        """i16 wire at world > 1: dequantise the gathered int16 sums on every rank."""
        if self.world > 1 and self.wire == "i16" and self.collective != "allreduce":
            ops.dequantize(self.s16_full, self.k, out=self.full)

    def _quantize(self, grad: torch.Tensor):
        n = self.plan.n
        if grad.numel() != n:
            raise ValueError("bucket size changed")
        x = grad.reshape(-1)
        if self.wire == "i32":
            ops.quantize(x, self.k, out=self.q[:n])
        else:
            ops.quantize_i16_wire(x, self.k, out=self.q[:n])

    def _decode(self, src: torch.Tensor, y: torch.Tensor, ovf=None):
        if self.wire == "i32":
            ops.dequantize(src, self.k, out=y)
        else:
            ops.i16_wire_finish(src, self.k, self.V, y=y, overflow=ovf, want_out16=False)

    def _call_chunked(self, grad: torch.Tensor) -> torch.Tensor:
        n, L, sc, V = self.plan.n, self.cplan.padded, self.sc, self.V
        if grad.numel() != n:
            raise ValueError("bucket size changed")
        x = grad.reshape(-1)
        rs = []
        for c in range(self.chunks):           # quantise chunk c, then its RS on RCCL's stream
            lo, hi = c * L, min((c + 1) * L, n)
            if hi > lo:
                if self.wire == "i32":
                    ops.quantize(x[lo:hi], self.k, out=self._qbuf[lo:hi])
                else:
                    ops.quantize_i16_wire(x[lo:hi], self.k, out=self._qbuf[lo:hi])
            rs.append(reduce_scatter_sum(self._qbuf[c * L:(c + 1) * L], self.cplan, self.group,
                                         out=self.sum_c[c * sc:(c + 1) * sc], async_op=True)[1])
        ag = []
        for c in range(self.chunks):           # decode shard c once its RS is done, gather it
            _wait(rs[c])
            part = self.sum_c[c * sc:(c + 1) * sc]
            if self.wire == "i32":
                ops.dequantize(part, self.k, out=self.f_c[c * sc:(c + 1) * sc])
                ag.append(all_gather_shards(self.f_c[c * sc:(c + 1) * sc], self.cplan, self.group,
                                            out=self._fbuf[c * L:(c + 1) * L], async_op=True)[1])
            else:
                o16 = self.s16_c[c * sc:(c + 1) * sc]
                of = self.ovf_c[c * sc // V:(c + 1) * sc // V]
                ops.i16_wire_finish(part, self.k, V, out16=o16, overflow=of, want_y=False)
                ag.append(all_gather_shards(o16, self.cplan, self.group,
                                            out=self._s16buf[c * L:(c + 1) * L], async_op=True)[1])
                ag.append(all_gather_shards(of, self.cplan, self.group,
                                            out=self._obuf[c * L // V:(c + 1) * L // V], async_op=True)[1])
        for w in ag:
            _wait(w)
        if self.wire == "i16":
            ops.dequantize(self._s16buf[: self.cpad], self.k, out=self._fbuf[: self.cpad])
        return self._fbuf[:n]

    def __call__(self, grad: torch.Tensor) -> torch.Tensor:
        """fp32 [n] local bucket -> fp32 [n] dequantised sum over all ranks (one rank:
        the collectives are identities, quantise -> decode)."""
        if self.chunks > 1:
            return self._call_chunked(grad)
        self.phase_quantize(grad)
        self.phase_reduce_scatter()
        self.phase_decode()
        self.phase_all_gather()
        self.phase_expand()
        return self.full[: self.plan.n]

    def aggregate_int(self, grad: torch.Tensor) -> torch.Tensor:
        """fp32 [n] -> this rank's integer shard of the aggregate (no gather): the
        int32 wrapped sum, or on the i16 wire the int16 saturated sum (its slot flags
        in `ovf_shard`)."""
        self._quantize(grad)
        if self.collective == "a2a":
            s = reduce_scatter_a2a(self.q, self.plan, self.group, out=self.sum_shard, recv=self._recv)
        else:
            s = reduce_scatter_sum(self.q, self.plan, self.group, out=self.sum_shard)
        if self.wire == "i32":
            return s
        out16, _, _ = ops.i16_wire_finish(s, self.k, self.V, overflow=self.ovf_shard, want_y=False)
        return out16


class RangeAggregator:
    """Layout B of SURVEY.md 8e: rank r holds the W workers' fp32 slices of its own range
    `plan.range_of(r)` (the workers sent slot range r to GPU r: per-slot independence,
    ngaa.p4:87-168).  __call__ reduces them on this GPU -- the fused quantise + wrapping
    int32 sum (processor.p4:14-24), or on wire="i16" the int16 saturating sum with its
    per-slot overflow flags (headers.p4:30) -- dequantises, and all-gathers the fp32
    aggregate (and the flags) to every rank.  Each rank's shard is bit-identical to the
    single-GPU ina_quantize_reduce_f32_i32 / _i16_sat over the same W buckets, since the
    ranges hold whole slots.
    """

    def __init__(self, n: int, k: int = 16, group=None, device=None, align: int = 1024,
                 wire: str = "i32", V: int = 256):
        if wire not in ("i32", "i16"):
            raise ValueError("wire must be 'i32' or 'i16'")
        if V <= 0:
            raise ValueError("V must be > 0")
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if wire == "i16":
            align = align * V // math.gcd(align, V)        # ranges hold whole slots
        self.plan = ShardPlan(n, self.world, align)
        self.k, self.group, self.wire, self.V = k, group, wire, V
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.lo, self.hi = self.plan.range_of(self.rank)
        sdt = torch.int32 if wire == "i32" else torch.int16
        self.sum_shard = torch.zeros(self.plan.shard, dtype=sdt, device=dev)
        self.f_shard = torch.zeros(self.plan.shard, dtype=torch.float32, device=dev)   # pad stays 0
        # one rank: the gather is an identity, so the decode writes the aggregate in place
        self.full = self.f_shard if self.world == 1 else torch.empty(self.plan.padded, dtype=torch.float32,
                                                                     device=dev)
        if wire == "i16":
            self.slots_per_shard = self.plan.shard // V
            self.ovf_shard = torch.zeros(self.slots_per_shard, dtype=torch.uint8, device=dev)
            self.ovf_full = self.ovf_shard if self.world == 1 else torch.empty(
                self.slots_per_shard * self.world, dtype=torch.uint8, device=dev)
            if self.world > 1:        # the gather moves the int16 sums, decoded afterwards
                self.s16_full = torch.empty(self.plan.padded, dtype=torch.int16, device=dev)

    @property
    def range(self):
        """(lo, hi): the values of the bucket whose worker slices this rank holds."""
        return self.lo, self.hi

    @property
    def overflow(self) -> torch.Tensor:
        """Per-slot overflow flags of the last i16 aggregation (ceil(n / V) bytes)."""
        if self.wire != "i16":
            raise AttributeError("overflow flags exist only on the i16 wire")
        return self.ovf_full[: -(-self.plan.n // self.V)]

    def _reduce(self, slices) -> int:
        m = self.hi - self.lo
        if isinstance(slices, torch.Tensor):
            slices = list(slices.unbind(0)) if slices.dim() > 1 else [slices]
        slices = [t.reshape(-1) for t in slices]
        if not slices or any(t.numel() != m for t in slices):
            raise ValueError(f"every worker slice must hold this rank's {m} values")
        if m == 0:                    # more ranks than ranges: nothing here, zeros gathered
            return 0
        if self.wire == "i32":
            ops.quantize_reduce(slices, self.k, out=self.sum_shard[:m])
        else:
            ops.quantize_reduce_i16(slices, self.k, self.V, out=self.sum_shard[:m],
                                    overflow=self.ovf_shard[: -(-m // self.V)])
        return m

    @property
    def gather_bytes(self) -> int:
        """Bytes the all-gather brings to each rank over xGMI (values + flags)."""
        if self.world == 1:
            return 0
        per = self.plan.shard * (2 if self.wire == "i16" else 4)
        if self.wire == "i16":
            per += self.slots_per_shard
        return (self.world - 1) * per

    # The step's phases, in order (bench.py times each one between HIP events).
    def phase_reduce_decode(self, slices) -> int:
        """Local fused quantise + reduce; on the i32 wire (or one rank) also the decode."""
        m = self._reduce(slices)
        if m and (self.wire == "i32" or self.world == 1):
            ops.dequantize(self.sum_shard[:m], self.k, out=self.f_shard[:m])
        return m

    def phase_all_gather(self):
        if self.world == 1:
            return
        if self.wire == "i32":
            all_gather_shards(self.f_shard, self.plan, self.group, out=self.full)
        else:
            all_gather_shards(self.sum_shard, self.plan, self.group, out=self.s16_full)
            all_gather_shards(self.ovf_shard, self.plan, self.group, out=self.ovf_full)

    def phase_expand(self):
        """i16 wire at world > 1: dequantise the gathered int16 sums on every rank."""
        if self.world > 1 and self.wire == "i16":
            ops.dequantize(self.s16_full, self.k, out=self.full)

    def __call__(self, slices) -> torch.Tensor:
        """W fp32 slices of this rank's range -> fp32 [n] aggregate on every rank."""
        self.phase_reduce_decode(slices)
        self.phase_all_gather()
        self.phase_expand()
        return self.full[: self.plan.n]

    def aggregate_int(self, slices) -> torch.Tensor:
        """W fp32 slices -> this rank's integer aggregate (int32 wrapped, or int16
        saturated with its slot flags in `ovf_shard`), no gather."""
        m = self._reduce(slices)
        return self.sum_shard[:m]
