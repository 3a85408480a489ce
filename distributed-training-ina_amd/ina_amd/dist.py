"""Multi-GPU aggregation of one bucket that outgrows a GPU (BASELINE config 5).

Layout A of SURVEY.md 8e: every rank is one worker holding its full fp32
gradient bucket.  Each rank quantises its bucket on its GPU (int32, 2^k fixed
point), RCCL reduce-scatters the integers with SUM over xGMI -- integer addition
mod 2^32 is associative and commutative, so the shard each rank receives is
bit-identical to the switch's per-slot sum (processor.p4:14-24) in any ring or
tree order -- the owner dequantises its shard, and an all-gather returns the
full aggregate to every rank (the PS broadcast).  The int16 path never reduces
saturated int16 through RCCL (saturation is not associative): it accumulates in
int32 and saturates once after the reduce.

Shards are contiguous slot ranges padded to `align` values (default one V=256
slot x 4 = 1024 values = 4 KiB), so no slot straddles two ranks.
The collective plumbing (ShardPlan, reduce_scatter_sum, all_gather_shards) is
device-agnostic and covered on CPU with gloo; the quantise/dequantise steps are
the device kernels (no CPU path).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops


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


def reduce_scatter_sum(x_padded: torch.Tensor, plan: ShardPlan, group=None, out=None):
    """int32 [padded] -> this rank's [shard] of the element-wise sum over ranks."""
    if x_padded.numel() != plan.padded:
        raise ValueError("input must be padded to plan.padded")
    out = torch.empty(plan.shard, dtype=x_padded.dtype, device=x_padded.device) if out is None else out
    if plan.world == 1:
        out.copy_(x_padded)
        return out
    dist.reduce_scatter_tensor(out, x_padded, op=dist.ReduceOp.SUM, group=group)
    return out


def all_gather_shards(shard: torch.Tensor, plan: ShardPlan, group=None, out=None):
    out = torch.empty(plan.padded, dtype=shard.dtype, device=shard.device) if out is None else out
    if plan.world == 1:
        out.copy_(shard)
        return out
    dist.all_gather_into_tensor(out, shard, group=group)
    return out


class ShardedAggregator:
    """Reusable buffers for repeated sharded aggregation of same-sized buckets."""

    def __init__(self, n: int, k: int = 16, group=None, device=None, align: int = 1024):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.plan = ShardPlan(n, self.world, align)
        self.k, self.group = k, group
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.q = torch.zeros(self.plan.padded, dtype=torch.int32, device=dev)   # pad stays 0
        self.sum_shard = torch.empty(self.plan.shard, dtype=torch.int32, device=dev)
        self.f_shard = torch.empty(self.plan.shard, dtype=torch.float32, device=dev)
        self.full = torch.empty(self.plan.padded, dtype=torch.float32, device=dev)

    def __call__(self, grad: torch.Tensor) -> torch.Tensor:
        """fp32 [n] local bucket -> fp32 [n] dequantised sum over all ranks."""
        n = self.plan.n
        if grad.numel() != n:
            raise ValueError("bucket size changed")
        if self.world == 1:      # the collectives are identities: quantise -> dequantise
            ops.quantize(grad.reshape(-1), self.k, out=self.q[:n])
            return ops.dequantize(self.q[:n], self.k, out=self.full[:n])
        ops.quantize(grad.reshape(-1), self.k, out=self.q[:n])
        reduce_scatter_sum(self.q, self.plan, self.group, out=self.sum_shard)
        ops.dequantize(self.sum_shard, self.k, out=self.f_shard)
        all_gather_shards(self.f_shard, self.plan, self.group, out=self.full)
        return self.full[:n]

    def aggregate_int(self, grad: torch.Tensor) -> torch.Tensor:
        """fp32 [n] -> this rank's int32 shard of the integer aggregate (no gather)."""
        ops.quantize(grad.reshape(-1), self.k, out=self.q[: self.plan.n])
        return reduce_scatter_sum(self.q, self.plan, self.group, out=self.sum_shard)
