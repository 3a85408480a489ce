"""One rank of the sharded-aggregation GPU test (tests/test_gpu_dist.py), launched by
torch.distributed.run.  Every rank lives on cuda:0 and the group is gloo (one GPU cannot
host two RCCL ranks), so the collectives stage through host memory while quantise,
wire decode and dequantise run as the libina.so kernels: the product path of
ina_amd.dist.ShardedAggregator (layout A) or RangeAggregator (layout B) at world size > 1.  Writes its aggregate to
OUT/rank<r>.npz for the test to compare with the oracle."""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
sys.path.insert(0, REPO)


def bucket(rank: int, n: int, wire: str) -> np.ndarray:
    rng = np.random.default_rng(1000 + rank)
    if wire == "i32":
        x = (rng.standard_normal(n) * 3e3).astype(np.float32)   # wraps mod 2^32 at k=20
    else:
        x = rng.standard_normal(n).astype(np.float32)
        idx = rng.choice(n, max(1, n // 200), replace=False)
        x[idx] *= 100                                            # saturates at k=11
    if n > 7:
        x[7] = np.nan
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--wire", choices=("i32", "i16"), required=True)
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--V", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--layout", choices=("A", "B"), default="A")
    ap.add_argument("--workers", type=int, default=0, help="layout B: W buckets (default: world)")
    ap.add_argument("--collective", choices=("rs_ag", "a2a", "allreduce"), default="rs_ag")
    ap.add_argument("--chunks", type=int, default=1)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from ina_amd import _lib
    from ina_amd.dist import RangeAggregator, ShardedAggregator
    dev = torch.device("cuda", 0)
    if a.layout == "A":
        x = torch.from_numpy(bucket(rank, a.size, a.wire)).to(dev)
        agg = ShardedAggregator(a.size, k=a.k, device=dev, wire=a.wire, V=a.V,
                                collective=a.collective, chunks=a.chunks)
    else:                                      # every worker's slice of this rank's range
        agg = RangeAggregator(a.size, k=a.k, device=dev, wire=a.wire, V=a.V)
        lo, hi = agg.range
        x = [torch.from_numpy(bucket(w, a.size, a.wire)[lo:hi].copy()).to(dev)
             for w in range(a.workers or world)]
    for _ in range(a.steps):                   # buffers are reused across calls
        full = agg(x)
    torch.cuda.synchronize()
    res = {"full": full.cpu().numpy(), "world": np.array([world]),
           "gather_bytes": np.array([agg.gather_bytes, agg.plan.shard if getattr(agg, "chunks", 1) == 1
                                     else agg.chunks * agg.sc])}
    if a.wire == "i16":
        res["ovf"] = agg.overflow.cpu().numpy()
    shard = agg.aggregate_int(x)
    torch.cuda.synchronize()
    lo, hi = agg.plan.range_of(rank)
    res["shard"] = shard[: hi - lo].cpu().numpy()
    res["range"] = np.array([lo, hi])
    res["lib"] = np.array([os.path.realpath(_lib.LIB_PATH)])
    np.savez(os.path.join(a.out, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
