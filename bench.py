#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X INA aggregation path.

Metric (BASELINE.json): aggregated-gradient GB/s (device-resident), 8-worker x
100 MB int32 sum-reduce.  One "step" = one W-way sum-reduce launch over one
bucket of BASELINE config 3: W = 8 worker buffers of 26,214,400 int32 (100 MiB
each, V = 256 packet slots -> 102,400 slots), resident in HBM, reduced into one
aggregate -- the work the Tofino's Processor registers do per slot
(processor.p4:14-24).  value = W * n * 4 bytes * steps * ranks / max-rank time.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU; each rank
      aggregates its own bucket: slot ranges shard with no data-path collective,
      "scaling": "weak")

Extra rows (not the headline): --extra writes per-kernel timings of the other
configs (fused quantise+reduce C2, int16 C4, pack/unpack, PS combine, end-to-end
with pinned H2D/D2H) to gpurun_out/bench_extra.json.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
sys.path.insert(0, REPO)

METRIC = "aggregated-gradient GB/s (device-resident), 8-worker×100 MB int32 sum-reduce"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
W_WORKERS = 8
N_VALUES = 26_214_400        # 100 MiB of int32 per worker (config 3)
V_SLOT = 256
ROTATE = 2                   # input sets alternated per step (943 MB each > 256 MB MALL)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workers", type=int, default=W_WORKERS)
    ap.add_argument("--values", type=int, default=N_VALUES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=N_VALUES,
                    help="values per worker in the CPU-baseline sample (default: the whole "
                         "config-3 bucket, ~2-4 s of host work)")
    ap.add_argument("--extra", action="store_true")
    ap.add_argument("--mode", choices=("reduce", "sharded"), default="reduce",
                    help="reduce: the headline (config 3); sharded: config 5, one 1 GiB fp32 "
                         "bucket per rank aggregated with quantise -> RCCL reduce-scatter -> "
                         "dequantise -> all-gather")
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "traffic_sum_reduce_c3.json"))
    return ap.parse_args()


BACKEND = os.environ.get("INA_BENCH_BACKEND", "nccl")   # "gloo": rehearse N>1 on one GPU


def init_dist(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if BACKEND == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(BACKEND)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_inputs(W, n, seed_base, dev):
    g = torch.Generator(device=dev)
    bufs = []
    for w in range(W):
        g.manual_seed(seed_base + w)   # seed = 1000 + w, offset per rank/set
        bufs.append(torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev,
                                  generator=g))
    return bufs


def load_traffic(path, W, n):
    try:
        t = json.load(open(path))
        if t.get("workers") == W and t.get("values") == n:
            return t.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def cpu_baseline(args, bufs_host, gpu_out_sample):
    from oracle import oracle as orc
    n = bufs_host[0].size
    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(cores, 16))
    res = {}
    for P in sorted({1, threads}):
        ts = []
        out = None
        for it in range(13):             # 3 warm-up runs, median of 10
            out, secs = orc.cpu_packetise_aggregate(bufs_host, V_SLOT, P)
            if it >= 3:
                ts.append(secs)
        res[P] = (statistics.median(ts), out)
    tP, outP = res[threads]
    t1, _ = res[1]
    W = len(bufs_host)
    ok = bool(np.array_equal(outP, gpu_out_sample))
    # the PS's own float update, aggregate() as launch.py:42-52 writes it, in torch on the
    # same host cores over fp32 buffers of the same sample size
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(7)
    paras = [torch.randn(n, generator=g) * 1e-2 for _ in range(W)]
    local = torch.randn(n, generator=g)
    ta = []
    for _ in range(3):
        t0 = time.perf_counter()
        local += (1.0 / (W + 1)) * 1.0 * sum([p - local for p in paras])
        ta.append(time.perf_counter() - t0)
    t_agg = statistics.median(ta)
    part = "the whole" if n == N_VALUES else f"first {n * 4 // (1 << 20)} MiB of each"
    return {
        "value": round(W * n * 4 / tP / 1e9, 3), "unit": "GB/s", "cores": threads,
        "kind": "port",
        "sample": (f"{W} workers x {n} int32 ({part} config-3 "
                   f"bucket): NGA-{V_SLOT} packetise (header + memcpy + htonl per packet, "
                   f"communicator.cc:23-37) -> P4 aggregator restatement (count/frag/Processor "
                   f"registers, ngaa.p4:120-196) -> PS ack, 3 warm-up runs then median of 10, {threads} threads split "
                   f"as communicator.py:133-157"),
        "value_1core": round(W * n * 4 / t1 / 1e9, 3),
        "torch_aggregate_GBps": round(W * n * 4 / t_agg / 1e9, 3),
        "affinity_cores": cores,
        "matches_gpu": ok,
    }


def run_sharded(args, rank, world, dev):
    """Config 5: every rank is one worker with an n-value fp32 bucket (default 1 GiB)."""
    from ina_amd.dist import ShardedAggregator
    n = args.values if args.values != N_VALUES else 268_435_456
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    bucket = torch.randn(n, device=dev, generator=g) * 1e-2
    agg = ShardedAggregator(n, k=16, device=dev)
    for _ in range(args.warmup):
        agg(bucket)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agg(bucket)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    shard_bytes = agg.plan.shard * 4
    # spot check: the first 64 Ki aggregated values == dequantise(sum over ranks of
    # quantise(bucket)), the per-rank quantised prefixes exchanged with an all-gather
    from ina_amd import ops
    m = min(n, 1 << 16)
    out = agg(bucket)[:m]
    qp = ops.quantize(bucket[:m].contiguous(), 16)
    if world > 1:
        import torch.distributed as dist
        allq = torch.empty(world * m, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(allq, qp)
        qsum = (allq.view(world, m).to(torch.int64).sum(0) & 0xFFFFFFFF)
        qsum = torch.where(qsum >= (1 << 31), qsum - (1 << 32), qsum).to(torch.int32)
    else:
        qsum = qp
    parity = bool(torch.equal(out, ops.dequantize(qsum.contiguous(), 16)))
    return {
        "metric": "aggregated-gradient GB/s (config 5: 1 GiB fp32 bucket per rank, sharded RCCL)",
        "value": round(world * n * 4 * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": "C5: 1 GiB fp32 bucket per worker, quantise k=16 -> "
                               "reduce_scatter(int32,SUM) -> dequantise -> all_gather(fp32)",
                   "values_per_worker": n, "workers": world, "shard_values": agg.plan.shard,
                   "parallelism": f"RCCL x {world}"},
        "parity_spot_check": parity,
        "xgmi": {"rs_bytes_per_rank": (world - 1) * shard_bytes,
                 "ag_bytes_per_rank": (world - 1) * shard_bytes},
    }


def main():
    args = parse()
    rank, world, local = init_dist(args)
    dev = torch.device(f"cuda:{local}")
    from ina_amd import ops
    if args.mode == "sharded":
        line = run_sharded(args, rank, world, dev)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    W, n = args.workers, args.values
    sets = [make_inputs(W, n, 1000 + 100 * (rank * ROTATE + r), dev) for r in range(ROTATE)]
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(ROTATE)]
    torch.cuda.synchronize()

    for i in range(args.warmup):
        ops.sum_reduce(sets[i % ROTATE], out=outs[i % ROTATE])
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    t0 = time.perf_counter()
    ev0.record(stream)                      # HIP events on the launch stream, around
    for i in range(args.steps):             # exactly the K timed launches
        ops.sum_reduce(sets[i % ROTATE], out=outs[i % ROTATE])
    ev1.record(stream)
    barrier(world)
    t1 = time.perf_counter()
    elapsed = max_over_ranks(t1 - t0, world)
    # average launch duration over the timed region (back-to-back launches, so this
    # includes the kernel boundaries -- a slight over-estimate of the kernel alone)
    avg_launch_s = max_over_ranks(ev0.elapsed_time(ev1) / 1e3 / args.steps, world)

    # spot check of the measured output (first slots) against a numpy wrapping sum
    check_n = min(n, 1 << 16)
    last = (args.steps - 1) % ROTATE
    want = np.zeros(check_n, np.uint32)
    for b in sets[last]:
        want += b[:check_n].cpu().numpy().view(np.uint32)
    parity = bool(np.array_equal(outs[last][:check_n].cpu().numpy().view(np.uint32), want))

    worker_bytes = W * n * 4
    algo_bytes = (W + 1) * n * 4
    value = worker_bytes * args.steps * world / elapsed / 1e9
    achieved = algo_bytes / avg_launch_s / 1e9
    traffic = load_traffic(args.traffic_file, W, n)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (int32 uniform in [-2^20, 2^20), torch generator seed 1000+w per worker)",
        "config": {"workload": "C3: 8 workers x 100 MiB int32 (26,214,400 values), V=256 slots",
                   "workers": W, "values_per_worker": n, "slot_values": V_SLOT,
                   "slots": (n + V_SLOT - 1) // V_SLOT,
                   "parallelism": f"slot-range shards, one bucket per rank x {world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": "ina::k_sum_reduce_i32_vec<8,4,true> (512 x 256 threads)",
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_launch_us": round(avg_launch_s * 1e6, 2)},
        "parity_spot_check": parity,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        s = min(args.cpu_sample, n)
        host = [b[:s].cpu().numpy() for b in sets[last]]
        line["cpu_baseline"] = cpu_baseline(args, host, outs[last][:s].cpu().numpy())
    if rank == 0 and args.extra:
        from bench_extra import run_extra
        extra = run_extra(dev)
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        json.dump(extra, open(os.path.join(REPO, "gpurun_out", "bench_extra.json"), "w"), indent=1)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
