#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X INA aggregation path.

Metric (BASELINE.json): aggregated-gradient GB/s (device-resident), 8-worker x
100 MB int32 sum-reduce.  One "step" = one W-way sum-reduce launch over one
bucket of BASELINE config 3: W = 8 worker buffers of 26,214,400 int32 (100 MiB
each, V = 256 packet slots -> 102,400 slots), resident in HBM, reduced into one
aggregate -- the work the Tofino's Processor registers do per slot
(processor.p4:14-24).  value = W * n * 4 bytes * steps * ranks / max-rank time.

  python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts N ranks
itself (torch.distributed.run, 127.0.0.1, one rank per GPU) before anything
touches the GPU; under an external torchrun it runs as one of those ranks.  Every
rank asserts that the process group holds exactly N ranks (backend nccl = RCCL).

Multi-GPU:
  * headline, "scaling": "weak" -- the switch aggregates every slot independently
    (ngaa.p4:87-168), so N GPUs aggregate N config-3 slot ranges (rank r owns
    slots [r*102400, (r+1)*102400) of an N x 100 MiB job) with no data-path
    collective: a 100 MiB bucket never outgrows one GPU, and the north star
    shards over xGMI only when one does;
  * "sharded_c5" -- in the same run, every rank times config 5 through RCCL:
    a 1 GiB fp32 bucket per rank, quantise -> reduce_scatter(int32, SUM) ->
    dequantise -> all_gather(fp32) (ina_amd.dist.ShardedAggregator), with per-
    phase times, the xGMI bytes per rank and a parity check of the aggregate.
  --mode sharded makes config 5 the headline line instead.
  * "switch_c3" -- the packet-stream switch (ina_switch_process) on
    config 3 as 819,200 NGA-256 packets, worker-major and round-robin arrival, with its
    own roofline fraction on its algorithmic bytes; at N > 1 every rank switches its own
    bucket (max-over-ranks time, aggregate bytes/s).
  * "sharded_c5.layout_b" -- config 5 when the workers' slices arrive split by range
    (ina_amd.dist.RangeAggregator): local fused quantise + reduce, one all-gather.
    Every config-5 variant carries an xGMI `roofline` (per-rank bytes over the collective
    phases against 7 links x 153 GB/s; null at one rank) and the HBM fraction of its
    quantise / decode phases.

Single-GPU BASELINE configs in the same line, each with a roofline and a parity spot check:
  * "c2_fused" -- config 2: 4 x ResNet-50 fp32 -> fused quantise + int32 sum;
  * "c4_int16" -- config 4: 16 x ResNet-50 fp32 -> int16 saturating sum + slot flags;
  * "e2e_pcie" -- config 3 from pinned host memory through HBM and back (the PCIe-
    inclusive rate), against the pinned H2D rate measured in the same run.

Extra rows (not the headline): --extra writes per-kernel timings of the other
configs (fused quantise+reduce C2, int16 C4, pack/unpack, PS combine, end-to-end
with pinned H2D/D2H) to gpurun_out/bench_extra.json.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import statistics
import subprocess
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
C5_VALUES = 268_435_456      # 1 GiB of fp32 per worker (config 5)
C5_CHUNKS = 4                # pipelined config-5 variant at N > 1: 256 MiB chunks
V_SLOT = 256
ROTATE = 2                   # input sets alternated per step (943 MB each > 256 MB MALL)
RESNET50_PARAMS = 25_557_032  # communicator.py:11 (configs 2 and 4)
PCIE_SPEC_GBS = 63.0         # PCIe Gen5 x16, MI355X_MICROARCH.md (host link)
# per-GPU xGMI peak for the config-5 collectives: 7 links x ~153 GB/s (SURVEY.md section 5;
# the task's MI355X notes).  A single ring uses one link each way (153 GB/s).
XGMI_LINKS, XGMI_LINK_GBS = 7, 153.0
XGMI_PEAK_GBS = XGMI_LINKS * XGMI_LINK_GBS
_ACT_FWD_AGG, _ACT_FWD_ACK = 1, 3      # ina.h action codes: completed slot forwarded, PS ack


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workers", type=int, default=W_WORKERS)
    ap.add_argument("--values", type=int, default=N_VALUES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=N_VALUES,
                    help="values per worker in the CPU-baseline sample (default: the whole "
                         "config-3 bucket)")
    ap.add_argument("--extra", action="store_true")
    ap.add_argument("--mode", choices=("reduce", "sharded"), default="reduce",
                    help="reduce: the headline (config 3); sharded: config 5 as the headline, "
                         "one 1 GiB fp32 bucket per rank aggregated with quantise -> RCCL "
                         "reduce-scatter -> dequantise -> all-gather")
    ap.add_argument("--c5-values", type=int, default=C5_VALUES,
                    help="fp32 values per rank of the config-5 measurement")
    ap.add_argument("--c5-steps", type=int, default=10)
    ap.add_argument("--wire", choices=("i32", "i16"), default="i32",
                    help="config-5 wire: int32, or the int16 saturating wire (config 4 rule)")
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 sub-measurement")
    ap.add_argument("--no-c2", action="store_true", help="skip config 2 (fused quantise + reduce)")
    ap.add_argument("--no-c4", action="store_true", help="skip config 4 (int16 saturating, 16 workers)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the PCIe-inclusive rate (pinned host buckets -> HBM -> reduce -> host)")
    ap.add_argument("--no-switch", action="store_true",
                    help="skip the packet-stream switch sub-measurement (config 3 as NGA-256 packets)")
    ap.add_argument("--check-launch", action="store_true",
                    help="launcher self-check: start the ranks, form the group, assert its size, "
                         "print one JSON line; no GPU work (runs on CPU with gloo)")
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "traffic_sum_reduce_c3.json"))
    return ap.parse_args(argv)


BACKEND = os.environ.get("INA_BENCH_BACKEND", "nccl")   # "gloo": rehearse N>1 on one GPU


# -- launching and the process group ----------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks with torch.distributed.run as
    child processes.  This process never initialises the GPU (nothing above touched
    torch.cuda), and it waits for the ranks and exits with their status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, cwd=REPO).returncode


def init_dist(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    use_gpu = not args.check_launch
    if use_gpu:
        if BACKEND == "gloo":
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
    backend = "none"
    if world > 1:
        import torch.distributed as dist
        backend = BACKEND if use_gpu else "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
        got = dist.get_world_size()
        if got != args.gpus:
            raise SystemExit(f"bench.py: process group holds {got} ranks, expected {args.gpus}")
        backend = dist.get_backend()
    return rank, world, local, backend


def barrier(world, gpu=True):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    if gpu:
        torch.cuda.synchronize()


def reduce_over_ranks(x: float, world: int, op: str = "max") -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if BACKEND == "nccl" and torch.cuda.is_available() else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
    return float(t.item())


def max_over_ranks(x: float, world: int) -> float:
    return reduce_over_ranks(x, world, "max")


def all_ranks_true(ok: bool, world: int) -> bool:
    return reduce_over_ranks(1.0 if ok else 0.0, world, "min") == 1.0


# -- inputs --------------------------------------------------------------------------------
def make_inputs(W, n, seed_base, dev):
    g = torch.Generator(device=dev)
    bufs = []
    for w in range(W):
        g.manual_seed(seed_base + w)   # seed = 1000 + w, offset per rank/set
        bufs.append(torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev,
                                  generator=g))
    return bufs


HEADLINE_KERNEL = "ina::k_sum_reduce_i32_vec<8,4,true>"


def _kernel_symbol(name: str) -> str:
    """'void ina::k<8, 4, true>(args...)' -> 'ina::k<8,4,true>' (comparable form)."""
    name = name.split("(")[0].strip()
    if name.startswith("void "):
        name = name[5:]
    return "".join(name.split())


def load_traffic(path, W, n, kernel=HEADLINE_KERNEL):
    """Per-launch HBM bytes from the committed PMC file (tools/pmc_traffic.py: two rocprofv3
    --pmc passes, FETCH_SIZE doubled per the gfx950 half-count, WRITE_SIZE) and where they
    came from: (bytes, source).  The bytes are null unless the file measured THIS kernel
    symbol at this size -- a file from another kernel build must not be quoted."""
    try:
        t = json.load(open(path))
    except Exception as e:                # noqa: BLE001 -- no file: traffic unmeasured
        return None, {"file": os.path.relpath(path, REPO), "error": type(e).__name__}
    ok = (t.get("workers") == W and t.get("values") == n
          and _kernel_symbol(t.get("kernel", "")) == _kernel_symbol(kernel))
    src = {"file": os.path.relpath(path, REPO), "session": t.get("session"),
           "kernel": t.get("kernel"), "matches_kernel_and_size": ok,
           "measured": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc_traffic.py)"}
    return (t.get("hbm_bytes_per_launch") if ok else None), src


# -- CPU baseline ----------------------------------------------------------------------------
def cgroup_cpus():
    """CPUs the cgroup quota grants (cpu.max), or None when unlimited/unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return round(int(q) / int(p), 2)
    except Exception:
        pass
    return None


def _median_of_10(fn):
    ts = []
    out = None
    for it in range(13):             # 3 warm-up runs, median of 10
        out, secs = fn()
        if it >= 3:
            ts.append(secs)
    return statistics.median(ts), out


def cpu_baseline(args, bufs_host, gpu_out_sample):
    """the reference's CPU path (packetise + P4 aggregator restatement) on the
    host's cores, threads split as communicator.py:133-157, at 1 thread, at every core of
    the affinity mask, and at the CPU count the cgroup quota grants (and twice that);
    `value` is the best of them and `cores` the thread count that reached it.  Plus torch's
    float aggregate() (launch.py:42-52) at that thread count."""
    from oracle import oracle as orc
    n = bufs_host[0].size
    W = len(bufs_host)
    cores = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    counts = {1, cores}
    if quota:
        q = max(1, int(quota))
        counts |= {min(q, cores), min(2 * q, cores)}
    counts = sorted(counts)
    res = {}
    for P in counts:
        res[P] = _median_of_10(lambda: orc.cpu_packetise_aggregate(bufs_host, V_SLOT, P))
    best = min(counts, key=lambda P: res[P][0])
    tP, outP = res[best]
    ok = all(bool(np.array_equal(res[P][1], gpu_out_sample)) for P in counts)
    # the PS's own float update, aggregate() as launch.py:42-52 writes it, in torch over
    # fp32 buffers of the same sample size
    torch.set_num_threads(best)
    g = torch.Generator().manual_seed(7)
    paras = [torch.randn(n, generator=g) * 1e-2 for _ in range(W)]
    local = torch.randn(n, generator=g)

    def agg_once():
        nonlocal local
        t0 = time.perf_counter()
        local += (1.0 / (W + 1)) * 1.0 * sum([p - local for p in paras])
        return None, time.perf_counter() - t0
    t_agg, _ = _median_of_10(agg_once)
    part = "the whole" if n == N_VALUES else f"first {n * 4 // (1 << 20)} MiB of each"
    gbs = {P: round(W * n * 4 / res[P][0] / 1e9, 3) for P in counts}
    # CPUs this process may actually run on at once: the affinity mask, capped by the
    # cgroup quota (on the GPU box 256 CPUs are visible but 16 granted)
    granted = min(cores, max(1, int(quota))) if quota else cores
    extra = {}
    if cores <= granted:                    # the affinity mask is what the process gets
        extra["value_all_affinity_cores"] = gbs[cores]
    else:                                   # more threads than granted CPUs time-share them
        extra[f"value_{cores}_threads"] = gbs[cores]
    return {
        "value": gbs[best], "unit": "GB/s", "cores": granted, "threads": best,
        "kind": "port",
        "sample": (f"{W} workers x {n} int32 ({part} config-3 "
                   f"bucket): NGA-{V_SLOT} packetise (header + memcpy + htonl per packet, "
                   f"communicator.cc:23-37) -> P4 aggregator restatement (count/frag/Processor "
                   f"registers, ngaa.p4:120-196) -> PS ack, 3 warm-up runs then median of 10, "
                   f"threads split as communicator.py:133-157; timed at {counts} threads "
                   f"(affinity mask {cores} CPUs, cgroup quota {quota} CPUs: {granted} CPUs "
                   f"granted), best = {best} threads"),
        "value_1core": gbs[1],
        **extra,
        "value_by_threads": {str(P): v for P, v in gbs.items()},
        "cgroup_cpu_quota": quota,
        "torch_aggregate_GBps": round(W * n * 4 / t_agg / 1e9, 3),
        "torch_aggregate_threads": best,
        "affinity_cores": cores,
        "matches_gpu": ok,
    }


# -- config 5: sharded over RCCL --------------------------------------------------------------
def _phase_times(phases, stream, world, passes=6):
    """Per-phase device time (s) of a step made of `phases` (callables that enqueue work on
    `stream`): HIP events between the phases over `passes` back-to-back passes, the median
    over passes 2.. (the first passes start with an empty queue, so the host's launch time
    would sit between the events; afterwards the host is ahead of the GPU), max over ranks."""
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(phases) + 1)] for _ in range(passes)]
    barrier(world)
    for p in range(passes):
        ev[p][0].record(stream)
        for i, fn in enumerate(phases):
            fn()
            ev[p][i + 1].record(stream)
    torch.cuda.synchronize()
    out = []
    for i in range(len(phases)):
        t = sorted(ev[p][i].elapsed_time(ev[p][i + 1]) / 1e3 for p in range(2, passes))
        out.append(max_over_ranks(t[len(t) // 2], world))
    return out


def measure_c5(args, rank, world, dev, warmup=2, collective="rs_ag", chunks=1):
    """quantise -> reduce_scatter(int32, SUM) -> decode -> all_gather of one n-value fp32
    bucket per rank (the i32 wire gathers fp32; the i16 wire gathers the saturated int16
    sums + slot flags and dequantises after); per-phase HIP-event times on the launch
    stream.  collective="allreduce": one all-reduce of the integer wire, every rank
    decodes the whole bucket (phase "reduce_scatter" is then the all-reduce).
    chunks > 1: the pipelined step (ShardedAggregator(chunks=C)); its phases overlap, so
    only the step time is reported."""
    from ina_amd import ops
    from ina_amd.dist import ShardedAggregator, all_gather_shards
    n = args.c5_values
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    bucket = torch.randn(n, device=dev, generator=g) * 1e-2
    k = 16 if args.wire == "i32" else 20
    agg = ShardedAggregator(n, k=k, device=dev, wire=args.wire, V=V_SLOT, collective=collective,
                            chunks=chunks)
    for _ in range(warmup):
        agg(bucket)
    steps = args.c5_steps
    stream = torch.cuda.current_stream(dev)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        agg(bucket)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)

    # per-phase breakdown: events between the aggregator's own phases
    phase = None
    if agg.chunks == 1:
        phase = _phase_times([lambda: agg.phase_quantize(bucket), agg.phase_reduce_scatter,
                              agg.phase_decode, agg.phase_all_gather, agg.phase_expand],
                             stream, world)

    # parity: the aggregate at a sample of positions == decode(sum over ranks of the
    # per-rank wire of those values), the per-rank wires all-gathered.  The sample covers
    # the first 64 Ki values and 4 Ki values at the start of every (chunk, rank) shard --
    # every reduce-scatter and all-gather the pipelined variant overlaps -- and every
    # rank's whole-bucket shard
    pos = [torch.arange(0, min(n, 1 << 16))]
    if agg.chunks > 1:
        L, sc = agg.cplan.padded, agg.sc
        starts = [c * L + r * sc for c in range(agg.chunks) for r in range(world)]
        ends = [min(c * L + r * sc + sc, n) for c in range(agg.chunks) for r in range(world)]
    else:
        sh = agg.plan.shard
        starts = [r * sh for r in range(world)]
        ends = [min(r * sh + sh, n) for r in range(world)]
    for lo, hi in zip(starts, ends):
        if hi > lo:
            pos.append(torch.arange(lo, min(hi, lo + 4096)))
            pos.append(torch.arange(max(lo, hi - 64), hi))
    pos = torch.unique(torch.cat(pos)).to(dev)
    m = pos.numel()
    out = agg(bucket)[pos].clone()
    head = bucket[pos].contiguous()
    wp = ops.quantize(head, k) if args.wire == "i32" else ops.quantize_i16_wire(head, k)
    if world > 1:
        from ina_amd.dist import ShardPlan
        allw = all_gather_shards(wp, ShardPlan(m * world, world, align=m))
        wsum = allw.view(world, m).to(torch.int64).sum(0)
        wsum = ((wsum + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)
    else:
        wsum = wp
    if args.wire == "i32":
        want = ops.dequantize(wsum.contiguous(), k)
    else:
        # the sampled positions are not whole slots, so only the values are compared here
        # (the flags: tests/test_gpu_dist.py)
        _, want, _ = ops.i16_wire_finish(wsum.contiguous(), k, 1, want_out16=False)
    parity = all_ranks_true(bool(torch.equal(out, want)), world)

    G = world
    S = agg.plan.padded * 4
    xgmi = (G - 1) * S // G                # int32 wire words reduce-scattered
    ag = agg.gather_bytes                  # fp32 (i32 wire) or int16 + flags (i16 wire)
    t_step = elapsed / steps
    if phase is None:                      # pipelined: the step time and its bytes only
        rs = (G - 1) * agg.chunks * agg.sc * 4
        return {
            "value": round(world * n * 4 * steps / elapsed / 1e9, 2), "unit": "GB/s",
            "ms_per_step": round(t_step * 1e3, 3), "steps": steps, "warmup": warmup,
            "workload": (f"C5 pipelined: the same step in {agg.chunks} chunks, chunk c+1's "
                         f"quantise under chunk c's reduce_scatter (async RCCL work)"),
            "collective": collective, "chunks": agg.chunks,
            "xgmi": {"rs_send_bytes_per_rank": rs, "ag_recv_bytes_per_rank": ag,
                     "busbw_GBps": round((rs + ag) / t_step / 1e9, 1) if world > 1 else None},
            "roofline": _xgmi_roofline(rs + ag, t_step if world > 1 else None,
                                       "whole step (phases overlap): RS send + AG receive bytes / step time"),
            "parity_spot_check": parity,
            "parity_sample": f"{m} values: the first 64 Ki and the head and tail of every (chunk, rank) shard",
        }
    q_bytes = 8 * n                                        # fp32 in, int32 wire out
    shard = agg.plan.shard
    if collective == "allreduce" or world == 1:            # decode of the whole bucket
        d_bytes = 8 * agg.plan.padded if args.wire == "i32" else 8 * agg.plan.padded + agg.plan.padded // V_SLOT
    elif args.wire == "i32":
        d_bytes = 8 * shard                                # int32 shard in, fp32 out
    else:
        d_bytes = 6 * shard + shard // V_SLOT              # int32 in, int16 + slot flags out
    coll_bytes = 2 * xgmi if collective == "allreduce" else xgmi + ag
    coll_s = (phase[1] + phase[3]) if world > 1 else None
    roofline = _xgmi_roofline(coll_bytes, coll_s,
                              "collective phases only: (all-reduce, or RS send + AG receive) bytes / "
                              "their HIP-event time")
    roofline["hbm_phases"] = {
        "quantize": _phase_frac(q_bytes, phase[0]),
        "decode": _phase_frac(d_bytes, phase[2]),
        **({"expand": _phase_frac(6 * agg.plan.padded, phase[4])}
           if args.wire == "i16" and world > 1 and collective != "allreduce" else {}),
    }
    return {
        "value": round(world * n * 4 * steps / elapsed / 1e9, 2), "unit": "GB/s",
        "metric": "aggregated-gradient GB/s (config 5: fp32 bucket per rank, sharded over RCCL)",
        "ms_per_step": round(t_step * 1e3, 3), "steps": steps, "warmup": warmup,
        "workload": (f"C5: {n} fp32 values ({n * 4 / 2 ** 30:.2f} GiB) per rank, quantise "
                     f"({args.wire} wire, k={k}) -> "
                     + ("all_reduce(int32, SUM) -> decode the whole bucket on every rank"
                        if collective == "allreduce" else
                        ("all_to_all(int32) + device sum of the slices -> " if collective == "a2a" else
                         "reduce_scatter(int32, SUM) -> ")
                        + ("dequantise -> all_gather(fp32)" if args.wire == "i32" else
                           "saturate once -> all_gather(int16 + slot flags) -> dequantise"))),
        "values_per_rank": n, "shard_values": agg.plan.shard, "rccl_world": world,
        "collective": collective,
        "phase_ms": {"quantize": round(phase[0] * 1e3, 3), "reduce_scatter": round(phase[1] * 1e3, 3),
                     "decode": round(phase[2] * 1e3, 3), "all_gather": round(phase[3] * 1e3, 3),
                     "expand": round(phase[4] * 1e3, 3)},
        "xgmi": ({"rs_send_bytes_per_rank": xgmi, "ag_recv_bytes_per_rank": ag,
                  "rs_busbw_GBps": round(xgmi / phase[1] / 1e9, 1) if world > 1 and phase[1] > 0 else None,
                  "ag_busbw_GBps": round(ag / phase[3] / 1e9, 1) if world > 1 and phase[3] > 0 else None}
                 if collective != "allreduce" else
                 {"allreduce_bytes_per_rank": 2 * xgmi,     # nccl-tests busbw: 2(G-1)/G x S / t
                  "allreduce_busbw_GBps": round(2 * xgmi / phase[1] / 1e9, 1) if world > 1 and phase[1] > 0 else None}),
        "roofline": roofline,
        "parity_spot_check": parity,
        "parity_sample": f"{m} values: the first 64 Ki and the head and tail of every rank's shard",
    }


def _xgmi_roofline(nbytes, secs, what):
    """Per-rank xGMI roofline of a config-5 variant (null at one rank: no link traffic)."""
    ach = nbytes / secs / 1e9 if secs and nbytes else None
    return {"bound": "xgmi", "unit": "GB/s", "bytes_per_rank": int(nbytes),
            "achieved": round(ach, 1) if ach is not None else None,
            "peak": XGMI_PEAK_GBS,
            "peak_source": f"{XGMI_LINKS} xGMI links x {XGMI_LINK_GBS:.0f} GB/s per GPU (SURVEY.md section 5)",
            "frac": round(ach / XGMI_PEAK_GBS, 4) if ach is not None else None,
            "frac_of_one_link": round(ach / XGMI_LINK_GBS, 4) if ach is not None else None,
            "measures": what}


def _phase_frac(nbytes, secs):
    gbs = nbytes / secs / 1e9 if secs > 0 else None
    return {"bytes": int(nbytes), "us": round(secs * 1e6, 1),
            "GBps": round(gbs, 1) if gbs else None,
            "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None}


def measure_c5_layout_b(args, rank, world, dev, warmup=2):
    """Layout B of config 5 (ina_amd.dist.RangeAggregator): the same W = world buckets of
    n values, but already split by range -- rank r holds every worker's slice of range r
    (n values in all) -- so the step is a local fused quantise + reduce, a decode, and
    one all-gather (no reduce-scatter).  Per-phase HIP-event times; parity: the shard's
    first 64 Ki values against the per-slice device quantise summed on the host."""
    from ina_amd import ops
    from ina_amd.dist import RangeAggregator
    n = args.c5_values
    k = 16 if args.wire == "i32" else 20
    agg = RangeAggregator(n, k=k, device=dev, wire=args.wire, V=V_SLOT)
    lo, hi = agg.range
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    slices = [torch.randn(hi - lo, device=dev, generator=g) * 1e-2 for _ in range(world)]
    for _ in range(warmup):
        agg(slices)
    steps = args.c5_steps
    stream = torch.cuda.current_stream(dev)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        agg(slices)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    m = agg.phase_reduce_decode(slices)
    phase = _phase_times([lambda: agg.phase_reduce_decode(slices), agg.phase_all_gather,
                          agg.phase_expand], stream, world)
    c = min(m, 1 << 16)
    ok = True
    if c:
        agg(slices)
        got = agg.full[lo:lo + c].clone()
        heads = [t[:c].contiguous() for t in slices]
        if args.wire == "i32":
            wsum = torch.stack([ops.quantize(h, k) for h in heads]).to(torch.int64).sum(0)
            wsum = ((wsum + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)
            want = ops.dequantize(wsum.contiguous(), k)
        else:
            wsum = torch.stack([ops.quantize_i16_wire(h, k) for h in heads]).sum(0, dtype=torch.int32)
            _, want, _ = ops.i16_wire_finish(wsum.contiguous(), k, V_SLOT, want_out16=False)
        ok = bool(torch.equal(got, want))
    parity = all_ranks_true(ok, world)
    ag = agg.gather_bytes
    roofline = _xgmi_roofline(ag, phase[1] if world > 1 else None,
                              "all-gather receive bytes / its HIP-event time")
    W = world
    if args.wire == "i32":                 # fused quantise + reduce, then the decode
        rd_bytes = (4 * W + 4) * m + 8 * m
    else:                                  # int16 sums + flags (decoded after the gather)
        rd_bytes = (4 * W + 2) * m + m // V_SLOT + (8 * m if world == 1 else 0)
    roofline["hbm_phases"] = {"reduce_decode": _phase_frac(rd_bytes, phase[0])}
    if args.wire == "i16" and world > 1:
        roofline["hbm_phases"]["expand"] = _phase_frac(6 * agg.plan.padded, phase[2])
    return {
        "value": round(world * n * 4 * steps / elapsed / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "workload": (f"C5 layout B: {world} workers x {n} values, rank r holds every worker's "
                     f"slice of range r ({agg.plan.shard} values each): fused quantise + reduce "
                     f"({args.wire}) -> " + ("dequantise -> all_gather(fp32)" if args.wire == "i32" else
                                         "all_gather(int16 + slot flags) -> dequantise")),
        "phase_ms": {"reduce_decode": round(phase[0] * 1e3, 3), "all_gather": round(phase[1] * 1e3, 3),
                     "expand": round(phase[2] * 1e3, 3)},
        "xgmi": {"ag_recv_bytes_per_rank": ag,
                 "ag_busbw_GBps": round(ag / phase[1] / 1e9, 1) if world > 1 and phase[1] > 0 else None},
        "roofline": roofline,
        "parity_spot_check": parity,
    }


# -- configs 2 and 4 and the PCIe-inclusive rate (single-GPU BASELINE configs) ------------------
# Spot checks restate the build-defined quantiser in numpy on a strided
# sample of the measured outputs, as the headline's check restates the wrapping sum.
def _np_q32(x: np.ndarray, k: int) -> np.ndarray:
    with np.errstate(invalid="ignore", over="ignore"):
        y = np.rint(x.astype(np.float32) * np.float32(2.0 ** k)).astype(np.float64)
    y = np.nan_to_num(y, nan=0.0, posinf=2.0 ** 31, neginf=-(2.0 ** 31) - 1)
    return np.clip(y, -(2.0 ** 31), 2.0 ** 31 - 1).astype(np.int64)


def _np_q16(x: np.ndarray, k: int):
    """(int16 value as int64, saturated-or-NaN bool) per element."""
    with np.errstate(invalid="ignore", over="ignore"):
        y = np.rint(x.astype(np.float32) * np.float32(2.0 ** k)).astype(np.float64)
    nan = np.isnan(y)
    sat = nan | (y > 32767) | (y < -32768)
    return np.where(nan, 0, np.clip(y, -32768, 32767)).astype(np.int64), sat


def _sample_idx(n: int, step: int = 997) -> np.ndarray:
    """Strided sample (every step-th value, the first 4 Ki and the last 4 Ki)."""
    return np.unique(np.concatenate([np.arange(0, n, step), np.arange(min(n, 4096)),
                                     np.arange(max(0, n - 4096), n)]))


def _time_rotating(fn_for_set, rotate, steps, warm, stream, min_warm_s=0.05):
    """HIP events on the launch stream around `steps` back-to-back launches alternating
    `rotate` input sets (the headline's method); returns the average launch in seconds.
    Warm-up: `warm` launches and at least `min_warm_s` of them, so the timed launches do
    not start while the GPU's clocks are still ramping up from an idle phase."""
    t0, i = time.perf_counter(), 0
    while i < warm or time.perf_counter() - t0 < min_warm_s:
        fn_for_set(i % rotate)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(steps):
        fn_for_set(i % rotate)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / steps


def _hbm_roofline(algo_bytes, avg_s, kernel):
    ach = algo_bytes / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "kernel": kernel,
            "algorithmic_bytes_per_launch": int(algo_bytes), "avg_launch_us": round(avg_s * 1e6, 2)}


def measure_c2(dev, world=1, steps=20, warm=3, rank=0):
    """BASELINE config 2: 4 workers x 25,557,032 fp32 (ResNet-50, communicator.py:11) ->
    fused quantise (k=16) + wrapping int32 sum (ina_quantize_reduce_f32_i32), the work
    launch.py:42-52's consumer receives.  Algorithmic bytes (4W+4) per value."""
    from ina_amd import ops
    W, n, k = 4, RESNET50_PARAMS, 16
    g = torch.Generator(device=dev)
    sets = []
    for r in range(ROTATE):
        g.manual_seed(3000 + 100 * (rank * ROTATE + r))
        sets.append([torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)])
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(ROTATE)]
    s = torch.cuda.current_stream(dev)
    barrier(world)
    avg = max_over_ranks(_time_rotating(lambda r: ops.quantize_reduce(sets[r], k, out=outs[r]),
                                        ROTATE, steps, warm, s), world)
    last = (steps - 1) % ROTATE
    idx = _sample_idx(n)
    ti = torch.from_numpy(idx).to(dev)
    want = np.zeros(idx.size, np.int64)
    for x in sets[last]:
        want += _np_q32(x[ti].cpu().numpy(), k)
    want = ((want + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int32)
    ok = all_ranks_true(bool(np.array_equal(outs[last][ti].cpu().numpy(), want)), world)
    algo = (4 * W + 4) * n
    res = {"workload": f"C2: {W} workers x {n} fp32 (ResNet-50 bucket) -> fused quantise (k={k}) "
                       f"+ int32 wrapping sum, inputs resident in HBM, {ROTATE} input sets alternated",
           "value": round(W * n * 4 / avg / 1e9, 2), "unit": "GB/s (worker fp32 bytes aggregated)",
           "steps": steps, "warmup": warm,
           "roofline": _hbm_roofline(algo, avg, "ina::k_quant_reduce_i32<4>"),
           "parity_spot_check": ok,
           "parity_sample": f"{idx.size} values (every 997th + both ends) vs numpy quantise + wrapping sum"}
    del sets, outs
    torch.cuda.empty_cache()
    return res


def measure_c4(dev, world=1, steps=20, warm=3, rank=0):
    """BASELINE config 4: 16 workers x 25,557,032 fp32 -> int16 saturating quantise (k=13)
    + exact sum + one final saturation, per-slot overflow flags (the ngaa_h overflow bit,
    headers.p4:30) at V = 256 (ina_quantize_reduce_f32_i16_sat).  Saturation is injected
    at ~1 of every 997 slots (half per-worker, half in the sum) so the flag count is known.
    Algorithmic bytes (4W+2) per value + 1 per slot."""
    from ina_amd import ops
    W, n, k, V = 16, RESNET50_PARAMS, 13, V_SLOT
    nslot = (n + V - 1) // V
    hot = np.arange(0, nslot, 997)
    worker_hot, sum_hot = hot[0::2], hot[1::2]
    g = torch.Generator(device=dev)
    sets = []
    for r in range(ROTATE):
        g.manual_seed(4000 + 100 * (rank * ROTATE + r))
        bufs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
        for s_ in worker_hot:                     # one worker value past 2^15 / 2^13 = 4.0
            bufs[int(s_) % W][int(s_) * V + int(s_) % V] = 8.0
        tsum = torch.from_numpy(sum_hot * V + 3).to(dev)
        for b in bufs:                            # 16 x 2048 = 32768: only the sum saturates
            b[tsum] = 0.25
        sets.append(bufs)
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(ROTATE)]
    flags = [torch.empty(nslot, dtype=torch.uint8, device=dev) for _ in range(ROTATE)]
    s = torch.cuda.current_stream(dev)
    barrier(world)
    avg = max_over_ranks(_time_rotating(
        lambda r: ops.quantize_reduce_i16(sets[r], k, V, out=outs[r], overflow=flags[r]),
        ROTATE, steps, warm, s), world)
    last = (steps - 1) % ROTATE
    # values: the strided sample plus every value of the hot slots; flags: every slot
    idx = np.unique(np.concatenate([_sample_idx(n), (hot[:, None] * V + np.arange(V)).ravel()]))
    idx = idx[idx < n]
    ti = torch.from_numpy(idx).to(dev)
    acc = np.zeros(idx.size, np.int64)
    sat = np.zeros(idx.size, bool)
    for x in sets[last]:
        q, sw = _np_q16(x[ti].cpu().numpy(), k)
        acc += q
        sat |= sw
    sat |= (acc > 32767) | (acc < -32768)
    want_v = np.clip(acc, -32768, 32767).astype(np.int16)
    got_f = flags[last].cpu().numpy()
    want_f = np.zeros(nslot, np.uint8)
    want_f[np.unique(idx[sat] // V)] = 1          # randn * 1e-2 never reaches 4.0 elsewhere
    ok = bool(np.array_equal(outs[last][ti].cpu().numpy(), want_v)) and bool(np.array_equal(got_f, want_f))
    ok = all_ranks_true(ok, world)
    algo = (4 * W + 2) * n + nslot
    res = {"workload": f"C4: {W} workers x {n} fp32 (ResNet-50) -> int16 saturating quantise (k={k}) "
                       f"+ exact sum + final saturation, V={V} slot flags, {ROTATE} input sets alternated",
           "value": round(W * n * 4 / avg / 1e9, 2), "unit": "GB/s (worker fp32 bytes aggregated)",
           "steps": steps, "warmup": warm,
           "roofline": _hbm_roofline(algo, avg, "ina::k_quant_reduce_i16<16>"),
           "overflow_slots": int(got_f.sum()), "overflow_slots_injected": int(hot.size),
           "parity_spot_check": ok,
           "parity_sample": (f"{idx.size} values (every 997th, both ends, every value of the {hot.size} "
                             f"injected slots) and all {nslot} slot flags vs numpy int16 saturation")}
    del sets, outs, flags
    torch.cuda.empty_cache()
    return res


def measure_e2e(dev, world=1, reps=5, warm=1, rank=0):
    """The PCIe-inclusive rate the north star asks for: config 3's 8 x 100 MiB int32 buckets
    in PINNED host memory (what the worker sockets deliver) -> W-way reduce -> the aggregate
    back in pinned host memory, by ina_sum_reduce_host_i32: one reduce launch reading the
    buckets across PCIe in place (zero copy, the product default); the chunked H2D /
    reduce / D2H copy pipeline is timed beside it.  The call returns when the aggregate is
    in host memory, so wall time is the step time.  Its bound is the host link: the
    roofline peak is the pinned H2D rate of the same 8 x 100 MiB measured in this run (two
    copy streams), next to the PCIe Gen5 x16 spec (MI355X_MICROARCH.md)."""
    from ina_amd import ops
    W, n = W_WORKERS, N_VALUES
    gens = np.random.default_rng(5000 + rank)
    hosts = []
    for r in range(ROTATE):
        hosts.append([torch.from_numpy(gens.integers(-(1 << 20), 1 << 20, n, dtype=np.int32)).pin_memory()
                      for _ in range(W)])
    outs = [torch.empty(n, dtype=torch.int32).pin_memory() for _ in range(ROTATE)]
    scratch = torch.empty(ops.load().ina_host_reduce_scratch_bytes(W, 0), dtype=torch.uint8, device=dev)
    # the link: 8 x 100 MiB pinned H2D on two copy streams (the pipeline's own split)
    dbuf = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(W)]
    cs = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    h2d = []
    for it in range(warm + reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for w in range(W):
            with torch.cuda.stream(cs[w % 2]):
                dbuf[w].copy_(hosts[it % ROTATE][w], non_blocking=True)
        torch.cuda.synchronize()
        if it >= warm:
            h2d.append(time.perf_counter() - t0)
    del dbuf
    h2d_gbs = W * n * 4 / statistics.median(h2d) / 1e9
    def run(zero_copy):
        ops.set_tuning(host_zero_copy=zero_copy)
        ts = []
        for it in range(warm + reps):
            barrier(world)
            t0 = time.perf_counter()
            ops.sum_reduce_host(hosts[it % ROTATE], out=outs[it % ROTATE], scratch=scratch, device=dev)
            if it >= warm:
                ts.append(time.perf_counter() - t0)
        last = (warm + reps - 1) % ROTATE
        want = np.zeros(n, np.uint32)
        for h in hosts[last]:
            want += h.numpy().view(np.uint32)
        ok = all_ranks_true(bool(np.array_equal(outs[last].numpy().view(np.uint32), want)), world)
        return max_over_ranks(statistics.median(ts), world), ok

    try:
        t_pipe, ok_pipe = run(False)
        t, ok = run(True)
    finally:
        ops.set_tuning(host_zero_copy=True)
    ach = W * n * 4 / t / 1e9
    res = {"workload": (f"C3 from pinned host memory: {W} x {n} int32 (100 MiB each) -> reduce -> "
                        f"aggregate in pinned host memory (ina_sum_reduce_host_i32: one reduce launch "
                        f"reading the buckets across PCIe in place), {ROTATE} host input sets alternated"),
           "value": round(ach, 2), "unit": "GB/s (worker int32 bytes aggregated, PCIe-inclusive)",
           "ms_per_step": round(t * 1e3, 3), "steps": reps, "warmup": warm,
           "roofline": {"bound": "pcie_h2d", "achieved": round(ach, 2), "peak": round(h2d_gbs, 2),
                        "unit": "GB/s", "frac": round(ach / h2d_gbs, 4),
                        "peak_source": "pinned H2D of the same 8 x 100 MiB on two copy streams, this run",
                        "pcie_gen5_x16_spec_GBps": PCIE_SPEC_GBS,
                        "frac_of_spec": round(ach / PCIE_SPEC_GBS, 4)},
           "copy_pipeline": {"value": round(W * n * 4 / t_pipe / 1e9, 2), "ms_per_step": round(t_pipe * 1e3, 3),
                             "frac": round(W * n * 4 / t_pipe / 1e9 / h2d_gbs, 4), "parity_spot_check": ok_pipe,
                             "workload": "the same through HBM: 4 Mi-value chunks, H2D on 2 copy streams, "
                                         "reduce, D2H, over a 3-slot device ring"},
           "parity_spot_check": ok and ok_pipe, "parity_sample": f"all {n} aggregate values vs numpy wrapping sum"}
    del hosts, outs, scratch
    torch.cuda.empty_cache()
    return res


# -- the whole INA packet path, steady state (SURVEY 8f-1 + 8f-2) ---------------------------
def measure_packet_path(dev, steps=10, warm=3, rank=0, world=1, split=False, V=V_SLOT, slots=1 << 17):
    """One step of the INA data path on one GPU, as a PS co-located with the switch runs it
    in steady state: 8 workers quantise their deltas (p_w - p_global, k=16) straight into
    NGA-256 packets (DataManager.py:37 + 111-165, fused), the PS's acks of the previous
    step ride in the same switch batch in front of the packets (fragcheck.p4:26-31), the
    switch aggregates every slot (ngaa.p4:120-196) and each completed slot's sum goes from
    the switch's registers straight into the PS update p_global + (1/(W+1)) * sum * 2^-k
    (launch.py:46-50) and its ack row (ina_switch with a PS step).  Config-3 sizes: 8 x
    26,214,400 fp32, 102,400 slots.  HIP events around `steps` back-to-back steps; the
    roofline is the path's algorithmic bytes (packs, switch + PS, acks) over the step time.
    Parity: every worker packet completes its slot once, every ack frees one, and the
    update at a strided sample equals a numpy restatement bit for bit.
    split=True: the same step over split rows (include/ina.h: 16-byte header rows + aligned
    1 KiB payload rows, the same datagrams) -- ina_quantize_pack_nga_multi_split and
    ina_switch (split rows + PS step).  V=32, slots=2^20: the P4 program's own NGA-32 format
    (headers.p4:40-73) at the same config-3 size, 8 x 819,200 packets + 819,200 acks."""
    from ina_amd import ops
    W, n, k = W_WORKERS, N_VALUES, 16
    npk = n // V
    g = torch.Generator(device=dev)
    g.manual_seed(6000 + rank)
    xs = [torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)]
    glob = torch.randn(n, device=dev, generator=g) * 1e-2
    upd = torch.empty_like(glob)
    stride = ops.nga_stride(V)
    if split:
        hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=dev)      # [acks | workers]
        pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=dev)
        ack_rows = hdr[:npk]
        hdrs_w, pays_w = list(hdr[npk:].view(W, npk, 16).unbind(0)), list(pay[npk:].view(W, npk, 4 * V).unbind(0))
        big = None
    else:
        big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=dev)   # [acks | workers]
        ack_rows, rows_w = big[:npk], big[npk:].view(W, npk, stride)
    desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=dev)
    desc_ack, desc_w = desc[:npk], desc[npk:].view(W, npk)
    acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=dev)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    ws = 1.0 / (W + 1)

    descs_w = list(desc_w.unbind(0))
    outs_w = None if split else list(rows_w.unbind(0))
    bms = [w + 1 for w in range(W)]

    def pack():
        # the 8 workers' quantise + packs as ONE launch (p_global read once for all of them)
        if split:
            ops.quantize_pack_nga_multi_split(xs, k, V, bms, W, 1, 1, base=glob, num_slots=slots,
                                              hdrs=hdrs_w, pays=pays_w, descs=descs_w)
        else:
            ops.quantize_pack_nga_multi(xs, k, V, bms, W, 1, 1, base=glob, num_slots=slots,
                                        outs=outs_w, descs=descs_w)

    def switch():
        # the fused run kernel writes each ack row's descriptor beside it (ack_desc), so the
        # next step's batch -- these acks in front of the packets -- needs no gather pass
        if split:
            sw.process_apply_split(hdr, pay, 1, glob, k, ws, out=upd, ack_hdr=ack_rows, ack_desc=desc_ack,
                                   keep_forwarded=False, actions=acts, desc=desc)
        else:
            sw.process_apply(big, 1, glob, k, ws, out=upd, acks=ack_rows, keep_forwarded=False,
                             actions=acts, desc=desc, ack_desc=desc_ack)

    def step(_r=0):
        pack()
        switch()
    ops.nga_descriptors(ack_rows, out=desc_ack)    # the first step's ack rows are another switch's
    step()
    s = torch.cuda.current_stream(dev)
    barrier(world)
    avg = max_over_ranks(_time_rotating(step, 1, steps, warm, s), world)
    # phase split (after the timed region): events between the packs and the switch pass of
    # each step, medians over `steps` steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in ev:
        e[0].record(s)
        pack()
        e[1].record(s)
        switch()
        e[2].record(s)
    torch.cuda.synchronize()
    t_pack = statistics.median(e[0].elapsed_time(e[1]) for e in ev) / 1e3
    t_sw = statistics.median(e[1].elapsed_time(e[2]) for e in ev) / 1e3
    ok = bool(int((acts[npk:] == _ACT_FWD_AGG).sum()) == npk) and bool((acts[:npk] == _ACT_FWD_ACK).all())
    idx = _sample_idx(n)
    ti = torch.from_numpy(idx).to(dev)
    gl = glob[ti].cpu().numpy()
    acc = np.zeros(idx.size, np.int64)
    for x in xs:
        acc += _np_q32(x[ti].cpu().numpy() - gl, k)
    acc = ((acc + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int32)
    want = gl + (acc.astype(np.float32) * np.float32(2.0 ** -k)) * np.float32(ws)
    ok = all_ranks_true(ok and bool(np.array_equal(upd[ti].cpu().numpy().view(np.uint32),
                                                   want.astype(np.float32).view(np.uint32))), world)
    rb, npk_all = (16 + 4 * V if split else stride), W * npk
    b_pack = W * (4 * n + npk * rb) + 4 * n + W * npk * 8  # fused worker quantise + packs (one
                                                          # launch, p_global read once) + descriptors
    b_sw = (npk * 8                                       # ack descriptors (run kernel)
            + npk_all * rb + npk * (4 * V + 5) + npk_all  # switch: packets, registers, actions
            + npk * rb + 8 * n + 16 * npk)                # PS fused: acks in, local + update, ack rows
    path = b_pack + b_sw
    res = {"workload": ("INA packet path, steady state, PS fused into the switch pass: 8 workers x "
                        f"{n} fp32 -> quantise(p_w - p_global) + NGA-{V} pack -> one switch batch of "
                        f"{npk} PS acks + {npk_all} worker packets -> completed slots applied to "
                        "p_global (launch.py:46-50) + ack rows"
                        + (f" -- split rows: 16-byte header rows + {4 * V}-byte payload rows" if split else
                           f" -- packed rows: 15 + {4 * V} bytes in a {stride}-byte row")),
           "rows": "split" if split else "packed",
           "value": round(W * n * 4 / avg / 1e9, 2), "unit": "GB/s (worker fp32 bytes aggregated)",
           "ms_per_step": round(avg * 1e3, 3), "steps": steps, "warmup": warm,
           "launches_per_step": 1 + 3,
           "switch_batch_path": sw.batch_path((W + 1) * npk),
           "roofline": {"bound": "hbm", "achieved": round(path / avg / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(path / avg / 1e9 / HBM_PEAK_GBS, 4),
                        "path_bytes_per_step": int(path),
                        "measures": "the step's algorithmic bytes (all its kernels) / the step time"},
           "phases": {"worker_packs": {"kernel": ("ina::k_qpack_nga_multi_split<8>" if split else
                                                  "ina::k_qpack_nga_multi_v256<8>") + " (one launch)",
                                       "us": round(t_pack * 1e6, 1), "bytes": int(b_pack),
                                       "frac": round(b_pack / t_pack / 1e9 / HBM_PEAK_GBS, 4)},
                      "switch_and_ps": {"kernels": "k_sort_chunks, k_sort_buckets (finds 9 dense runs: "
                                                   "no sort), k_switch_run2<true> (writes the ack "
                                                   "rows and their descriptors)",
                                        "batch_path": sw.batch_path((W + 1) * npk),
                                        "us": round(t_sw * 1e6, 1), "bytes": int(b_sw),
                                        "frac": round(b_sw / t_sw / 1e9 / HBM_PEAK_GBS, 4)},
                      "measures": "HIP events between the two phases of each step, medians"},
           "parity_spot_check": ok,
           "parity_sample": (f"every worker packet completes its slot, every ack frees one; the update at "
                             f"{idx.size} positions vs numpy quantise + wrapping sum + launch.py update")}
    del xs, glob, upd, big, desc, acts, sw
    if split:
        del hdr, pay, hdrs_w, pays_w
    torch.cuda.empty_cache()
    return res


# -- the packet-stream switch on config 3 ----------------------------------------
def measure_switch(dev, reps=10, warm=2, rank=0, world=1, V=V_SLOT, slots=1 << 17, orders=None):
    """ina_switch_process over config 3 as NGA-256 packets: 8 workers x 102,400 packets
    (2^17-slot pool, keys from the pack kernels' descriptors), in worker-major and in
    round-robin arrival (a NIC interleaving the workers).  HIP events on the launch stream
    around `reps` back-to-back calls (the headline's method); the replayed batch completes
    every slot again, so no state reset sits in the timed region.  Algorithmic bytes: every
    packet read, the completing 1/W written back, each slot's registers + count + frag
    written, one action byte per packet.
    At N > 1 every rank runs its own switch on its own bucket (slots are independent,
    ngaa.p4:87-168): `us` is the max over ranks, `aggregate_GBps` all ranks' bytes / that."""
    from ina_amd import ops
    W, n = W_WORKERS, N_VALUES
    g = torch.Generator(device=dev)
    g.manual_seed(4242 + rank)
    packed = []
    npk = -(-n // V)
    samp = np.unique(np.concatenate([np.arange(0, npk, 997), [npk - 1]]))   # parity sample slots
    vidx = (samp[:, None] * V + np.arange(V)).ravel()
    vidx = vidx[vidx < n]
    want = np.zeros(vidx.size, np.uint32)
    for w in range(W):
        b = torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=dev, generator=g)
        want += b[torch.from_numpy(vidx).to(dev)].cpu().numpy().view(np.uint32)
        packed.append(ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True))
        del b
    stream = torch.cat([p for p, _ in packed])
    desc = torch.cat([d for _, d in packed])
    del packed
    pristine = stream.clone()                  # the timed calls rewrite packets in place
    npk_all, stride = stream.shape
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    acts = torch.empty(npk_all, dtype=torch.uint8, device=dev)
    algo = npk_all * stride + npk * stride + npk * (4 * V + 5) + npk_all
    s = torch.cuda.current_stream(dev)
    res = {"workload": (f"C3 as NGA-{V} packets: {W} workers x {npk:,} packets ({npk_all:,}), "
                        f"2^{slots.bit_length() - 1}-slot pool, keys from descriptors; ina_switch_process "
                        f"incl. its slot sort"),
           "algorithmic_bytes": algo, "ranks": world, "V": V, "stride": stride}
    # worker_major: 8 dense runs of consecutive slots (no sort: the run table); round_robin:
    # already in slot order (no sort); worker_major_sorted: the same worker-major batch with
    # the run table off (tuning key 18 = 0: the chunk + bucket sort); shuffled: a random
    # arrival order (the sort, unavoidably)
    gperm = torch.Generator(device=dev)
    gperm.manual_seed(77 + rank)
    # worker_major_split: the worker-major batch in split rows (16-byte header rows + aligned
    # 4V-byte payload rows: the same datagrams, include/ina.h), the run table path
    # round_robin_jitterJ: the round-robin arrival with local disorder -- every packet displaced
    # by fewer than J positions (sort key = position + U[0, J)): W sequence-ordered senders
    # (DataManager.py:116-134) interleaved by a NIC that reorders within a window (the
    # near-sorted path: per-slot lists, no sort)
    rr = torch.arange(npk_all, device=dev).view(W, npk).t().reshape(-1)
    shuf = torch.randperm(npk_all, device=dev, generator=gperm)

    def jitter(J):
        key = torch.arange(npk_all, device=dev) + torch.randint(0, J, (npk_all,), device=dev, generator=gperm)
        return rr[torch.sort(key, stable=True).indices]
    if orders is None:                         # NGA-256 defaults: the split row layout once
        orders = ("worker_major", "worker_major_split", "round_robin", "worker_major_sorted", "shuffled")
    order = {}
    for name in orders:
        base = name[:-len("_split")] if name.endswith("_split") else name
        if base == "worker_major" or base == "worker_major_sorted":
            order[name] = None
        elif base == "round_robin":
            order[name] = rr
        elif base == "shuffled":
            order[name] = shuf
        elif base.startswith("round_robin_jitter"):
            J = int(base[len("round_robin_jitter"):])
            order[name] = order.get(base) if order.get(base) is not None else jitter(J)
        else:
            raise ValueError(f"unknown arrival order {name}")
    def split_rows(rows):
        h = torch.zeros((rows.shape[0], 16), dtype=torch.uint8, device=dev)
        h[:, :15] = rows[:, :15]
        return h, rows[:, 15:15 + 4 * V].contiguous()

    def parity(perm, split=False):
        """A fresh switch over a pristine copy of the batch in this arrival order: every slot
        completes exactly once, and each sampled slot's completing packet carries the
        wrapping int32 sum of the 8 workers' values (big-endian payload at byte 15, or the
        payload row)."""
        cp = pristine.clone() if perm is None else pristine[perm]
        chk = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
        if split:
            hp, pp = split_rows(cp)
            a = chk.process_split(hp, pp, desc=desc if perm is None else desc[perm])
            cp[:, 15:15 + 4 * V] = pp
            del hp, pp
        else:
            a = chk.process(cp, desc=desc if perm is None else desc[perm])
        pos = torch.arange(npk_all, device=dev) if perm is None else torch.argsort(perm)
        ts = torch.from_numpy(samp).to(dev)
        cand = torch.stack([pos[w * npk + ts] for w in range(W)])          # [W, samples]
        fwd = a[cand] == _ACT_FWD_AGG
        ok = bool(int((a == _ACT_FWD_AGG).sum()) == npk) and bool((fwd.sum(0) == 1).all())
        at = cand.gather(0, fwd.to(torch.int64).argmax(0, keepdim=True)).reshape(-1)
        pay = cp[at, 15:15 + 4 * V].contiguous().cpu().numpy().view(">u4").reshape(-1, V)
        # the last slot may be partial: its values past n are the pack's zero padding
        got = np.concatenate([pay[i, : min(V, n - int(sl) * V)] for i, sl in enumerate(samp)]).astype(np.uint32)
        del cp, chk, a
        return ok and bool(np.array_equal(got, want))

    for name, perm in order.items():
        st, ds = (stream, desc) if perm is None else (stream[perm], desc[perm])
        split = name.endswith("_split")
        if split:
            hp, pp = split_rows(st)
            call = lambda: sw.process_split(hp, pp, acts, desc=ds)   # noqa: E731
        else:
            call = lambda: sw.process(st, acts, desc=ds)             # noqa: E731
        with _tuning(switch_runs=name != "worker_major_sorted"):
            res[name] = _time_switch_order(call, sw, acts, npk, npk_all, algo, reps, warm, s, world)
            if split:
                res[name]["rows"] = "split: 16-byte header rows + 4V-byte payload rows"
                del hp, pp
            del st, ds, call
            res[name]["parity_spot_check"] = all_ranks_true(parity(perm, split), world)
        if world > 1:
            res[name]["aggregate_GBps"] = round(world * algo / res[name]["us"] / 1e3, 1)
    for name in res:                           # the near-sorted legs beside the in-order one
        if name.startswith("round_robin_jitter") and isinstance(res[name], dict):
            ref = res.get("round_robin_split" if name.endswith("_split") else "round_robin")
            if isinstance(ref, dict) and ref.get("us"):
                res[name]["vs_round_robin"] = round(res[name]["us"] / ref["us"], 3)
    tr = _switch_traffic(V)
    for name, t in tr.items():
        if isinstance(res.get(name), dict):
            res[name]["traffic"] = t
    res["parity_sample"] = (f"{samp.size} slots (every 997th + the last): the completing packet's payload "
                            f"vs the numpy wrapping sum of the {W} workers' values, on a fresh switch "
                            f"in each arrival order; every slot completes exactly once")
    del stream, desc, sw, acts, pristine
    torch.cuda.empty_cache()
    return res


@contextlib.contextmanager
def _tuning(**kw):
    """Process-wide switch tuning for one leg, restored to the defaults however the leg ends
    (a leg that raises must not leave the later legs on a non-default path)."""
    from ina_amd import ops
    ops.set_tuning(**kw)
    try:
        yield
    finally:
        ops.set_tuning(**{k: True for k in kw})


def _time_switch_order(call, sw, acts, npk, npk_all, algo, reps, warm, s, world):
    """One arrival order of measure_switch: `warm` untimed calls, then HIP events on the launch
    stream around `reps` back-to-back calls (3 passes, median) and a pair per call beside it."""
    for _ in range(warm):
        call()
    barrier(world)
    # like the headline's avg_launch_us: one event pair around `reps` back-to-back calls
    # (a pair per call adds ~7 us of event overhead, tools/lab/event_overhead_lab.py;
    # reported beside it as us_event_pair_per_call)
    per_rep = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            call()
        e1.record(s)
        torch.cuda.synchronize()
        per_rep.append(e0.elapsed_time(e1) * 1e3 / reps)
    evs = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        call()
        e1.record(s)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    us = max_over_ranks(statistics.median(per_rep), world)
    us_pair = max_over_ranks(statistics.median(a.elapsed_time(b) for a, b in evs) * 1e3, world)
    done = int((acts == 1).sum())
    return {"us": round(us, 2), "achieved_GBps": round(algo / us / 1e3, 1),
            "frac": round(algo / us / 1e3 / HBM_PEAK_GBS, 4), "slots_completed": done,
            "ok": all_ranks_true(done == npk, world), "us_event_pair_per_call": round(us_pair, 2),
            "batch_path": sw.batch_path(npk_all)}


def _switch_traffic(V):
    """Committed PMC traffic of the run kernel per arrival order (profiles/traffic_switch_v<V>.json,
    tools/switch_traffic.py: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over
    tools/prof_switch.py, gfx950 corrections), or {} when none is committed."""
    try:
        doc = json.load(open(os.path.join(REPO, "profiles", f"traffic_switch_v{V}.json")))
    except Exception:                     # noqa: BLE001 -- no file: traffic unmeasured
        return {}
    out = {}
    for order, d in doc.get("orders", {}).items():
        out[order] = {k: d[k] for k in ("kernel", "avg_us", "hbm_read_bytes", "hbm_write_bytes",
                                         "algorithmic_bytes", "traffic_ratio") if k in d}
        out[order]["source"] = doc.get("source", "")
    return out


# -- modes ---------------------------------------------------------------------------------------
def run_check_launch(args, rank, world, backend):
    import torch.distributed as dist
    ranks = [rank]
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, rank)
        ranks = got
    if rank == 0:
        print(json.dumps({"check_launch": True, "n_gpus": world, "rccl_world": world,
                          "backend": backend, "ranks": ranks}), flush=True)


def run_sharded_headline(args, rank, world, dev, backend):
    c5 = measure_c5(args, rank, world, dev)
    torch.cuda.empty_cache()
    c5_b = measure_c5_layout_b(args, rank, world, dev)
    c5_ar = c5_pl = c5_a2a = None
    if world > 1:
        torch.cuda.empty_cache()
        c5_ar = measure_c5(args, rank, world, dev, collective="allreduce")
        torch.cuda.empty_cache()
        c5_pl = measure_c5(args, rank, world, dev, chunks=C5_CHUNKS)
        torch.cuda.empty_cache()
        c5_a2a = measure_c5(args, rank, world, dev, collective="a2a")
    return {
        "metric": c5["metric"], "value": c5["value"], "unit": "GB/s",
        "n_gpus": world, "steps": c5["steps"], "warmup": c5["warmup"],
        "ms_per_step": c5["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": c5["workload"], "values_per_worker": c5["values_per_rank"],
                   "workers": world, "shard_values": c5["shard_values"],
                   "parallelism": f"RCCL x {world}"},
        "rccl_world": world, "backend": backend,
        "phase_ms": c5["phase_ms"], "xgmi": c5["xgmi"],
        "parity_spot_check": c5["parity_spot_check"],
        "layout_b": c5_b,
        "allreduce": c5_ar,
        "pipelined": c5_pl,
        "a2a": c5_a2a,
    }


def run_reduce(args, rank, world, dev, backend):
    from ina_amd import ops
    W, n = args.workers, args.values
    # rank r owns slot range r of an N-bucket job: its own inputs (seeds per rank)
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
    # includes the kernel boundaries -- a slight over-estimate of the kernel alone); the
    # slowest rank's, so `frac` is the minimum over ranks
    my_avg_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    avg_launch_s = max_over_ranks(my_avg_s, world)
    best_avg_s = reduce_over_ranks(my_avg_s, world, "min")

    # spot check of the measured output against a numpy wrapping sum: every 997th value over
    # the whole bucket plus its first and last 4 Ki values
    last = (args.steps - 1) % ROTATE
    idx = _sample_idx(n)
    ti = torch.from_numpy(idx).to(dev)
    want = np.zeros(idx.size, np.uint32)
    for b in sets[last]:
        want += b[ti].cpu().numpy().view(np.uint32)
    parity = all_ranks_true(
        bool(np.array_equal(outs[last][ti].cpu().numpy().view(np.uint32), want)), world)

    worker_bytes = W * n * 4
    algo_bytes = (W + 1) * n * 4
    value = worker_bytes * args.steps * world / elapsed / 1e9
    achieved = algo_bytes / avg_launch_s / 1e9
    traffic, traffic_source = load_traffic(args.traffic_file, W, n)
    slots = (n + V_SLOT - 1) // V_SLOT
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
                   "slots": slots,
                   "parallelism": (f"independent replicas x {world}: rank r aggregates its own "
                                   f"config-3 bucket (slots [r*{slots}, (r+1)*{slots}) of a "
                                   f"{world}-bucket job), no data-path collective, so value grows "
                                   f"with N by construction; collective scaling is sharded_c5")},
        "rccl_world": world,
        "backend": backend,
        "devices_visible": torch.cuda.device_count(),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_source,
                     "kernel": f"{HEADLINE_KERNEL} (512 x 256 threads)",
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_launch_us": round(avg_launch_s * 1e6, 2),
                     "per_rank_frac_min": round(algo_bytes / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4),
                     "per_rank_frac_max": round(algo_bytes / best_avg_s / 1e9 / HBM_PEAK_GBS, 4)},
        "parity_spot_check": parity,
        "parity_sample": (f"{idx.size} values (every 997th over the whole bucket, the first and last "
                          f"4 Ki) vs numpy wrapping int32 sum"),
    }
    cpu_in = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # timed last: a CPU phase of seconds leaves the GPU idle and its clocks low, and
        # the GPU legs below would start inside that ramp
        s = min(args.cpu_sample, n)
        cpu_in = ([b[:s].cpu().numpy() for b in sets[last]], outs[last][:s].cpu().numpy())
    del sets, outs
    torch.cuda.empty_cache()
    if not args.no_c2:
        run_leg(line, "c2_fused", lambda: measure_c2(dev, world, rank=rank))
    if not args.no_c4:
        run_leg(line, "c4_int16", lambda: measure_c4(dev, world, rank=rank))
    if not args.no_e2e:
        run_leg(line, "e2e_pcie", lambda: measure_e2e(dev, world, rank=rank))
    if not args.no_c5:
        c5 = run_leg(line, "sharded_c5", lambda: measure_c5(args, rank, world, dev))
        run_leg(c5, "layout_b", lambda: measure_c5_layout_b(args, rank, world, dev))
        if world > 1:
            run_leg(c5, "allreduce", lambda: measure_c5(args, rank, world, dev, collective="allreduce"))
            run_leg(c5, "pipelined", lambda: measure_c5(args, rank, world, dev, chunks=C5_CHUNKS))
            run_leg(c5, "a2a", lambda: measure_c5(args, rank, world, dev, collective="a2a"))
    if not args.no_switch:
        run_leg(line, "switch_c3", lambda: measure_switch(dev, rank=rank, world=world))
        # the P4 program's own format (headers.p4:40-73, parser.p4:43-55: NGA-32, 32 x bit<32>
        # behind the 15-byte header) at config-3 size: 6,553,600 packets, a 2^20-slot pool
        # (keys of 21 bits: the 2,048-bin chunk + bucket sort, and its run / in-order paths)
        # near-sorted arrivals (round robin with local jitter, packed and split rows) beside the
        # in-order round robin, and the shuffled batch in both layouts (the full sort)
        run_leg(line, "switch_c3_v32", lambda: measure_switch(dev, rank=rank, world=world, V=32, slots=1 << 20,
                                                              orders=("worker_major", "worker_major_split",
                                                                      "round_robin", "round_robin_split",
                                                                      "round_robin_jitter64",
                                                                      "round_robin_jitter64_split",
                                                                      "round_robin_jitter4096",
                                                                      "round_robin_jitter4096_split",
                                                                      "shuffled", "shuffled_split")))
        # the INA step in the split-row layout (the device format: same datagrams on the wire,
        # aligned payload rows), and in packed 1,040-byte rows beside it
        run_leg(line, "packet_path", lambda: measure_packet_path(dev, rank=rank, world=world, split=True))
        run_leg(line, "packet_path_packed", lambda: measure_packet_path(dev, rank=rank, world=world))
        # the same step in NGA-32 packets (the P4 program's format), split rows, 2^20 slots
        run_leg(line, "packet_path_v32", lambda: measure_packet_path(dev, rank=rank, world=world, split=True,
                                                                     V=32, slots=1 << 20))
    if cpu_in is not None:
        run_leg(line, "cpu_baseline", lambda: cpu_baseline(args, *cpu_in))
    return line


def legs_summary(line: dict) -> dict:
    """The JSON line's last key: one compact entry per leg -- us (per launch, call or step),
    roofline frac, parity spot check (and the switch's batch path) -- so the whole run reads
    at a glance; the full legs stay under their own keys."""
    def one(d):
        if not isinstance(d, dict):
            return None
        if "error" in d:
            return {"error": d["error"][:120]}
        rf = d.get("roofline") if isinstance(d.get("roofline"), dict) else {}
        us = d.get("us") or rf.get("avg_launch_us") or (d["ms_per_step"] * 1e3 if d.get("ms_per_step") else None)
        e = {"us": round(float(us), 1) if us else None, "frac": d.get("frac", rf.get("frac")),
             "parity": d.get("parity_spot_check")}
        if d.get("batch_path") or d.get("switch_batch_path"):
            e["path"] = d.get("batch_path") or d.get("switch_batch_path")
        return e
    out = {"headline": one(line)}
    for key in ("c2_fused", "c4_int16", "e2e_pcie", "sharded_c5", "packet_path", "packet_path_packed",
                "packet_path_v32"):
        if key in line:
            out[key] = one(line[key])
    c5 = line.get("sharded_c5")
    if isinstance(c5, dict):
        for sub in ("layout_b", "allreduce", "pipelined", "a2a"):
            if isinstance(c5.get(sub), dict):
                out[f"sharded_c5.{sub}"] = one(c5[sub])
    for sw in ("switch_c3", "switch_c3_v32"):
        d = line.get(sw)
        if isinstance(d, dict) and "error" in d:
            out[sw] = one(d)
        elif isinstance(d, dict):
            for k, v in d.items():
                if isinstance(v, dict) and "us" in v:
                    out[f"{sw}.{k}"] = one(v)
    cb = line.get("cpu_baseline")
    if isinstance(cb, dict):
        out["cpu_baseline"] = {"value": cb.get("value"), "unit": cb.get("unit"), "parity": cb.get("matches_gpu")}
    return out


def run_leg(parent: dict, key: str, fn) -> dict:
    """parent[key] = fn(), or {"error": ...} if the leg raises: a leg that fails the same
    way on every rank (an RCCL or memory error at some N) is reported in the line instead of
    taking the headline down with it.  Returns the leg's dict."""
    try:
        parent[key] = fn()
    except Exception as e:          # noqa: BLE001 -- reported in the JSON line
        parent[key] = {"error": f"{type(e).__name__}: {str(e)[:400]}"}
    try:
        torch.cuda.empty_cache()
    except Exception:               # noqa: BLE001 -- a sticky device error is already reported
        pass
    return parent[key]


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    rank, world, local, backend = init_dist(args)
    try:
        if args.check_launch:
            run_check_launch(args, rank, world, backend)
            return
        dev = torch.device(f"cuda:{local}")
        if args.mode == "sharded":
            line = run_sharded_headline(args, rank, world, dev, backend)
        else:
            line = run_reduce(args, rank, world, dev, backend)
        if rank == 0 and args.extra:
            from bench_extra import run_extra
            extra = run_extra(dev)
            os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
            json.dump(extra, open(os.path.join(REPO, "gpurun_out", "bench_extra.json"), "w"), indent=1)
        if rank == 0:
            line["legs"] = legs_summary(line)      # the last key
            print(json.dumps(line), flush=True)
    finally:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
