#!/usr/bin/env python3
"""Write profiles/README.md from the committed evidence files of one round
(INA_EVIDENCE_ROUND, default r02) and the driver's own bench lines (BENCH_r*.json).

usage: profiles_readme.py SESSION_TAG"""
import csv
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
RD = os.environ.get("INA_EVIDENCE_ROUND", "r02")
tag = sys.argv[1]
R = os.path.join(P, RD)


def jl(name):
    return json.load(open(os.path.join(R, name)))


b = jl("bench.json")
tr = json.load(open(os.path.join(P, "traffic_sum_reduce_c3.json")))
sw = jl("traffic_switch.json")["kernels"]
prof = next(float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(os.path.join(R, "kernel_stats_bench.csv")))
            if "k_sum_reduce_i32_vec<8, 4, true>" in r["Name"])
run2 = next(k for k in sw if "run2" in k)
keys = next(k for k in sw if "keys" in k)
sort_us = sum(v["avg_us"] for k, v in sw.items() if "k_rs_" in k)
rf, cb = b["roofline"], b["cpu_baseline"]
c5 = b.get("sharded_c5", {})
drivers = []
for f in sorted(f for f in os.listdir(REPO) if re.fullmatch(r"BENCH_r\d+\.json", f)):
    try:
        d = json.load(open(os.path.join(REPO, f)))["parsed"]["roofline"]
        drivers.append(f"`{f}` {d['avg_launch_us']} us = {100 * d['frac']:.1f} %")
    except Exception:
        pass
opt = [(n, w) for n, w in (
    ("rehearse_2ranks_gloo.json", "bench.py --gpus 2 with no launcher: it starts two ranks itself (torch.distributed.run), both on the box's one GPU over gloo -- the multi-rank timing, max-over-ranks and the config-5 sharded path with device quantise/decode (collectives staged through host memory), with its all-reduce and 4-chunk pipelined variants (session r02o)"),
    ("rehearse_8ranks_gloo.json", "bench.py --gpus 8 starting its own 8 ranks, all on the box's one GPU over gloo: the N = 8 flow end to end (group-size assert, max-over-ranks timing, the 8-way config-5 shard plan, layout B, the all-reduce and pipelined variants, parity spot checks; session r02o); throughput numbers are meaningless with 8 ranks on one GPU"),
    ("bench_boxes.json", "the headline line on every box of this round's evidence sessions, next to the driver's round-1 line"),
    ("sharded_c5_1gpu_i32.json", "bench.py --mode sharded --wire i32: config 5 (1 GiB fp32 per rank) as the headline on one GPU; the collectives are identities at N = 1"),
    ("sharded_c5_1gpu_i16.json", "the same on the int16 saturating wire (q16 + saturation count in one int32 SUM, saturate once)"),
    ("config1_loopback.log", "examples/config1_loopback.py: config 1 (ResNet-50 parameter count, 2 workers, loopback sockets, device switch stand-in)"),
    ("kernel_stats_packet_path.csv", "rocprofv3 stats of tools/prof_path.py: the steady-state packet path with the PS step fused into the switch pass"),
    ("pytest_gpu.log", "the GPU suite (python -m pytest tests -m gpu) on the same box"),
) if os.path.exists(os.path.join(R, n))]
rows = "\n".join(f"| `{RD}/{n}` | {w} |" for n, w in opt)
txt = f"""# profiles/

Evidence from MI355X boxes via gpurun.  `{RD}/` holds ONE session on the final code of
this round (`tools/gpu_session.sh {tag} ...`, copied by `tools/refresh_profiles.sh {tag}`);
`r01/` is round 1's (kept as history, named in round 1's VERDICT).  The driver's own runs
of the headline bench on fresh boxes: {"; ".join(drivers) if drivers else "none yet"}.

| file | what |
|---|---|
| `{RD}/bench.json` | the bench.py line (N=1, 50 steps): {b['value']:,.0f} GB/s aggregated; sum-reduce {rf['avg_launch_us']} us/launch = {rf['achieved']:,.0f} GB/s = {100 * rf['frac']:.1f} % of 8 TB/s; cpu_baseline {cb['value']} GB/s at {cb['cores']} host threads (best of {sorted(int(k) for k in cb.get('value_by_threads', {}))} threads; affinity mask {cb.get('affinity_cores')} CPUs, cgroup quota {cb.get('cgroup_cpu_quota')} CPUs; {cb['value_1core']} GB/s on one core); config 5 at N = 1 {c5.get('value')} GB/s ({c5.get('ms_per_step')} ms per 1 GiB step) |
| `{RD}/kernel_stats_bench.csv` | `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline`: `k_sum_reduce_i32_vec<8,4,true>` average {prof:.1f} us (bench events: {rf['avg_launch_us']} us) |
| `{RD}/pmc_FETCH_SIZE.csv`, `{RD}/pmc_WRITE_SIZE.csv` | two separate `rocprofv3 --pmc` passes over `bench.py --steps 10`; per-launch traffic computed by `tools/pmc_traffic.py` into `traffic_sum_reduce_c3.json` (FETCH_SIZE doubled: gfx950 half-count of 16 B/lane streams; KiB units) = {tr['hbm_bytes_per_launch'] / 1e6:.2f} MB vs {tr['algorithmic_bytes'] / 1e6:.2f} MB algorithmic |
| `traffic_sum_reduce_c3.json` | the `roofline.traffic` source read by bench.py |
| `{RD}/bench_extra.json` | `bench.py --extra`: every other kernel (configs 2/4/5, quantise, pack/unpack, fused worker pack, fused PS apply, absmax, C-128, PS combine, device switch, the whole packet path step, end-to-end with pinned H2D/D2H) and the grid sweeps; cold caches (512 MiB read between timed launches); DESIGN.md's kernel table is generated from it (`tools/design_table.py`) |
| `{RD}/kernel_stats_switch.csv` | rocprofv3 stats of `tools/prof_switch.py` (device switch on 819,200 NGA-256 packets, keys from the pack kernels' descriptors): `k_switch_run2` {sw[run2]['avg_us']} us, keys {sw[keys]['avg_us']} us, sort {sort_us:.1f} us |
| `{RD}/switch_pmc_FETCH_SIZE.csv`, `{RD}/switch_pmc_WRITE_SIZE.csv`, `{RD}/traffic_switch.json` | PMC passes over the same program; per-kernel HBM bytes and rates computed by `tools/switch_traffic.py` (run kernel {(sw[run2]['hbm_read_bytes'] + sw[run2]['hbm_write_bytes']) / 1e9:.2f} GB at {sw[run2]['TB_per_s']} TB/s) |
{rows}
| `{RD}/lab/*` | interleaved A/B labs of this round (`tools/lab/`): slot sort variants (r01 passes, one-sweep, bucket + local), bucket workgroup waves, foreign-bucket skip, batched action stores, run-kernel window/batch/occupancy/prefetch/register-store policy, the run kernel's gather floor (`gather_lab.json`), switch arrival orders, the XCD-aware window map (`switch_lab_xcd.log`, and the same map on the flat packet kernels, `flat_lab_xcd.log`), head-chunk load policy, fused-PS occupancy and row prefetch, unpack header fields and pack descriptors as coalesced passes (`unpack_hdr_lab.log`, `pack_desc_lab.log`), elementwise and packet-kernel grid caps, absmax geometry, HIP-event overhead, lab buffer-placement check, a 600-seed switch fuzz on the final code (`fuzz_many.log`) |
| `r01/` | round 1: the same files for round 1's code, its labs (`r01/lab/`), the per-box bench spread (`r01/bench_boxes.json`) |
"""
open(os.path.join(P, "README.md"), "w").write(txt)
print("profiles/README.md written for", tag)
