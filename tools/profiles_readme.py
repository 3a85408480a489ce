#!/usr/bin/env python3
"""Write profiles/README.md from the committed evidence files.  usage: profiles_readme.py TAG"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
tag = sys.argv[1]
b = json.load(open(os.path.join(P, "r01", "bench.json")))
tr = json.load(open(os.path.join(P, "traffic_sum_reduce_c3.json")))
sw = json.load(open(os.path.join(P, "traffic_switch.json")))["kernels"]
prof = next(float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(os.path.join(P, "r01", "kernel_stats_bench.csv")))
            if "k_sum_reduce_i32_vec<8, 4, true>" in r["Name"])
run2 = next(k for k in sw if "run2" in k)
keys = next(k for k in sw if "keys" in k)
sort_us = sum(v["avg_us"] for k, v in sw.items() if "k_rs_" in k)
rf, cb = b["roofline"], b["cpu_baseline"]
txt = f"""# profiles/

Round-1 evidence, all from MI355X boxes via gpurun.  The files in `r01/` come from ONE
session on the final round-1 code (`tools/gpu_session.sh {tag} smoke test bench prof pmc
extra swprof`, copied by `tools/refresh_profiles.sh {tag}`).  The same bench line on other
boxes this round: 5.53-5.83 TB/s aggregated, 143.4-150.7 us per launch = 78-82 % of peak
(r01zc 143.4 us, r01j/r01t 147.2 us, r01y 150.7 us).

| file | what |
|---|---|
| `r01/bench.json` | the bench.py line (N=1, 50 steps): {b['value']:,.0f} GB/s aggregated; sum-reduce {rf['avg_launch_us']} us/launch = {rf['achieved']:,.0f} GB/s = {100 * rf['frac']:.1f} % of 8 TB/s; cpu_baseline {cb['value']} GB/s on {cb['cores']} host threads over the whole 8 x 100 MiB bucket ({cb['value_1core']} GB/s on one core) |
| `r01/kernel_stats_bench.csv` | `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline`: `k_sum_reduce_i32_vec<8,4,true>` average {prof:.1f} us (bench events: {rf['avg_launch_us']} us) |
| `r01/pmc_FETCH_SIZE.csv`, `r01/pmc_WRITE_SIZE.csv` | two separate `rocprofv3 --pmc` passes over `bench.py --steps 10`; per-launch traffic computed by `tools/pmc_traffic.py` into `traffic_sum_reduce_c3.json` (FETCH_SIZE doubled: gfx950 half-count of 16 B/lane streams; KiB units) = {tr['hbm_bytes_per_launch'] / 1e6:.2f} MB vs {tr['algorithmic_bytes'] / 1e6:.2f} MB algorithmic |
| `traffic_sum_reduce_c3.json` | the `roofline.traffic` source read by bench.py |
| `r01/bench_extra.json` | `bench.py --extra`: every other kernel (configs 2/4, quantise, pack/unpack, fused worker pack, fused PS apply, absmax, C-128, PS combine, device switch, the whole packet path step, end-to-end with pinned H2D/D2H -- phases in sequence and the pipelined `ina_sum_reduce_host_i32`) and the grid sweeps; cold caches (512 MiB read between timed launches); DESIGN.md's kernel table is generated from it (`tools/design_table.py`) |
| `r01/kernel_stats_switch.csv` | rocprofv3 stats of `tools/prof_switch.py` (device switch on 819,200 NGA-256 packets): `k_switch_run2` {sw[run2]['avg_us']} us, keys {sw[keys]['avg_us']} us, sort passes {sort_us:.1f} us |
| `r01/switch_pmc_FETCH_SIZE.csv`, `r01/switch_pmc_WRITE_SIZE.csv`, `traffic_switch.json` | PMC passes over the same program; per-kernel HBM bytes and rates computed by `tools/switch_traffic.py` (run kernel {(sw[run2]['hbm_read_bytes'] + sw[run2]['hbm_write_bytes']) / 1e9:.2f} GB at {sw[run2]['TB_per_s']} TB/s) |
| `r01/bench_boxes.json` | the same bench line on every box of the round's evidence sessions (8 boxes: 77.9-82.3 % of peak, median 79.8 %) |
| `r01/kernel_stats_packet_path.csv` | rocprofv3 stats of `tools/prof_path.py`: the steady-state packet path with the PS step fused (per step: 8 x `k_pack_nga_flat<SrcQ32,1>` 54.5 us, `k_switch_run2<true>` 235 us, keys 37 us, sort passes 47 us) |
| `r01/sharded_c5_1gpu.json`, `r01/rehearse_2ranks_gloo.json`, `r01/config1_loopback.log` | session r01zf: `bench.py --mode sharded` on one GPU (config 5 plumbing, collectives are identities); bench.py at N=2 over gloo with both ranks on one GPU (the multi-rank timing/reduction path); `examples/config1_loopback.py` (config 1: ResNet-50, 2 workers, loopback sockets, device switch stand-in) |
| `r01/lab/*.log` | interleaved A/B labs (`tools/lab/`): reduce structures, grids, store and copy cache policies; fused-kernel grids and chunks in flight; int16 layouts; C-128 pack; switch run/sort variants, nt loads, tail-chunk policy, sort chunk geometry; PS apply batch/window/action scan; packet-path stage times |
| `r01/lab/switch_pmc_run2_vs_run3.txt` | PMC counters (SQ instruction/wait mix, TCC, FETCH/WRITE) of the switch run kernel vs the scalar-header rewrite (`tools/lab/switch_pmc.sh`) |
"""
open(os.path.join(P, "README.md"), "w").write(txt)
print("profiles/README.md written for", tag)
