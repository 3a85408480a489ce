#!/bin/bash
# Copy one evidence session (gpu_session.sh stages smoke test contract bench prof pmc swprof
# swtrace:SPLIT=1 swpmc:SPLIT=1 pathtrace:SPLIT=1 pathpmc:SPLIT=1 pathtrace:SPLIT=0
# swtrace:V=32,SLOTS=1048576,ORDER=wm [...]) into profiles/<round> and regenerate the traffic
# summaries.  Stages that did not run are skipped.
# usage: tools/refresh_profiles.sh TAG        (INA_EVIDENCE_ROUND=r05 by default)
set -eu
TAG=$1
S=gpurun_out/$TAG
D=profiles/${INA_EVIDENCE_ROUND:-r05}
mkdir -p "$D/pmc"
cpif() { [ -f "$1" ] && cp "$1" "$2" || true; }
cpif "$S/bench.json" "$D/bench.json"
for f in pytest_gpu.log pytest_gpu_storecheck.log contract.log smoke.log; do cpif "$S/$f" "$D/$f"; done
cpif "$S/prof/run_kernel_stats.csv" "$D/kernel_stats_bench.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  cpif "$S/pmc_$c/run_counter_collection.csv" "$D/pmc/bench_$c.csv"
  cpif "$S/swpmc_$c/run_counter_collection.csv" "$D/pmc/switch_$c.csv"
  cpif "$S/swpmc_SPLIT_1_$c/run_counter_collection.csv" "$D/pmc/switch_split_$c.csv"
  cpif "$S/pathpmc_SPLIT_1_$c/run_counter_collection.csv" "$D/pmc/packet_path_split_$c.csv"
done
[ -d "$S/pmc_FETCH_SIZE" ] && python tools/pmc_traffic.py "$S" "k_sum_reduce_i32_vec<8, 4, true>" \
  profiles/traffic_sum_reduce_c3.json > /dev/null
cpif "$S/swprof/run_kernel_stats.csv" "$D/kernel_stats_switch.csv"
[ -d "$S/swprof" ] && python tools/switch_traffic.py "$S" "$D/traffic_switch.json" "$TAG" > /dev/null
cpif "$S/swtrace_SPLIT_1/run_kernel_stats.csv" "$D/kernel_stats_switch_split.csv"
[ -d "$S/swtrace_SPLIT_1" ] && python tools/switch_traffic.py "$S" "$D/traffic_switch_split.json" "$TAG" SPLIT_1 > /dev/null
cpif "$S/pathtrace_SPLIT_1_TRACE/run_kernel_stats.csv" "$D/kernel_stats_packet_path_split.csv"
[ -d "$S/pathpmc_SPLIT_1_FETCH_SIZE" ] && python tools/path_traffic.py "$S" "$D/traffic_packet_path_split.json" "$TAG" > /dev/null
cpif "$S/pathtrace_SPLIT_0_TRACE/run_kernel_stats.csv" "$D/kernel_stats_packet_path_packed.csv"
cpif "$S/swtrace_V_32_SLOTS_1048576_ORDER_wm/run_kernel_stats.csv" "$D/kernel_stats_switch_v32_wm.csv"
cpif "$S/bench_extra.json" "$D/bench_extra.json"
cpif "$S/rehearse2.json" "$D/rehearse_2ranks_gloo.json"
[ -f "$S/rehearse8.json" ] && grep '^{' "$S/rehearse8.json" > "$D/rehearse_8ranks_gloo.json" || true
cpif "$S/sharded1_i32.json" "$D/sharded_c5_1gpu_i32.json"
cpif "$S/sharded1_i16.json" "$D/sharded_c5_1gpu_i16.json"
cpif "$S/config1.log" "$D/config1_loopback.log"
# every switch / packet-path trace and PMC pass of the session (swtrace:K=V,.. swpmc:K=V,..
# pathtrace:K=V,..), named after its env
for d in "$S"/swtrace_* "$S"/pathtrace_*; do
  [ -f "$d/run_kernel_stats.csv" ] && cp "$d/run_kernel_stats.csv" "$D/kernel_stats_$(basename "$d").csv"
done
for d in "$S"/swpmc_*; do
  [ -f "$d/run_counter_collection.csv" ] && cp "$d/run_counter_collection.csv" "$D/pmc/$(basename "$d").csv"
done
echo "profiles refreshed from $TAG into $D"
