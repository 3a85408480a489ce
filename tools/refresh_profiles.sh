#!/bin/bash
# Copy one gpu_session.sh run (stages test bench prof pmc extra swprof [rehearse sharded
# config1 pathprof]) into profiles/<round> and regenerate the traffic summaries.
# usage: tools/refresh_profiles.sh TAG
set -eu
TAG=$1
S=gpurun_out/$TAG
D=profiles/${INA_EVIDENCE_ROUND:-r03}
mkdir -p "$D"
cp "$S/bench.json" "$D/bench.json"
cp "$S/prof/run_kernel_stats.csv" "$D/kernel_stats_bench.csv"
cp "$S/pmc_FETCH_SIZE/run_counter_collection.csv" "$D/pmc_FETCH_SIZE.csv"
cp "$S/pmc_WRITE_SIZE/run_counter_collection.csv" "$D/pmc_WRITE_SIZE.csv"
python tools/pmc_traffic.py "$S" "k_sum_reduce_i32_vec<8, 4, true>" profiles/traffic_sum_reduce_c3.json > /dev/null
cp "$S/swprof/run_kernel_stats.csv" "$D/kernel_stats_switch.csv"
cp "$S/swpmc_FETCH_SIZE/run_counter_collection.csv" "$D/switch_pmc_FETCH_SIZE.csv"
cp "$S/swpmc_WRITE_SIZE/run_counter_collection.csv" "$D/switch_pmc_WRITE_SIZE.csv"
python tools/switch_traffic.py "$S" "$D/traffic_switch.json" "$TAG" > /dev/null
cp "$S/bench_extra.json" "$D/bench_extra.json"
# optional stages
[ -f "$S/pytest_gpu.log" ] && cp "$S/pytest_gpu.log" "$D/pytest_gpu.log"
[ -f "$S/rehearse2.json" ] && cp "$S/rehearse2.json" "$D/rehearse_2ranks_gloo.json"
[ -f "$S/rehearse8.json" ] && grep '^{' "$S/rehearse8.json" > "$D/rehearse_8ranks_gloo.json"
[ -f "$S/sharded1_i32.json" ] && cp "$S/sharded1_i32.json" "$D/sharded_c5_1gpu_i32.json"
[ -f "$S/sharded1_i16.json" ] && cp "$S/sharded1_i16.json" "$D/sharded_c5_1gpu_i16.json"
[ -f "$S/config1.log" ] && cp "$S/config1.log" "$D/config1_loopback.log"
[ -f "$S/pathprof/run_kernel_stats.csv" ] && cp "$S/pathprof/run_kernel_stats.csv" "$D/kernel_stats_packet_path.csv"
echo "profiles refreshed from $TAG into $D"
