#!/bin/bash
# Copy one gpu_session.sh run (stages bench prof pmc extra swprof) into profiles/r01 and
# regenerate the traffic summaries.  usage: tools/refresh_profiles.sh TAG
set -eu
TAG=$1
S=gpurun_out/$TAG
D=profiles/r01
cp "$S/bench.json" "$D/bench.json"
cp "$S/prof/run_kernel_stats.csv" "$D/kernel_stats_bench.csv"
cp "$S/pmc_FETCH_SIZE/run_counter_collection.csv" "$D/pmc_FETCH_SIZE.csv"
cp "$S/pmc_WRITE_SIZE/run_counter_collection.csv" "$D/pmc_WRITE_SIZE.csv"
python tools/pmc_traffic.py "$S" "k_sum_reduce_i32_vec<8, 4, true>" profiles/traffic_sum_reduce_c3.json > /dev/null
cp "$S/swprof/run_kernel_stats.csv" "$D/kernel_stats_switch.csv"
cp "$S/swpmc_FETCH_SIZE/run_counter_collection.csv" "$D/switch_pmc_FETCH_SIZE.csv"
cp "$S/swpmc_WRITE_SIZE/run_counter_collection.csv" "$D/switch_pmc_WRITE_SIZE.csv"
python tools/switch_traffic.py "$S" profiles/traffic_switch.json "$TAG" > /dev/null
cp "$S/bench_extra.json" "$D/bench_extra.json"
echo "profiles refreshed from $TAG"
python tools/design_table.py "$TAG" && python tools/profiles_readme.py "$TAG"
