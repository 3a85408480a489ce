set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "switch or pack or unpack or apply" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03m/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m/path -o run -- python3 tools/prof_path.py > gpurun_out/r03m/path.log 2>&1 || exit 1
timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_lc4.so tools/lab/libina_sweep.so > gpurun_out/r03m/sw_wm.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r03m/sw_wm.log
python - <<'PY'
import csv
tot = 0.0
for r in csv.DictReader(open("gpurun_out/r03m/path/run_kernel_stats.csv")):
    if "ina::" in r["Name"]:
        avg = float(r['AverageNs']) / 1e3
        tot += avg * int(r['Calls']) / 6
        print(f"   {r['Name'][:58]:58s} {r['Calls']:>4} avg {avg:8.2f} us")
print(f"kernel time per step {tot:.1f} us")
PY
