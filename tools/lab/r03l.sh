# bucket tile 4096 (lc4) vs 8192 (lc8) items; the packet path with sc1 vs nt streaming stores
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "switch" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l/switch_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03l/switch_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_lc4.so tools/lab/libina_lc8.so > gpurun_out/r03l/lc_wm.log 2>&1 || exit 1
ORDER=rr timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_lc4.so tools/lab/libina_lc8.so > gpurun_out/r03l/lc_rr.log 2>&1 || exit 1
L=distributed-training-ina_amd/ina_amd/libina.so
cp $L gpurun_out/r03l/keep.so
for v in lc4 lc8 nt; do
  cp tools/lab/libina_$v.so $L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03l/path_$v -o run -- python3 tools/prof_path.py > gpurun_out/r03l/path_$v.log 2>&1 || { cp gpurun_out/r03l/keep.so $L; exit 1; }
done
cp gpurun_out/r03l/keep.so $L
grep -v amdgpu gpurun_out/r03l/lc_wm.log gpurun_out/r03l/lc_rr.log
python - <<'PY'
import csv
for tag in ("path_lc4", "path_lc8", "path_nt"):
    tot = 0.0
    rows = []
    for r in csv.DictReader(open(f"gpurun_out/r03l/{tag}/run_kernel_stats.csv")):
        if "ina::" in r["Name"]:
            avg = float(r['AverageNs']) / 1e3
            per_step = avg * int(r['Calls']) / 6
            tot += per_step
            rows.append(f"   {r['Name'][:58]:58s} {r['Calls']:>4} avg {avg:8.2f} us")
    print(tag, f"kernel time per step {tot:.1f} us"); print("\n".join(rows))
PY
