# per-kernel profile of the fused steady-state packet path and of the switch in random
# arrival, with the current library but round 2's switch source (tools/lab/libina_r02sw.so) and the current one
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/path_ab
L=distributed-training-ina_amd/ina_amd/libina.so
cp $L gpurun_out/path_ab/keep.so
for v in r02 cur; do
  [ $v = r02 ] && cp tools/lab/libina_r02sw.so $L
  [ $v = cur ] && cp gpurun_out/path_ab/keep.so $L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/path_ab/path_$v -o run -- python3 tools/prof_path.py > gpurun_out/path_ab/path_$v.log 2>&1 || { cp gpurun_out/path_ab/keep.so $L; exit 1; }
  ORDER=random REPS=6 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/path_ab/rand_$v -o run -- python3 tools/prof_switch.py > gpurun_out/path_ab/rand_$v.log 2>&1 || { cp gpurun_out/path_ab/keep.so $L; exit 1; }
done
cp gpurun_out/path_ab/keep.so $L
python - <<'PY'
import csv
for tag in ("path_r02", "path_cur", "rand_r02", "rand_cur"):
    print(tag)
    for r in csv.DictReader(open(f"gpurun_out/path_ab/{tag}/run_kernel_stats.csv")):
        if "ina::" in r["Name"]:
            print(f"   {r['Name'][:58]:58s} {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
