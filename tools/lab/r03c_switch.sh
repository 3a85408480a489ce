# switch sort A/B (r02 bucket + local vs r03 chunk + bucket) and a rocprof kernel split of the new sort
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "switch or absmax" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c/switch_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03c/switch_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_r02sort.so tools/lab/libina_r03sort.so > gpurun_out/r03c/switch_lab_wm.log 2>&1 || exit $?
ORDER=rr timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_r02sort.so tools/lab/libina_r03sort.so > gpurun_out/r03c/switch_lab_rr.log 2>&1 || exit $?
REPS=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c/swprof -o run -- python3 tools/prof_switch.py > gpurun_out/r03c/swprof.log 2>&1 || exit $?
cat gpurun_out/r03c/switch_lab_wm.log gpurun_out/r03c/switch_lab_rr.log
