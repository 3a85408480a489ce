mkdir -p gpurun_out/r03b
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "switch" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b/switch_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03b/switch_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_r02sort.so tools/lab/libina_r03sort.so > gpurun_out/r03b/switch_lab_wm.log 2>&1 || exit $?
ORDER=rr timeout -k 10 200 python tools/lab/switch_lab.py tools/lab/libina_r02sort.so tools/lab/libina_r03sort.so > gpurun_out/r03b/switch_lab_rr.log 2>&1 || exit $?
cat gpurun_out/r03b/switch_lab_wm.log gpurun_out/r03b/switch_lab_rr.log
