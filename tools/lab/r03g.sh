# host-path tests (zero copy and pipeline), C ABI binary, bench contract, bench, profile
mkdir -p gpurun_out/r03g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capi_binary.py -k "sum_reduce_host or capi or quant_reduce" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/host_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03g/host_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r03g bench contract prof
