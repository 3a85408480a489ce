#!/bin/bash
# GPU-box session: parity tests -> bench -> rocprofv3 kernel trace -> PMC passes.
# Every GPU step has its own time limit; the script stops at the first crash,
# abort or timeout (only an ordinary pytest failure, rc 1, lets it continue).
# usage: tools/gpu_session.sh TAG [stages...]   stages: smoke test bench prof pmc extra swprof
#        contract config1 rehearse rehearse8 sharded swlab pathprof
#        lab:<name> (tools/lab/<name>.py)   ptest:<expr> (GPU tests -k <expr>, or -k "$PTEST_K")
set -u
TAG=${1:-r02}; shift || true
STAGES=${*:-"smoke test bench prof pmc extra"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { echo "STOP after $1 (rc=$2)"; exit "$2"; }
ok_or_fail() { local rc=$2; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then fatal "$1" "$rc"; fi; }
for st in $STAGES; do
  case $st in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -3 "$OUT/smoke.log"; [ $rc -ne 0 ] && fatal smoke $rc ;;
    test)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -25 "$OUT/pytest_gpu.log"; ok_or_fail pytest $rc ;;
    testchk)
      # the whole GPU suite under the checked stream_store build (make -C csrc storecheck)
      INA_LIBRARY=libina_storecheck.so timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 120 \
        --timeout-method thread > "$OUT/pytest_gpu_storecheck.log" 2>&1
      rc=$?; tail -25 "$OUT/pytest_gpu_storecheck.log"; ok_or_fail pytest_storecheck $rc ;;
    lab:*)
      nm=${st#lab:}
      timeout -k 10 300 python tools/lab/$nm.py > "$OUT/$nm.log" 2>&1
      rc=$?; cat "$OUT/$nm.log"; [ $rc -ne 0 ] && fatal "$st" $rc ;;
    pfile:*)
      f=${st#pfile:}
      timeout -k 10 600 python -u -m pytest tests/$f -m gpu -q -rf --timeout 120 --timeout-method thread \
        > "$OUT/pfile_${f%.py}.log" 2>&1
      rc=$?; tail -15 "$OUT/pfile_${f%.py}.log"; ok_or_fail "$st" $rc ;;
    ptest:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread \
        -k "${PTEST_K:-${st#ptest:}}" > "$OUT/ptest.log" 2>&1
      rc=$?; tail -8 "$OUT/ptest.log"; ok_or_fail "$st" $rc ;;
    ew16lab)
      timeout -k 10 300 python tools/lab/ew16_lab.py > "$OUT/ew16_lab.log" 2>&1
      rc=$?; cat "$OUT/ew16_lab.log"; [ $rc -ne 0 ] && fatal ew16lab $rc ;;
    bkphase)
      timeout -k 10 200 python tools/lab/bucket_phase_lab.py > "$OUT/bucket_phase_lab.log" 2>&1
      rc=$?; cat "$OUT/bucket_phase_lab.log"; [ $rc -ne 0 ] && fatal bkphase $rc ;;
    zerocopy)
      timeout -k 10 200 python tools/lab/zerocopy_lab.py > "$OUT/zerocopy_lab.log" 2>&1
      rc=$?; cat "$OUT/zerocopy_lab.log"; [ $rc -ne 0 ] && fatal zerocopy $rc ;;
    contract)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_contract.py -m gpu -v -rf --timeout 600 --timeout-method thread > "$OUT/contract.log" 2>&1
      rc=$?; tail -8 "$OUT/contract.log"; ok_or_fail contract $rc ;;
    bench)
      # the driver's own command (BENCH_rNN.json), so the session's line and the driver's are the
      # same measurement
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; [ $rc -ne 0 ] && fatal bench $rc ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
      rc=$?; tail -2 "$OUT/prof.err"; [ $rc -ne 0 ] && fatal prof $rc ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
          python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
        rc=$?; tail -2 "$OUT/pmc_$c.err"; [ $rc -ne 0 ] && fatal "pmc $c" $rc
      done ;;
    swtrace:*)
      # kernel trace of tools/prof_switch.py with env overrides, e.g. swtrace:V=32,ORDER=wm,RUNS=1
      envs=${st#swtrace:}; tag=$(echo "$envs" | tr ',=' '__')
      ( export ${envs//,/ }; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/swtrace_$tag" -o run -- python3 tools/prof_switch.py > "$OUT/swtrace_$tag.log" 2>&1 )
      rc=$?; tail -2 "$OUT/swtrace_$tag.log"; [ $rc -ne 0 ] && fatal "$st" $rc ;;
    swpmc:*|pathtrace:*|pathpmc:*)
      # swpmc:K=V,..  FETCH/WRITE PMC passes of tools/prof_switch.py with env overrides;
      # pathtrace:K=V,.. / pathpmc:K=V,..  kernel trace / PMC passes of tools/prof_path.py
      kind=${st%%:*}; envs=${st#*:}; tag=$(echo "$envs" | tr ',=' '__')
      case $kind in swpmc|pathpmc) cs="FETCH_SIZE WRITE_SIZE" ;; *) cs="TRACE" ;; esac
      case $kind in swpmc) tgt=tools/prof_switch.py ;; *) tgt=tools/prof_path.py ;; esac
      for c in $cs; do
        if [ "$c" = TRACE ]; then args="--kernel-trace --stats"; else args="--pmc $c"; fi
        ( export ${envs//,/ }; timeout -k 10 300 rocprofv3 $args --output-format csv \
            -d "$OUT/${kind}_${tag}_$c" -o run -- python3 $tgt > "$OUT/${kind}_${tag}_$c.log" 2>&1 )
        rc=$?; tail -2 "$OUT/${kind}_${tag}_$c.log"; [ $rc -ne 0 ] && fatal "$st $c" $rc
      done ;;
    swsq:*)
      # swsq:K=V,..  one PMC pass of SQ issue / wait counters over tools/prof_switch.py
      envs=${st#swsq:}; tag=$(echo "$envs" | tr ',=' '__')
      ( export ${envs//,/ }; timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv \
          -d "$OUT/swsq_$tag" -o run -- python3 tools/prof_switch.py > "$OUT/swsq_$tag.log" 2>&1 )
      rc=$?; tail -2 "$OUT/swsq_$tag.log"; [ $rc -ne 0 ] && fatal "$st" $rc ;;
    swprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/swprof" -o run -- \
        python3 tools/prof_switch.py > "$OUT/swprof.log" 2>&1
      rc=$?; tail -2 "$OUT/swprof.log"; [ $rc -ne 0 ] && fatal swprof $rc
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/swpmc_$c" -o run -- \
          python3 tools/prof_switch.py > "$OUT/swpmc_$c.log" 2>&1
        rc=$?; tail -2 "$OUT/swpmc_$c.log"; [ $rc -ne 0 ] && fatal "swpmc $c" $rc
      done ;;
    pathprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pathprof" -o run -- \
        python3 tools/prof_path.py > "$OUT/pathprof.log" 2>&1
      rc=$?; tail -2 "$OUT/pathprof.log"; [ $rc -ne 0 ] && fatal pathprof $rc ;;
    config1)
      timeout -k 10 600 python examples/config1_loopback.py --epochs 3 --local-steps 5 > "$OUT/config1.log" 2>&1
      rc=$?; tail -8 "$OUT/config1.log"; [ $rc -ne 0 ] && fatal config1 $rc ;;
    rehearse)
      # bench.py starts its own two ranks (no launcher); both on the box's one GPU over gloo
      INA_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 \
        --c5-values 67108864 > "$OUT/rehearse2.json" 2> "$OUT/rehearse2.err"
      rc=$?; cat "$OUT/rehearse2.json"; tail -3 "$OUT/rehearse2.err"; [ $rc -ne 0 ] && fatal rehearse $rc ;;
    rehearse8)
      # bench.py --gpus 8 the way the driver's scale run starts it, 8 ranks on one GPU over gloo
      INA_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 10 --warmup 3 \
        --c5-values 16777216 --c5-steps 3 > "$OUT/rehearse8.json" 2> "$OUT/rehearse8.err"
      rc=$?; tail -c 600 "$OUT/rehearse8.json"; tail -3 "$OUT/rehearse8.err"; [ $rc -ne 0 ] && fatal rehearse8 $rc ;;
    sharded)
      for wire in i32 i16; do
        timeout -k 10 400 python bench.py --mode sharded --wire $wire > "$OUT/sharded1_$wire.json" 2> "$OUT/sharded1_$wire.err"
        rc=$?; cat "$OUT/sharded1_$wire.json"; tail -3 "$OUT/sharded1_$wire.err"; [ $rc -ne 0 ] && fatal sharded $rc
      done ;;
    swlab)
      timeout -k 10 400 python tools/lab/switch_sort_lab.py > "$OUT/switch_sort_lab.json" 2> "$OUT/switch_sort_lab.err"
      rc=$?; cat "$OUT/switch_sort_lab.json"; [ $rc -ne 0 ] && fatal swlab $rc ;;
    extra)
      timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extra > "$OUT/extra_bench.json" 2> "$OUT/extra.err"
      rc=$?; tail -3 "$OUT/extra.err"; [ $rc -ne 0 ] && fatal extra $rc
      cp gpurun_out/bench_extra.json "$OUT/" ;;
  esac
done
echo "session $TAG done"
