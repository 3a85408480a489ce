# A/B of the product library built with nt (INA_STORE_SC1=0) and sc1 (default) streaming
# stores: bench.py legs, alternating builds twice (the product path's libina.so is swapped)
set -u
mkdir -p gpurun_out/store_ab
L=distributed-training-ina_amd/ina_amd/libina.so
cp $L gpurun_out/store_ab/libina_keep.so
for rep in 1 2; do
  for v in nt sc1; do
    cp tools/lab/libina_$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/store_ab/bench_${v}_$rep.json 2> gpurun_out/store_ab/bench_${v}_$rep.err || { cp gpurun_out/store_ab/libina_keep.so $L; exit 1; }
  done
done
cp gpurun_out/store_ab/libina_keep.so $L
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/store_ab/bench_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    c5 = d["sharded_c5"]["roofline"]["hbm_phases"]
    print(f.split("/")[-1], "C3", d["roofline"]["avg_launch_us"], "C2", d["c2_fused"]["roofline"]["avg_launch_us"],
          "C4", d["c4_int16"]["roofline"]["avg_launch_us"], "q", c5["quantize"]["us"], "dq", c5["decode"]["us"],
          "e2e", d["e2e_pcie"]["value"], "sw", d["switch_c3"]["worker_major"]["us"], d["switch_c3"]["round_robin"]["us"],
          "parity", all([d["parity_spot_check"], d["c2_fused"]["parity_spot_check"], d["c4_int16"]["parity_spot_check"],
                         d["e2e_pcie"]["parity_spot_check"], d["sharded_c5"]["parity_spot_check"]]))
PY
