#!/bin/bash
# A store-policy change in its real context: bench.py's switch_c3 and packet_path legs (back-
# to-back switch calls; the steady-state INA step) with the product library swapped between
# two builds tools/lab/libina_$A.so and libina_$B.so, alternated A, B, A, B on one box
# (first use: A=po0 default PS-output stores, B=po2 nt).
set -u
mkdir -p gpurun_out/psout
L=distributed-training-ina_amd/ina_amd/libina.so
cp $L gpurun_out/psout/keep.so
for run in 1 2; do
  for v in ${A:-po0} ${B:-po2}; do
    cp tools/lab/libina_$v.so $L
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c2 --no-c4 --no-e2e --no-c5 \
      > gpurun_out/psout/${v}_$run.json 2> gpurun_out/psout/${v}_$run.err || { cp gpurun_out/psout/keep.so $L; exit 1; }
  done
done
cp gpurun_out/psout/keep.so $L
python - <<'PY'
import json
import os
for run in (1, 2):
    for v in (os.environ.get("A", "po0"), os.environ.get("B", "po2")):
        d = json.loads(open(f"gpurun_out/psout/{v}_{run}.json").read().strip().splitlines()[-1])
        pp, sw = d["packet_path"], d["switch_c3"]
        print(f"{v} run {run}: packet_path {pp['ms_per_step']:.3f} ms (frac {pp['roofline']['frac']}), "
              f"switch wm {sw['worker_major']['us']} us, rr {sw['round_robin']['us']} us")
PY
