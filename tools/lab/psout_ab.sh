#!/bin/bash
# The fused PS output's store policy in its real context: bench.py's packet_path leg (the
# steady-state INA step) with the product library swapped between two builds, alternated
# A, B, A, B on one box (tools/lab/libina_po0.so: default stores, libina_po2.so: nt).
set -u
mkdir -p gpurun_out/psout
L=distributed-training-ina_amd/ina_amd/libina.so
cp $L gpurun_out/psout/keep.so
for run in 1 2; do
  for v in po0 po2; do
    cp tools/lab/libina_$v.so $L
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c2 --no-c4 --no-e2e --no-c5 \
      > gpurun_out/psout/${v}_$run.json 2> gpurun_out/psout/${v}_$run.err || { cp gpurun_out/psout/keep.so $L; exit 1; }
  done
done
cp gpurun_out/psout/keep.so $L
python - <<'PY'
import json
for run in (1, 2):
    for v in ("po0", "po2"):
        d = json.loads(open(f"gpurun_out/psout/{v}_{run}.json").read().strip().splitlines()[-1])
        pp, sw = d["packet_path"], d["switch_c3"]
        print(f"{v} run {run}: packet_path {pp['ms_per_step']:.3f} ms (frac {pp['roofline']['frac']}), "
              f"switch wm {sw['worker_major']['us']} us, rr {sw['round_robin']['us']} us")
PY
