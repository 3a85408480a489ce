#!/bin/bash
# PMC passes over switch_lab.py for each given variant (experiment only).
# usage: tools/lab/switch_pmc.sh OUTDIR variant.so...
set -u
OUT=$1; shift
export TMPDIR=/tmp
cd "$(dirname "$0")"
mkdir -p "../../$OUT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for v in "$@"; do
  n=$(basename "$v" .so)
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "../../$OUT/${n}_p$i" -o run -- \
      python3 switch_lab.py "$v" > "../../$OUT/${n}_p$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $n p$i rc=$rc"; tail -5 "../../$OUT/${n}_p$i.log"; exit $rc; fi
  done
done
echo pmc done
