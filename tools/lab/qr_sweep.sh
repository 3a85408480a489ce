set -e
for sb in 256 512 1024 8192; do
  echo "## STREAM_BLOCKS=$sb"
  STREAM_BLOCKS=$sb ROUNDS=6 ONLY=qreduce_C2 timeout -k 10 120 python tools/lab/ew_lab.py ./tools/lab/libina_q1.so ./tools/lab/libina_q2.so ./tools/lab/libina_q4.so 2>/dev/null
done
