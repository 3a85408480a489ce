set -e
mkdir -p gpurun_out
for wa in 0 16 8 4 2 1; do WIN_ACK=$wa REPS=8 timeout -k 10 100 python tools/lab/path_lab.py 2>/dev/null; done > gpurun_out/win_ack.log
for wd in 0 16 12 8; do WIN_DATA=$wd REPS=8 timeout -k 10 100 python tools/lab/path_lab.py 2>/dev/null; done > gpurun_out/win_data.log
cat gpurun_out/win_ack.log gpurun_out/win_data.log
