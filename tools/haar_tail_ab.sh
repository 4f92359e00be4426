#!/bin/bash
# Haar device time vs tail grid size (FM_HAAR_TAIL_BLOCKS), alternating, 2 rounds.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for b in 512 1024 2048 4096 8192; do
  FM_HAAR_TAIL_BLOCKS=$b timeout -k 10 200 python tools/bench_haar.py --cpu-frames 0 > gpurun_out/haar_tb_$b.log 2>&1 || { tail -5 gpurun_out/haar_tb_$b.log; exit 1; }
  tail -1 gpurun_out/haar_tb_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('blocks $b', d['device_ms_per_call'], d['device_frames_per_s'])"
done
done
