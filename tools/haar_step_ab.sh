#!/bin/bash
# Haar parity, then device time per call vs stages per tail pass (FM_HAAR_STEP; 1000 = one tail pass).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/haar7.log 2>&1 || { tail -30 gpurun_out/haar7.log; exit 1; }
tail -1 gpurun_out/haar7.log
for r in 1 2; do
for st in 1 2 4 1000; do
  FM_HAAR_STEP=$st timeout -k 10 200 python tools/bench_haar.py --cpu-frames 0 > gpurun_out/haar_step_$st.log 2>&1 || { tail -5 gpurun_out/haar_step_$st.log; exit 1; }
  tail -1 gpurun_out/haar_step_$st.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step $st', d['device_ms_per_call'], d['device_frames_per_s'], d['value'])"
done
done
