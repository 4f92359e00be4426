#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Haar parity, then device time per call vs the number of head stages (FM_HAAR_SPLIT).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/haar4.log 2>&1 || { tail -30 gpurun_out/haar4.log; exit 1; }
tail -1 gpurun_out/haar4.log
for sp in 1 2 3 4 25; do
  FM_HAAR_SPLIT=$sp timeout -k 10 200 python tools/bench_haar.py --cpu-frames 0 > gpurun_out/haar_split_$sp.log 2>&1 || { tail -5 gpurun_out/haar_split_$sp.log; exit 1; }
  tail -1 gpurun_out/haar_split_$sp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('split $sp', d['device_ms_per_call'], d['device_frames_per_s'], d['value'])"
done
