#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
for B in 8 16 64; do
  for M in 0 15 14 13; do
    FM_SERIAL=1 FM_DEBUG_SKIP=$M timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --batch $B > gpurun_out/ablq.log 2>&1 || { tail -3 gpurun_out/ablq.log; exit 1; }
    tail -1 gpurun_out/ablq.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('batch=$B skip=$M', 'pix', k['pix']['avg_us'])"
  done
done
