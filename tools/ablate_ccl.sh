#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Contour-pass ablations (FM_DEBUG_SKIP bits >= 64; results invalid), serial mode.
mkdir -p gpurun_out
for M in 0 64 128 192 256; do
  FM_SERIAL=1 FM_DEBUG_SKIP=$M timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/abl_$M.log 2>&1 || { tail -3 gpurun_out/abl_$M.log; exit 1; }
  tail -1 gpurun_out/abl_$M.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('skip=$M', {n: v['avg_us'] for n, v in k.items()})"
done
