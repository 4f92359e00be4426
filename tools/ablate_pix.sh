#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Pixel-kernel stage ablations (FM_DEBUG_SKIP bits 1 gray, 2 chain, 4 raw loads, 8 raw->LDS; results invalid), serial mode.
mkdir -p gpurun_out
for M in ${MASKS:-0 1 2 3 4 8 12 13 14 15}; do
  FM_SERIAL=1 FM_DEBUG_SKIP=$M timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/ablp_$M.log 2>&1 || { tail -3 gpurun_out/ablp_$M.log; exit 1; }
  tail -1 gpurun_out/ablp_$M.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('skip=$M', 'pix', k['pix']['avg_us'])"
done
