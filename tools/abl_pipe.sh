#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Pipelined (default-mode) bench under stage ablations (results invalid): which side bounds the steady state.
mkdir -p gpurun_out
for M in ${MASKS:-0 64 15 79}; do
  FM_DEBUG_SKIP=$M timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > gpurun_out/ablpipe_$M.log 2>&1 || { tail -3 gpurun_out/ablpipe_$M.log; exit 1; }
  tail -1 gpurun_out/ablpipe_$M.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('skip=$M', d['value'], {n: v['avg_us'] for n, v in k.items()})"
done
