#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Pipelined bench under contour-pass ablations / stream counts (skip results invalid): what bounds the steady state.
mkdir -p gpurun_out
run() { N=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ap_$N.log 2>&1 || { tail -3 gpurun_out/ap_$N.log; exit 1; }
  tail -1 gpurun_out/ap_$N.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('$N', d['value'], {n: v['avg_us'] for n, v in k.items()})"; }
run base FM_X=0
run skip64 FM_DEBUG_SKIP=64
run skip192 FM_DEBUG_SKIP=192
run ccl1 FM_CCL_STREAMS=1
run ccl3 FM_CCL_STREAMS=3
run ccl4 FM_CCL_STREAMS=4
run prio_off FM_PIX_PRIO_OFF=1
