#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Contour-stream count x pixel-stream priority sweep of the default bench.
for P in "" "FM_PIX_PRIO_OFF=1"; do
for N in ${NS:-2 3 4}; do
    env $P FM_CCL_STREAMS=$N timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/q.log 2>&1 || { tail -3 gpurun_out/q.log; exit 1; }
    echo "$P ccl_streams=$N $(tail -1 gpurun_out/q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
done
done
