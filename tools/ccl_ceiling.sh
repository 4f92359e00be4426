#!/bin/bash
# Ceiling estimate: steady-state bench (dev build) with contour-pass stages skipped (results invalid).
export FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so
mkdir -p gpurun_out
for r in 1 2; do
for M in 0 64 192; do
  FM_DEBUG_SKIP=$M timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/ceil_$M.log 2>&1 || { tail -3 gpurun_out/ceil_$M.log; exit 1; }
  echo "skip=$M $(tail -1 gpurun_out/ceil_$M.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
done
done
