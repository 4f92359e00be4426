#!/bin/bash
# Steady-state A/B of contour-stream hardware-queue placement (dev build switches), alternating.
# Usage: tools/ab_qmode.sh "ENV=.. ENV=.." ...   ("-" = none)
set -o pipefail
mkdir -p gpurun_out
export FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed > gpurun_out/abq_$i.log 2>&1 || { tail -3 gpurun_out/abq_$i.log; exit 1; }
    echo "[$E] round $r $(tail -1 gpurun_out/abq_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
