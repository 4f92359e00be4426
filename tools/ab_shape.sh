#!/bin/bash
# A/B of abvar/<name> library variants on one bench shape, alternating rounds.
# Usage: ARGS="--width 3840 ..." tools/ab_shape.sh name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2 3}; do
  for N in "$@"; do
    FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/abs_$N.log 2>&1 || { tail -3 gpurun_out/abs_$N.log; exit 1; }
    echo "$N round $r $(tail -1 gpurun_out/abs_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])')"
  done
done
