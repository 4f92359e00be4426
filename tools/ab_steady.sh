#!/bin/bash
# Steady-state (default bench) A/B of abvar/<name> library variants, alternating, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2 3}; do
  for N in "$@"; do
    FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/abs_$N.log 2>&1 || { tail -3 gpurun_out/abs_$N.log; exit 1; }
    echo "$N round $r $(tail -1 gpurun_out/abs_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
