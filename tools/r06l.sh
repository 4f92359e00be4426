#!/bin/bash
# Round 6, call l: configs[2] (8 x 1080p on one GPU) at 256 frames per stream per step vs 128, alternating, 3 rounds
# (60 steps each, the same 256-frame device ring); TS="64 96 128" picks the sizes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
q() { python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
for r in 1 2 3; do
  for T in ${TS:-128 256}; do
    timeout -k 10 300 python bench.py --streams 8 --batch $T --steps 60 --warmup 5 $J > gpurun_out/r06l_T${T}_r$r.log 2>&1 || { tail -10 gpurun_out/r06l_T${T}_r$r.log; exit 1; }
    echo "r$r T$T $(q < gpurun_out/r06l_T${T}_r$r.log)"
  done
done
echo "done r06l"
