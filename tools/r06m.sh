#!/bin/bash
# Round 6, call m: configs[1] by frames per step (the driver's 20-step command otherwise), alternating, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
q() { python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
for r in 1 2 3; do
  for T in ${TS:-256 320 384}; do
    timeout -k 10 300 python bench.py --batch $T --ring $T --steps 20 --warmup 5 $J > gpurun_out/r06m_T${T}_r$r.log 2>&1 || { tail -10 gpurun_out/r06m_T${T}_r$r.log; exit 1; }
    echo "r$r T$T $(q < gpurun_out/r06m_T${T}_r$r.log)"
  done
done
echo "done r06m"
