#!/bin/bash
# The default bench line N times (steady state), value and pixel-kernel event average per run.
# Usage: tools/bench_n.sh N [bench args...]
set -o pipefail
mkdir -p gpurun_out
N=${1:-3}; shift
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed "$@" > gpurun_out/bn_$i.log 2>&1 || { tail -3 gpurun_out/bn_$i.log; exit 1; }
  echo "run $i $(tail -1 gpurun_out/bn_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"], d["contour_pass"])')"
done
