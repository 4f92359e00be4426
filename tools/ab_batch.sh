#!/bin/bash
# Steady-state bench at several batch sizes, alternating, 2 rounds: tools/ab_batch.sh 192 256 ...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for B in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --no-mjpeg --batch $B --ring $B > gpurun_out/abb_$B.log 2>&1 || { tail -3 gpurun_out/abb_$B.log; exit 1; }
    echo "batch $B round $r $(tail -1 gpurun_out/abb_$B.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
