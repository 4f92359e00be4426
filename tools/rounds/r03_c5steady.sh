#!/bin/bash
# Config 5's geometry (4 x 3840x2160, k 21, 64 frames per launch) at 20 timed steps after 10 warm-up steps, 3 runs.
set -o pipefail
mkdir -p gpurun_out
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/c5s.log 2>&1 || { tail -5 gpurun_out/c5s.log; exit 1; }
  tail -1 gpurun_out/c5s.log > gpurun_out/c5s_$r.json
  echo "run $r $(python3 -c 'import json; d=json.load(open("gpurun_out/c5s_'$r'.json")); r=d["roofline"]; print(d["value"], r["avg_launch_us"], r["frac"])')"
done
