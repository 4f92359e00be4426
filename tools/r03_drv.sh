#!/bin/bash
# The driver's bench command, N times on one box (headline spread).
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${1:-3}); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/drv.log 2>&1 || { tail -5 gpurun_out/drv.log; exit 1; }
  echo "run $r: $(tail -1 gpurun_out/drv.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])')"
done
