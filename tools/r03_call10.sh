#!/bin/bash
# Batch size at the driver's 20 steps with the round-3 scheduling (gate, 6 slots): 192 (default) vs 256 vs 320.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for T in 192 256 320; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --batch $T --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bt_$T.log 2>&1 || { tail -3 gpurun_out/bt_$T.log; exit 1; }
    echo "T $T round $r $(tail -1 gpurun_out/bt_$T.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["ms_per_step"])')"
  done
done
