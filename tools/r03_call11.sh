#!/bin/bash
# Round close at the 256-frame bench batch (r03l): suite, smoke, bench, rocprof stats + PMC (traffic entry for
# the new workload string), config 5; then 192 vs 256 once more.
set -o pipefail
bash tools/r03_final.sh r03l || exit 1
for r in 1 2; do
  for T in 192 256; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --batch $T --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bt_$T.log 2>&1 || { tail -3 gpurun_out/bt_$T.log; exit 1; }
    echo "T $T round $r $(tail -1 gpurun_out/bt_$T.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["ms_per_step"])')"
  done
done
