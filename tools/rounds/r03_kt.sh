#!/bin/bash
# Does the pixel kernel's HIP-event timing cost throughput?  default vs --no-ktimes, alternated.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "" "--no-ktimes"; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg $v > gpurun_out/kt.log 2>&1 || { tail -5 gpurun_out/kt.log; exit 1; }
    echo "[$v] $(tail -1 gpurun_out/kt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
