#!/bin/bash
# Batch 64 vs 128 over the same 64-frame synthetic cycle.
set -o pipefail
mkdir -p gpurun_out
for B in 64 128 64 128; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --batch $B --ring $B --ring-period 64 --steps $((1280/B)) --warmup 2 > gpurun_out/b128_$B.log 2>&1 || { tail -5 gpurun_out/b128_$B.log; exit 1; }
  tail -1 gpurun_out/b128_$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $B', d['value'], d['roofline']['frac'], d['kernels']['pix'])"
done
