#!/bin/bash
# Steady-state frames/s vs batch size (frames per pixel-kernel launch), 1080p k=5.
set -o pipefail
mkdir -p gpurun_out
run() { # tag args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bl_$tag.log 2>&1 || exit 1
  tail -1 gpurun_out/bl_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['steps'], d['ms_per_step'], d['roofline']['achieved'])"
}
for i in 1 2; do
run b64 
run b128 --batch 128 --ring 128 --ring-period 64 --steps 60
run b192 --batch 192 --ring 192 --ring-period 64 --steps 30
run b256 --batch 256 --ring 256 --ring-period 64 --steps 30
done
