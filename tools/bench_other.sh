#!/bin/bash
# The other workloads: mode D (reference default box 100), 4K k=21 (config 5 geometry), 8 streams (config 3).
set -o pipefail
mkdir -p gpurun_out
run() { N=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --all-ktimes "$@" > gpurun_out/oth_$N.log 2>&1 || { tail -5 gpurun_out/oth_$N.log; exit 1; }
  tail -1 gpurun_out/oth_$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print('$N', d['value'], r.get('kernel'), r.get('frac'), {k: v['avg_us'] for k, v in d['kernels'].items()})"; }
run modeD --mode D --steps 20
run modeD_s8 --mode D --streams 8 --steps 20
run 4k_k21 --width 3840 --height 2160 --blur-scale 183 --batch 16 --ring 32 --steps 10
