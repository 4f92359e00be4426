#!/bin/bash
# Config 5 geometry (4K, -b 183 -> k 21): one and four streams per GPU.
set -o pipefail
mkdir -p gpurun_out
run() { N=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --width 3840 --height 2160 --blur-scale 183 "$@" > gpurun_out/b4k_$N.log 2>&1 || { tail -5 gpurun_out/b4k_$N.log; exit 1; }
  tail -1 gpurun_out/b4k_$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$N', d['value'], r['frac'], r['avg_launch_us'])"; }
run s1b32 --batch 32 --ring 32 --steps 10
run s1b64 --batch 64 --ring 64 --steps 8
run s4b16 --streams 4 --batch 16 --ring 16 --steps 8
