#!/bin/bash
# configs[4] geometry: rocprofv3 kernel stats + PMC passes (tools/profile.sh), summary and traffic entry.
set -o pipefail
TAG=${1:-r03_c5w}
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
timeout -k 10 200 python bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
tools/profile.sh $TAG $C5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG > gpurun_out/pmc_$TAG.txt 2>&1
grep -A20 "k_pixw<21, false, false>" gpurun_out/pmc_$TAG.txt | head -21
