#!/bin/bash
# Round 3, first GPU pass: the whole GPU suite, the default bench line, then the configs[4]-geometry
# bench line + its rocprofv3 kernel stats and PMC passes (k_pix<21>).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_r03a.log 2>&1 || { tail -40 gpurun_out/parity_r03a.log; exit 1; }
tail -3 gpurun_out/parity_r03a.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03a.log 2>&1 || { tail -20 gpurun_out/bench_r03a.log; exit 1; }
tail -1 gpurun_out/bench_r03a.log | cut -c1-400
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
timeout -k 10 200 python bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bench_r03_c5.log 2>&1 || { tail -20 gpurun_out/bench_r03_c5.log; exit 1; }
tail -1 gpurun_out/bench_r03_c5.log | cut -c1-400
tools/profile.sh r03_c5 $C5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r03_c5 > gpurun_out/pmc_r03_c5.txt 2>&1
cat gpurun_out/pmc_r03_c5.txt | head -30
