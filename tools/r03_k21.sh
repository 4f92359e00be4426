#!/bin/bash
# k = 21 (k_pixw): parity at every k = 21 test, then the configs[4]-geometry bench line and its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-k21}
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread -k "k21 or config5 or large_k or ties" > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -3 gpurun_out/parity_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
timeout -k 10 200 python bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
python -c "import json;d=json.loads(open('gpurun_out/bench_$TAG.log').read().splitlines()[-1]);print(d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/prof_$TAG.log 2>&1 || exit 1
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -8
