#!/bin/bash
# Object-ROI stage: GPU Haar tests, then the frontalface bench + kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-haar}
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
timeout -k 10 300 python tools/bench_haar.py --frontalface --cpu-frames 0 > gpurun_out/haar_$TAG.log 2>&1 || { tail -20 gpurun_out/haar_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_$TAG.log | cut -c1-500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 tools/bench_haar.py --frontalface --cpu-frames 0 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -10
