#!/bin/bash
# Decode side: GPU JPEG tests, then the MJPEG decoder bench and its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-jpeg}
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_mjpeg_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
timeout -k 10 300 python tools/bench_mjpeg.py 192 75 > gpurun_out/mjpeg_$TAG.log 2>&1 || { tail -20 gpurun_out/mjpeg_$TAG.log; exit 1; }
tail -3 gpurun_out/mjpeg_$TAG.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 tools/bench_mjpeg.py 192 75 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -8
