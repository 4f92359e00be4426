#!/bin/bash
# JPEG GPU tests + decoder kernel profile + default MJPEG bench line.  Usage: tools/jpeg_quick.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/jpeg_quick}
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_jpeg.py tests/test_gpu_mjpeg_dropin.py > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/bench_mjpeg.py 192 75 > "$OUT/prof.log" 2>&1 || exit 1
