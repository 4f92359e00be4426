#!/bin/bash
# GPU MJPEG decoder: per-kernel times (rocprofv3) and a chunk-length / speculation-length sweep.
# Usage (on the GPU box): tools/jpeg_sweep.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/jpeg_sweep}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/bench_mjpeg.py 192 75 > "$OUT/prof.log" 2>&1 || exit 1
for cfg in "512 256" "1024 256" "1024 512" "2048 512" "2048 1024" "4096 1024"; do
    set -- $cfg
    echo "CB=$1 OV=$2 $(FM_JPEG_CB=$1 FM_JPEG_OV=$2 timeout -k 10 120 python3 tools/bench_mjpeg.py 192 75 2>/dev/null | tail -1)" >> "$OUT/sweep.log" || exit 1
done
