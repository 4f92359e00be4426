#!/bin/bash
# Round evidence for the decode side: bench.py line (with mjpeg_fed_per_gpu), the MJPEG bench tool and
# a rocprofv3 kernel summary of it.  Usage: tools/mjpeg_round.sh [tag]
set -o pipefail
TAG=${1:-r02_mjpeg}
OUT=gpurun_out/$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_mjpeg.py 192 75 > "$OUT/bench_mjpeg.log" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 tools/bench_mjpeg.py 192 75 > "$OUT/prof.log" 2>&1 || exit 1
