#!/bin/bash
# Kernel timeline of the default bench (rocprofv3 kernel trace) -> gaps between pixel kernels.
TAG=${1:-tl}; shift
OUT=$PWD/gpurun_out/tl_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
python3 tools/timeline.py "$OUT"
