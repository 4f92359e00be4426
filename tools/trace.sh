#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of the default bench (plus extra bench args); prints the top kernels.
# Usage: tools/trace.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=$PWD/gpurun_out/trace_$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-fed "$@" > "$OUT/log" 2>&1 || { tail -20 "$OUT/log"; exit 1; }
tail -1 "$OUT/log" | cut -c1-300
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -14
