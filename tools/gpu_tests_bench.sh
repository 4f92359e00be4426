#!/bin/bash
# GPU box: parity tests (all, or the given -k expression) then the default bench line.
# Usage: tools/gpu_tests_bench.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-run}; K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/parity_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/parity_$TAG.log | tail -30
[ $rc -ne 0 ] && { tail -60 gpurun_out/parity_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
