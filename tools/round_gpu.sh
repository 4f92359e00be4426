#!/bin/bash
# One GPU-box pass: parity tests, default bench line, rocprofv3 kernel stats + HBM PMC passes.
# Usage: tools/round_gpu.sh <tag> [bench args...]   (logs under gpurun_out/)
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -3 gpurun_out/parity_$TAG.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
tools/profile.sh $TAG "$@" || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG > gpurun_out/pmc_$TAG.txt 2>&1
cat gpurun_out/pmc_$TAG.txt
python tools/traffic.py gpurun_out/prof_$TAG gpurun_out/bench_$TAG.log $TAG > /dev/null || echo "traffic extraction failed"
