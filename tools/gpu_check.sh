#!/bin/bash
# Parity tests + bench summary on the GPU box.  Usage: tools/gpu_check.sh <tag> [bench args...]
TAG=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1
RC=$?
tail -3 gpurun_out/parity_$TAG.log
[ $RC -ne 0 ] && { grep -E "Error|assert|FAILED|error" gpurun_out/parity_$TAG.log | head -30; exit $RC; }
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', d['roofline'])
for k,v in d['kernels'].items(): print('  ', k, v)"
