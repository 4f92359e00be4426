#!/bin/bash
# bench.py at several batch sizes (frames per stream per step).  Usage: tools/bench_batches.sh <tag> [extra args]
TAG=${1:-b}; shift
mkdir -p gpurun_out
for B in ${BS:-16 32 64}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --batch $B --ring $((B * 2 > 32 ? B * 2 : 32)) "$@" > gpurun_out/bench_${TAG}_$B.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}_$B.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$B.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('batch $B value', d['value'], 'ms/step', d['ms_per_step'], {n: v['avg_us'] for n, v in k.items()})"
done
