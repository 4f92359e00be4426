#!/bin/bash
# bench.py --gpus 2 on the box's one GPU: both ranks pinned to device 0 over gloo (RCCL refuses two
# ranks on one device) -- exercises bench.py's own rank spawning and the N>1 code path.
set -o pipefail
mkdir -p gpurun_out
FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/n2.log 2>&1 || { tail -20 gpurun_out/n2.log; exit 1; }
grep '^{' gpurun_out/n2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n2', d['value'], d['n_gpus'], d['roofline']['frac'], d['cpu_baseline'])"
