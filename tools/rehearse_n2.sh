#!/bin/bash
# Two bench ranks on the box's one GPU over gloo: exercises the N>1 code path of bench.py.
set -o pipefail
mkdir -p gpurun_out
FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/n2.log 2>&1 || { tail -20 gpurun_out/n2.log; exit 1; }
grep '^{' gpurun_out/n2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n2', d['value'], d['n_gpus'], d['roofline']['frac'], d['cpu_baseline'])"
