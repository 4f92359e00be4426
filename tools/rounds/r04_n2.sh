#!/bin/bash
# Round 4, last: the multi-rank path on the final build -- 2 ranks x 8 streams on the one GPU (gloo
# barrier / max-over-ranks), and the torch.distributed.run form at 2 ranks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --streams 8 --steps 10 --warmup 3 --no-host-fed --no-mjpeg --no-cpu-baseline > gpurun_out/bench_r04n2s8.log 2>&1 || { tail -20 gpurun_out/bench_r04n2s8.log; exit 1; }
grep '^{' gpurun_out/bench_r04n2s8.log | cut -c1-220
FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-host-fed --no-mjpeg --no-cpu-baseline > gpurun_out/bench_r04n2tr.log 2>&1 || { tail -20 gpurun_out/bench_r04n2tr.log; exit 1; }
grep '^{' gpurun_out/bench_r04n2tr.log | cut -c1-220
echo done
