#!/bin/bash
# Round 4, call b: the whole GPU suite (the headline's exact shape included), smoke, the driver's bench
# line, mode D, configs[2] (8 streams: device-resident and host-fed), configs[4] with its Haar stage, and
# the configs[3] per-GPU shape rehearsed at 2 ranks on the one GPU (footprints printed).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04b}
J="--no-mjpeg --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 $J --no-host-fed > gpurun_out/bench_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_D.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_D.log | cut -c1-300
for B in 128 256; do
timeout -k 10 300 python bench.py --streams 8 --batch $B --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_c2_b$B.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c2_b$B.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c2_b$B.log | cut -c1-300
done
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --no-host-fed"
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c5h.log | cut -c1-300
timeout -k 10 300 python bench.py $C5 $J --masks > gpurun_out/bench_${TAG}_c5m.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5m.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c5m.log | cut -c1-300
FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --streams 8 --steps 10 --warmup 3 --no-host-fed $J > gpurun_out/bench_${TAG}_n2s8.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_n2s8.log; exit 1; }
grep '^{' gpurun_out/bench_${TAG}_n2s8.log | cut -c1-300
echo "done $TAG"
