#!/bin/bash
# Round 3 close: the whole GPU suite, smoke, the default bench line (the driver's command), then the
# same command under rocprofv3 (kernel stats + PMC passes) for profiles/.
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -3 gpurun_out/parity_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
tools/profile.sh $TAG --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG > gpurun_out/pmc_$TAG.txt 2>&1
echo "final $TAG done"
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
timeout -k 10 300 python bench.py $C5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/bench_${TAG}_c5.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}_c5.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c5.log | cut -c1-300
