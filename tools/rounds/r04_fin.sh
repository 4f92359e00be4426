#!/bin/bash
# Round 4, last call: the product with the input stream on every CU (mode D): the GPU suite, smoke, the
# driver's bench line and mode D.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04fin}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
for r in 1 2; do
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 --no-mjpeg --no-cpu-baseline --no-host-fed > gpurun_out/bench_${TAG}_D_$r.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_D_$r.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_D_$r.log | cut -c1-200
done
echo "done $TAG"
