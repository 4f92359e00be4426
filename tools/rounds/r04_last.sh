#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_r04last.log 2>&1 || { tail -40 gpurun_out/parity_r04last.log; exit 1; }
tail -1 gpurun_out/parity_r04last.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04last.log 2>&1 || { tail -20 gpurun_out/smoke_r04last.log; exit 1; }
tail -1 gpurun_out/smoke_r04last.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r04last.log 2>&1 || { tail -20 gpurun_out/bench_r04last.log; exit 1; }
tail -1 gpurun_out/bench_r04last.log | cut -c1-160
