#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_md.log 2>&1 || { tail -30 gpurun_out/parity_md.log; exit 1; }
tail -1 gpurun_out/parity_md.log
bash tools/bench_other.sh
