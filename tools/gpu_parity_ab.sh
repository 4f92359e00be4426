#!/bin/bash
# GPU parity of the in-tree build, then the abvar/ A/B (serial stamps + pipelined bench).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_ab.log 2>&1 || { tail -30 gpurun_out/parity_ab.log; exit 1; }
tail -2 gpurun_out/parity_ab.log
bash tools/ab_pts.sh "$@"
