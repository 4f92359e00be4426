#!/bin/bash
# gray by byte-split dot4 (FM_GRAY_DOT4): parity of the new build, then A/B on the default bench and config 5's geometry.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_ab10.log 2>&1 || { tail -30 gpurun_out/parity_ab10.log; exit 1; }
tail -1 gpurun_out/parity_ab10.log
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh G0 G1 || exit 1
export ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
ROUNDS="1 2 3" bash tools/ab_shape.sh G0 G1
