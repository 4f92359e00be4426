#!/bin/bash
# In-place background fma / SGPR frame base (FM_PIX_FMA_INPLACE, FM_PIX_SADDR): parity of the new
# build, then A/B of k_pix5 (default bench) and k_pixw (config-5 geometry) against the round's kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_ab5.log 2>&1 || { tail -30 gpurun_out/parity_ab5.log; exit 1; }
tail -1 gpurun_out/parity_ab5.log
ROUNDS="1 2 3" bash tools/ab_steady.sh orig p10 p11 || exit 1
export ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
ROUNDS="1 2" bash tools/ab_shape.sh orig p10 p11
