#!/bin/bash
# k_pixw at 6 waves per EU (<= 80 VGPRs, 3 workgroups per CU): k = 21 parity, then config 5's geometry A/B.
set -o pipefail
mkdir -p gpurun_out
FM_HIP_LIB=$PWD/abvar/W6/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "k21 or config5 or wide" > gpurun_out/parity_ab11.log 2>&1 || { tail -30 gpurun_out/parity_ab11.log; exit 1; }
tail -1 gpurun_out/parity_ab11.log
export ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
ROUNDS="1 2 3" bash tools/ab_shape.sh W4 W6
