#!/bin/bash
# Labelling gate on (default now): contour workgroups per frame 8 (default) vs 4 vs 6.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "bench_shape or in_flight or config3_perf or config5_perf or heavy or golden_contour or full_tiles or max_contours or pool" > gpurun_out/c5_parity.log 2>&1 || { tail -30 gpurun_out/c5_parity.log; exit 1; }
tail -1 gpurun_out/c5_parity.log
FM_HIP_LIB=$PWD/abvar/gw4/libfm_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "bench_shape or heavy or golden_contour" > gpurun_out/c5_parity_gw4.log 2>&1 || { tail -30 gpurun_out/c5_parity_gw4.log; exit 1; }
tail -1 gpurun_out/c5_parity_gw4.log
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh cur gw4 gw6 s4 || exit 1
