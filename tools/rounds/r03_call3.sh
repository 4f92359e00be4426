#!/bin/bash
# k_tile_ccl at 80 VGPRs (6 waves per SIMD, the new default) vs 72 (7), and 4 contour streams (one per slot).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FM_HIP_LIB=$PWD/abvar/w7/libfm_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "full_tiles or heavy or random_masks or golden_contour or bench_shape" > gpurun_out/c3_parity_w7.log 2>&1 || { tail -30 gpurun_out/c3_parity_w7.log; exit 1; }
tail -1 gpurun_out/c3_parity_w7.log
ROUNDS="1 2 3 4 5" bash tools/r03_ab9.sh cur s4 w7 || exit 1
