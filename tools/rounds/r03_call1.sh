#!/bin/bash
# Full-tile contour records and one-pass union-find labelling: parity tests, then A/B, and the
# contour-stream count A/B.
set -o pipefail
mkdir -p gpurun_out
K="full_tiles or heavy or random_masks or golden_contour or bench_shape or mode_f_1080p"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "$K" > gpurun_out/c1_parity.log 2>&1 || { tail -30 gpurun_out/c1_parity.log; exit 1; }
tail -2 gpurun_out/c1_parity.log
FM_HIP_LIB=$PWD/abvar/uf/libfm_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -k "$K" > gpurun_out/c1_parity_uf.log 2>&1 || { tail -30 gpurun_out/c1_parity_uf.log; exit 1; }
tail -2 gpurun_out/c1_parity_uf.log
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh nofull full uf || exit 1
ROUNDS="1 2 3" bash tools/r03_ccls.sh - 4 2 || exit 1
