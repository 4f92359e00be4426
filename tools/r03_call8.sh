#!/bin/bash
# With the labelling gate and 4 workgroups per frame: 6 batch slots, the merge kernels gated too, 2 workgroups per frame.
set -o pipefail
mkdir -p gpurun_out
for N in sl6 mgate; do
  FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "bench_shape or heavy or golden_contour" > gpurun_out/c8_parity_$N.log 2>&1 || { tail -30 gpurun_out/c8_parity_$N.log; exit 1; }
  echo "$N $(tail -1 gpurun_out/c8_parity_$N.log)"
done
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh cur sl6 mgate gw2 || exit 1
