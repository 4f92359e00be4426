#!/bin/bash
# k_tile_heavy on dynamic LDS (its VGPR allocation 264 -> 72): contour parity on the product library,
# A/B against the static-LDS build, and a kernel trace of the driver's command for the timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K="full_tiles or heavy or random_masks or golden_contour or bench_shape or mode_f_1080p or max_contours or pool or in_flight or config3 or config5 or contour_area"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "$K" > gpurun_out/c2_parity.log 2>&1 || { tail -30 gpurun_out/c2_parity.log; exit 1; }
tail -2 gpurun_out/c2_parity.log
FM_HIP_LIB=$PWD/abvar/ccl6/libfm_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/c2_parity_ccl6.log 2>&1 || { tail -30 gpurun_out/c2_parity_ccl6.log; exit 1; }
tail -2 gpurun_out/c2_parity_ccl6.log
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh heavystatic heavydyn ccl6 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/prof_c2.log 2>&1 || { tail -5 gpurun_out/prof_c2.log; exit 1; }
tail -1 gpurun_out/prof_c2.log | cut -c1-200
