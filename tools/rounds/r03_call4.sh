#!/bin/bash
# One batch's labelling kernel at a time (FM_CCL_GATE): parity on the gated build, A/B, and a trace of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FM_HIP_LIB=$PWD/abvar/gate/libfm_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "bench_shape or in_flight or config3_perf or heavy or golden_contour" > gpurun_out/c4_parity_gate.log 2>&1 || { tail -30 gpurun_out/c4_parity_gate.log; exit 1; }
tail -1 gpurun_out/c4_parity_gate.log
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh cur gate || exit 1
FM_HIP_LIB=$PWD/abvar/gate/libfm_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/prof_c4.log 2>&1 || { tail -5 gpurun_out/prof_c4.log; exit 1; }
