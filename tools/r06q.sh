#!/bin/bash
# Round 6, call q: k_fold / k_emit with lane = list entry (FM_CCL_DENSE) against the previous product (abvar/r06q_base).
# The pixel / configuration GPU tests through the new product and the bounds-checked build, configs[1] 4 alternating
# rounds, configs[2] 2, and one kernel trace of configs[1] per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/abvar/r06q_base/libfm_hip.so; P=$PWD/find_motion_amd/libfm_hip.so
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06q_checked.log 2>&1 || { tail -30 gpurun_out/r06q_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/r06q_checked.log)"
PARITY="tests/test_gpu_parity.py tests/test_gpu_configs.py" REPS=4 tools/ab_bench.sh r06q $B $P || exit 1
REPS=2 ARGS="--streams 8 --batch 128 --steps 20 --warmup 5" tools/ab_bench.sh r06qc2 $B $P || exit 1
for lib in $B $P; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r06q_trace_$n -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg --no-side \
    > gpurun_out/r06q_trace_$n.log 2>&1 || { tail -5 gpurun_out/r06q_trace_$n.log; exit 1; }
done
echo "done r06q"
