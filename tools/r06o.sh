#!/bin/bash
# Round 6, call o: the small-image kernels' LDS bank conflicts (verdict r05 item 3) -- k_small_blur's H at an odd
# row stride, k_small_scan's blur * alpha on the VALU instead of the LDS table. The pixel / configuration GPU
# tests through the new product library, mode D 3 alternating rounds against the previous product (abvar/r06o_base),
# then per library one kernel-trace run and one LDS-counter pass of mode D.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/abvar/r06o_base/libfm_hip.so; P=$PWD/find_motion_amd/libfm_hip.so
PARITY="tests/test_gpu_parity.py tests/test_gpu_configs.py" REPS=3 ARGS="--mode D --steps 60 --warmup 10" \
  tools/ab_bench.sh r06o $B $P || exit 1
for lib in $B $P; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o_trace_$n -o run --output-format csv \
    -- python3 bench.py --mode D --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg --no-side \
    > gpurun_out/r06o_trace_$n.log 2>&1 || { tail -5 gpurun_out/r06o_trace_$n.log; exit 1; }
  FM_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU \
    -d gpurun_out/r06o_pmc_$n -o run --output-format csv \
    -- python3 bench.py --mode D --steps 10 --warmup 3 --no-cpu-baseline --no-host-fed --no-mjpeg --no-side \
    > gpurun_out/r06o_pmc_$n.log 2>&1 || { tail -5 gpurun_out/r06o_pmc_$n.log; exit 1; }
done
echo "done r06o"
