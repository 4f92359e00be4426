#!/bin/bash
# Round 6, call e: gray row stride 24 dwords in k_pix5 / k_pixw (gs24: the tap jobs' rows in disjoint LDS banks)
# -- the pixel / configuration GPU tests through it, configs[1] 4 alternating rounds, configs[4] geometry 2, and one
# LDS-counter pass of configs[1] per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/find_motion_amd/libfm_hip.so; V=$PWD/abvar/gs24/libfm_hip.so
PARITY="tests/test_gpu_parity.py tests/test_gpu_configs.py" REPS=4 tools/ab_bench.sh gs24 $P $V || exit 1
REPS=2 ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --masks" tools/ab_bench.sh gs24c4 $P $V || exit 1
for lib in $P $V; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/pmc_gs24_$n -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-fed --no-mjpeg --no-side > gpurun_out/pmc_gs24_$n.log 2>&1 || { tail -5 gpurun_out/pmc_gs24_$n.log; exit 1; }
done
echo "done r06e"
