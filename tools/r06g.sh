#!/bin/bash
# Round 6, call g: k_pixw's horizontal taps as i8 MFMAs (hm, -DFM_PIXW_HMMA=1): the i8 MFMA lane-map probe first,
# then the pixel / configuration GPU tests through the variant, then configs[4] geometry and configs[4] with Haar.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 tools/ubench/mfma_i8_layout > gpurun_out/r06g_probe.log 2>&1; rc=$?
cat gpurun_out/r06g_probe.log
[ $rc -eq 0 ] || exit 1
P=$PWD/find_motion_amd/libfm_hip.so; V=$PWD/abvar/hm/libfm_hip.so
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
PARITY="tests/test_gpu_parity.py tests/test_gpu_configs.py" REPS=3 ARGS="$C4 --masks" tools/ab_bench.sh hm $P $V || exit 1
REPS=1 ARGS="$C4 --haar" tools/ab_bench.sh hmh $P $V || exit 1
echo "done r06g"
