#!/bin/bash
# Round 6, call j: k_pixw's band kernel with its job plans recomputed where used (rp, -DFM_PIXW_REPLAN=1: 99 instead
# of 119 VGPRs, so a 96-VGPR detector wave or an 80-VGPR contour wave fits beside two band workgroups) -- the
# pixel / configuration GPU tests through it, then configs[4] with its Haar stage 3 rounds and without 2 rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/find_motion_amd/libfm_hip.so; V=$PWD/abvar/rp/libfm_hip.so
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
PARITY="tests/test_gpu_parity.py tests/test_gpu_configs.py" REPS=3 ARGS="$C4 --haar" tools/ab_bench.sh rph $P $V || exit 1
REPS=2 ARGS="$C4 --masks" tools/ab_bench.sh rpm $P $V || exit 1
echo "done r06j"
