#!/bin/bash
# Round 6, call i: non-temporal frame loads -- the mode D resize (rsnt) and k_pix5 (p5nt) -- against the product,
# alternating: mode D (60 steps) 3 rounds, configs[1] 3 rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/find_motion_amd/libfm_hip.so
REPS=3 ARGS="--mode D --steps 60 --warmup 5" tools/ab_bench.sh rsnt $P $PWD/abvar/rsnt/libfm_hip.so || exit 1
REPS=3 tools/ab_bench.sh p5nt $P $PWD/abvar/p5nt/libfm_hip.so || exit 1
echo "done r06i"
