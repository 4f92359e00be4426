#!/bin/bash
# Round 5, call z: kernel trace + PMC passes of configs[4] with its Haar stage on face frames (the detector's
# kernels beside k_pixw: instruction counts and waits).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/profile.sh r05z_c5h --width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 4 --haar || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05z_c5h > gpurun_out/pmc_r05z_c5h.txt 2>&1
echo "done r05z"
