#!/bin/bash
# Round 5, call x: kernel trace + PMC passes of the headline with simple tiles (the contour kernels' new share).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/profile.sh r05x_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05x_F > gpurun_out/pmc_r05x_F.txt 2>&1
echo "done r05x"
