#!/bin/bash
# Round 4, last: kernel trace + PMC passes of mode D on the final build (resize and split pixel kernel).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/profile.sh r04fin_D --mode D --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r04fin_D > gpurun_out/pmc_r04fin_D.txt 2>&1
head -6 gpurun_out/prof_r04fin_D/trace/run_kernel_stats.csv | cut -c1-160
grep '^{' gpurun_out/prof_r04fin_D/trace.log | cut -c1-200
echo "done"
