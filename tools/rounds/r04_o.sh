#!/bin/bash
# Round 4, call o: kernel traces of configs[4] with its Haar stage (the Haar kernels beside k_pixw) and
# of the 64-frame frontalface call, + PMC passes of the latter (k_hdetect on stump records).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04o}
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --haar"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c5h -o run --output-format csv -- python3 bench.py $C5 --no-mjpeg --no-cpu-baseline --no-host-fed > gpurun_out/tr_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/tr_${TAG}_c5h.log; exit 1; }
grep '^{' gpurun_out/tr_${TAG}_c5h.log | cut -c1-200
PROG=tools/bench_haar.py tools/profile.sh ${TAG}_haar --frontalface --iters 10 --cpu-frames 0 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_haar > gpurun_out/pmc_${TAG}_haar.txt 2>&1
head -12 gpurun_out/prof_${TAG}_haar/trace/run_kernel_stats.csv | cut -c1-160
echo "done $TAG"
