#!/bin/bash
# Round 4, call f: kernel traces of the driver's command and of configs[2] (8 streams), and the Haar ROI
# call (1080p -> 300 INTER_AREA + frontalface) under rocprofv3 kernel stats + PMC passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04f}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_F -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $J > gpurun_out/tr_${TAG}_F.log 2>&1 || { tail -20 gpurun_out/tr_${TAG}_F.log; exit 1; }
grep '^{' gpurun_out/tr_${TAG}_F.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c2 -o run --output-format csv -- python3 bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/tr_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/tr_${TAG}_c2.log; exit 1; }
grep '^{' gpurun_out/tr_${TAG}_c2.log | cut -c1-200
PROG=tools/bench_haar.py tools/profile.sh ${TAG}_haar --frontalface --iters 10 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_haar > gpurun_out/pmc_${TAG}_haar.txt 2>&1
echo "done $TAG"
