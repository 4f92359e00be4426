#!/bin/bash
# Object-ROI stage on the GPU box: bench line + rocprofv3 kernel stats of the same command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_haar.py "$@" > gpurun_out/haar_bench.log 2>&1 || { tail -20 gpurun_out/haar_bench.log; exit 1; }
tail -1 gpurun_out/haar_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_haar -o run --output-format csv -- python3 tools/bench_haar.py --cpu-frames 0 "$@" > gpurun_out/haar_prof.log 2>&1 || { tail -20 gpurun_out/haar_prof.log; exit 1; }
find gpurun_out/prof_haar -name "*kernel_stats.csv" -exec cp {} gpurun_out/haar_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/haar_kernel_stats.csv | head -12
