#!/bin/bash
# Round-4 start: the driver's bench line, mode D (-B 100, the reference's CLI default) and its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-mjpeg > gpurun_out/r04a_bench.log 2>&1 || { tail -20 gpurun_out/r04a_bench.log; exit 1; }
tail -1 gpurun_out/r04a_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 --no-mjpeg --no-host-fed --no-cpu-baseline > gpurun_out/r04a_benchD.log 2>&1 || { tail -20 gpurun_out/r04a_benchD.log; exit 1; }
tail -1 gpurun_out/r04a_benchD.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04aD -o run --output-format csv -- python3 bench.py --mode D --steps 20 --warmup 5 --no-mjpeg --no-host-fed --no-cpu-baseline > gpurun_out/r04a_profD.log 2>&1 || { tail -20 gpurun_out/r04a_profD.log; exit 1; }
find gpurun_out/prof_r04aD -name '*kernel_stats.csv' -print -quit | xargs cat | cut -c1-200
