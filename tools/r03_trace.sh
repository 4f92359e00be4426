#!/bin/bash
# Kernel trace of the driver's bench command (no PMC): tools/r03_trace.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$1 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/tr_$1.log 2>&1 || { tail -5 gpurun_out/tr_$1.log; exit 1; }
tail -1 gpurun_out/tr_$1.log | cut -c1-200
