#!/bin/bash
# Round 4, call d: r04_c (new GPU tests, configs[4] with Haar at high priority), then the contour pass's
# per-phase cycles per labelled tile (dev build, FM_TS) serial and pipelined, and a kernel trace of the
# driver's command for the timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04d}
tools/r04_c.sh $TAG || exit 1
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 FM_SERIAL=1 timeout -k 10 200 python bench.py --steps 6 --warmup 2 $J > gpurun_out/ts_ser_$TAG.log 2>&1 || { tail -20 gpurun_out/ts_ser_$TAG.log; exit 1; }
grep "phase cycles" gpurun_out/ts_ser_$TAG.log
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ts_pipe_$TAG.log 2>&1 || { tail -20 gpurun_out/ts_pipe_$TAG.log; exit 1; }
grep "phase cycles" gpurun_out/ts_pipe_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_tr -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $J > gpurun_out/tr_$TAG.log 2>&1 || { tail -20 gpurun_out/tr_$TAG.log; exit 1; }
grep '^{' gpurun_out/tr_$TAG.log | cut -c1-200
echo "done $TAG"
