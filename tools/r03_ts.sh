#!/bin/bash
# Contour-pass phase stamps (dev build, FM_TS): mean cycles per labelled tile between stamps.
set -o pipefail
mkdir -p gpurun_out
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/ts.log 2>&1 || { tail -5 gpurun_out/ts.log; exit 1; }
grep "phase cycles" gpurun_out/ts.log
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 FM_SERIAL=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/ts_serial.log 2>&1 || { tail -5 gpurun_out/ts_serial.log; exit 1; }
grep "phase cycles" gpurun_out/ts_serial.log
