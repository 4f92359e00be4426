#!/bin/bash
# Round 6, call h: how much the contour pass costs the pixel kernel -- the dev build pipelined vs FM_SERIAL (the
# contour pass on the pixel stream: each pixel launch runs alone), configs[1] and configs[4] geometry, 2 rounds;
# frames/s, the pixel launch average (stamps) and the contour chain's kernels (HIP events, --all-ktimes off).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
D=$PWD/find_motion_amd/libfm_hip_dev.so
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --masks"
q() { python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'))"; }
for r in 1 2; do
  for mode in pipe serial; do
    e=""; [ $mode = serial ] && e="FM_SERIAL=1"
    env $e FM_HIP_LIB=$D timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/r06h_F_${mode}_r$r.log 2>&1 || { tail -5 gpurun_out/r06h_F_${mode}_r$r.log; exit 1; }
    echo "F r$r $mode $(q < gpurun_out/r06h_F_${mode}_r$r.log)"
    env $e FM_HIP_LIB=$D timeout -k 10 300 python bench.py $C4 $J > gpurun_out/r06h_c4_${mode}_r$r.log 2>&1 || { tail -5 gpurun_out/r06h_c4_${mode}_r$r.log; exit 1; }
    echo "c4 r$r $mode $(q < gpurun_out/r06h_c4_${mode}_r$r.log)"
  done
done
echo "done r06h"
