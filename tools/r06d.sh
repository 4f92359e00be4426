#!/bin/bash
# Round 6, call d: the Haar stage beside k_pixw's 128-row bands -- the wave-parallel tail (product) through the Haar
# GPU tests, then configs[4] with its Haar stage: product / serial tail (ht0) / bands capped at 96 VGPRs (wpe5) /
# 64-row tiles (nob), and configs[4] without the stage for wpe5 and the product.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r06d_haar.log 2>&1 || { tail -40 gpurun_out/parity_r06d_haar.log; exit 1; }
echo "haar suite: $(tail -1 gpurun_out/parity_r06d_haar.log)"
P=$PWD/find_motion_amd/libfm_hip.so
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
q() { python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; h=d.get('haar_stage') or {}
print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], h.get('device_ms'), h.get('share_of_step_time'), h.get('detections'))"; }
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
for r in 1 2; do
  for lib in $P $PWD/abvar/ht0/libfm_hip.so $PWD/abvar/wpe5/libfm_hip.so $PWD/abvar/nob/libfm_hip.so; do
    n=$(basename $(dirname $lib))
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C4 --haar $J > gpurun_out/r06d_h_${n}_r$r.log 2>&1 || { tail -20 gpurun_out/r06d_h_${n}_r$r.log; exit 1; }
    echo "haar r$r $n $(q < gpurun_out/r06d_h_${n}_r$r.log)"
  done
done
for lib in $P $PWD/abvar/wpe5/libfm_hip.so; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C4 --masks $J > gpurun_out/r06d_m_${n}.log 2>&1 || { tail -20 gpurun_out/r06d_m_${n}.log; exit 1; }
  echo "masks $n $(q < gpurun_out/r06d_m_${n}.log)"
done
echo "done r06d"
