#!/bin/bash
# Round 5, call ab: k_hdetect with the head stages on compacted (non-flat) windows (HC): the Haar GPU tests on it,
# configs[4] with its Haar stage A/B (3 alternating rounds), the standalone frontalface call A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HC=$PWD/abvar/hc/libfm_hip.so
P=$PWD/find_motion_amd/libfm_hip.so
FM_HIP_LIB=$HC timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05ab_hc.log 2>&1 || { tail -40 gpurun_out/parity_r05ab_hc.log; exit 1; }
echo "haar tests on HC: $(tail -1 gpurun_out/parity_r05ab_hc.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
qh() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; h=d.get('haar_stage') or {}; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r['frac'], {k: h.get(k) for k in ('detections', 'device_ms', 'share_of_step_time')})"; }
for r in 1 2 3; do
  for v in P HC; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C5 $J --haar | qh) || exit 1
    echo "C5 r$r $v $o"
  done
done
for v in P HC; do
  lib=${!v}
  FM_HIP_LIB=$lib timeout -k 10 300 python tools/bench_haar.py --frontalface > gpurun_out/bench_haar_r05ab_$v.log 2>&1 || { tail -20 gpurun_out/bench_haar_r05ab_$v.log; exit 1; }
  echo "haar $v: $(tail -2 gpurun_out/bench_haar_r05ab_$v.log | tr '\n' ' ' | cut -c1-300)"
done
echo "done r05ab"
