#!/bin/bash
# Round 5, call k: k_small_scan storing its column words once per 64 frames (SBLK) vs per frame (P):
# small-path parity on SBLK, mode D 3 alternating rounds; configs[4] with Haar, the detector stream at high (P)
# or normal (H) priority, 2 rounds; mode D kernel trace + PMC passes (product).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05k}
FM_HIP_LIB=$PWD/abvar/sblk/libfm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "small or mode_d or selection or frame_contour" --timeout 300 --timeout-method thread > gpurun_out/parity_${TAG}_sblk.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_sblk.log; exit 1; }
echo "sblk: $(tail -1 gpurun_out/parity_${TAG}_sblk.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'))"; }
P=$PWD/find_motion_amd/libfm_hip.so
B=$PWD/abvar/sblk/libfm_hip.so
for r in 1 2 3; do
  for v in P B; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
qh() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; h=d.get('haar_stage') or {}; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r['frac'], {k: h.get(k) for k in ('calls', 'roi_frames', 'detections', 'wall_ms', 'device_ms', 'share_of_step_time')})"; }
H=$PWD/abvar/hlo/libfm_hip.so
for r in 1 2; do
  for v in P H; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C5 $J --haar | qh) || exit 1
    echo "C5 r$r $v $o"
  done
done
tools/profile.sh ${TAG}_D --mode D --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_D > gpurun_out/pmc_${TAG}_D.txt 2>&1
echo "done $TAG"
