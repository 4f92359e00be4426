#!/bin/bash
# Round 4, call n: issue priorities.  cp3: every contour kernel at priority 3; q2cp3 / q3cp3: + k_pix5's
# priority falling with progress from 2 / 3 (the younger workgroup of a CU catches up; contour waves are
# never below it, so they cannot be starved into holding CU slots).  Workgroup stamps of q2cp3; A/B x 3
# on the driver's command; configs[4] geometry for prod / cp3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04n}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_PTS=gpurun_out/pts_${TAG}.bin FM_PTS_RING=25 FM_HIP_LIB=$PWD/abvar/ptsq2cp3/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_pts.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pts.log; exit 1; }
v gpurun_out/bench_${TAG}_pts.log "pts-q2cp3"
python tools/pts_ring.py gpurun_out/pts_${TAG}.bin 510 > gpurun_out/pts_${TAG}.txt 2>&1
cat gpurun_out/pts_${TAG}.txt
for round in 1 2 3; do
  for var in prod cp3 q2cp3 q3cp3; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for var in prod cp3; do
  FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J > gpurun_out/ab_${TAG}_c5_${var}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5_${var}.log; exit 1; }
  v gpurun_out/ab_${TAG}_c5_${var}.log "C5 $var"
done
echo "done $TAG"
