#!/bin/bash
# Round 4, call j: (1) k_pix5 workgroup stamps of 25 consecutive launches (dev build, no phase stamps):
# are the long launches late-dispatched or slow-running workgroups?  (2) A/B of k_pix5 at 6 waves per
# SIMD (78 VGPRs: three workgroups fit a CU) against the product build, headline and configs[2].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04j}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_PTS=gpurun_out/pts_${TAG}.bin FM_PTS_RING=25 FM_HIP_LIB=$PWD/abvar/pts/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_pts.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pts.log; exit 1; }
v gpurun_out/bench_${TAG}_pts.log "pts"
python tools/pts_ring.py gpurun_out/pts_${TAG}.bin 510 > gpurun_out/pts_${TAG}.txt 2>&1
cat gpurun_out/pts_${TAG}.txt
for round in 1 2 3; do
  for var in prod w6; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
for round in 1 2; do
  for var in prod w6; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_c2_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c2_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_c2_${var}_$round.log "C2 $var r$round"
  done
done
echo "done $TAG"
