#!/bin/bash
# Round 4, call k: (1) Haar GPU suite on the stump-record k_hdetect (product build), (2) Haar A/B:
# round-3 sweep (prod) vs scalar leaves (hleaf) vs stump records (hrec), 1080p -> 300 frontalface call
# and configs[4] with its Haar stage, (3) k_pix5 workgroup stamps over 25 launches, (4) k_pix5 at 6
# waves per SIMD (w6) vs prod, headline and configs[2].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04k}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/haar_parity_$TAG.log 2>&1 || { tail -40 gpurun_out/haar_parity_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_parity_$TAG.log
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'], (d.get('haar_stage') or {}).get('device_ms'))"; }
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2; do
  for var in prod hleaf hrec; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python tools/bench_haar.py --frontalface --iters 10 > gpurun_out/hb_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/hb_${TAG}_${var}_$round.log; exit 1; }
    echo "HB $var r$round $(grep '^{' gpurun_out/hb_${TAG}_${var}_$round.log | cut -c1-220)"
  done
  for var in prod hrec; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/ab_${TAG}_c5h_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5h_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_c5h_${var}_$round.log "C5H $var r$round"
  done
done
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
for var in prod w6; do
  FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_c2_${var}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c2_${var}.log; exit 1; }
  v gpurun_out/ab_${TAG}_c2_${var}.log "C2 $var"
done
echo "done $TAG"
