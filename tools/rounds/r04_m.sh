#!/bin/bash
# Round 4, call m: (1) Haar GPU suite + configs[4] with Haar on the page-locked frame table; (2) k_pix5
# issue priority falling with progress (FM_P5_QPRIO 1 / 3) against the product build, and the workgroup
# stamps of the QPRIO 3 build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04m}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/haar_parity_$TAG.log 2>&1 || { tail -40 gpurun_out/haar_parity_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_parity_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2; do
  timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h_$round.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h_$round.log; exit 1; }
  grep '^{' gpurun_out/bench_${TAG}_c5h_$round.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['haar_stage']; print('C5H r$round', d['value'], d['ms_per_step'], h['device_ms'], h['wall_ms'])"
done
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_PTS=gpurun_out/pts_${TAG}.bin FM_PTS_RING=25 FM_HIP_LIB=$PWD/abvar/ptsqp3/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_pts.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pts.log; exit 1; }
v gpurun_out/bench_${TAG}_pts.log "pts-qp3"
python tools/pts_ring.py gpurun_out/pts_${TAG}.bin 510 > gpurun_out/pts_${TAG}.txt 2>&1
head -12 gpurun_out/pts_${TAG}.txt
for round in 1 2 3; do
  for var in prod qp1 qp3; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
echo "done $TAG"
