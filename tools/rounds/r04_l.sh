#!/bin/bash
# Round 4, call l: k_pix5 on tile pairs (FM_P5_PAIR: two 64 x 64 tiles per 1,024-thread workgroup, one
# shared frame barrier): the pixel parity and configuration suites on it, its workgroup stamps, and an
# A/B against the product build (driver's command x 3, configs[2]).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04l}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
FM_HIP_LIB=$PWD/abvar/pair/libfm_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_pair_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_pair_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_pair_$TAG.log
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_PTS=gpurun_out/pts_${TAG}.bin FM_PTS_RING=25 FM_HIP_LIB=$PWD/abvar/ptspair/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_pts.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_pts.log; exit 1; }
v gpurun_out/bench_${TAG}_pts.log "pts-pair"
python tools/pts_ring.py gpurun_out/pts_${TAG}.bin 510 > gpurun_out/pts_${TAG}.txt 2>&1
head -12 gpurun_out/pts_${TAG}.txt
for round in 1 2 3; do
  for var in prod pair; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
for var in prod pair; do
  FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_c2_${var}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c2_${var}.log; exit 1; }
  v gpurun_out/ab_${TAG}_c2_${var}.log "C2 $var"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/haar_parity_$TAG.log 2>&1 || { tail -40 gpurun_out/haar_parity_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_parity_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2; do
  for var in prod hwalk; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python tools/bench_haar.py --frontalface --iters 10 --cpu-frames 0 > gpurun_out/hb_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/hb_${TAG}_${var}_$round.log; exit 1; }
    echo "HB $var r$round $(grep '^{' gpurun_out/hb_${TAG}_${var}_$round.log | cut -c100-260)"
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/ab_${TAG}_c5h_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5h_${var}_$round.log; exit 1; }
    grep '^{' gpurun_out/ab_${TAG}_c5h_${var}_$round.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['haar_stage']; print('C5H $var r$round', d['value'], d['ms_per_step'], h['device_ms'], h['wall_ms'], h['share_of_step_time'])"
  done
done
FM_HAAR_TIMES=1 FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so timeout -k 10 200 python tools/bench_haar.py --frontalface --iters 10 --cpu-frames 0 > gpurun_out/hb_${TAG}_times.log 2>&1 || { tail -20 gpurun_out/hb_${TAG}_times.log; exit 1; }
grep "fm_haar\]" gpurun_out/hb_${TAG}_times.log
FM_HAAR_TIMES=1 FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/ab_${TAG}_c5h_times.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5h_times.log; exit 1; }
grep "fm_haar\]" gpurun_out/ab_${TAG}_c5h_times.log
echo "done $TAG"
