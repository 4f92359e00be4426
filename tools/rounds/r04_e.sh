#!/bin/bash
# Round 4, call e: the whole GPU suite on k_resolve + the 2-D tile order, A/B of each against the
# build without it (driver's command; configs[4] geometry), configs[4] with Haar, contour phase stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04e}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; k=d['kernels']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --masks"
for round in 1 2; do
  for var in new resolve0 order0; do
    L=$PWD/find_motion_amd/libfm_hip.so; [ $var != new ] && L=$PWD/abvar/$var/libfm_hip.so
    FM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
  for var in new tall0 order0; do
    L=$PWD/find_motion_amd/libfm_hip.so; [ $var != new ] && L=$PWD/abvar/$var/libfm_hip.so
    FM_HIP_LIB=$L timeout -k 10 200 python bench.py $C5 $J > gpurun_out/ab_${TAG}_c5_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_c5_${var}_$round.log "C5 $var r$round"
  done
done
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_D.log; exit 1; }
v gpurun_out/bench_${TAG}_D.log "D bands"
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
grep '^{' gpurun_out/bench_${TAG}_c5h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5h', d['value'], d['ms_per_step'], d['haar_stage'])"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 FM_SERIAL=1 timeout -k 10 200 python bench.py --steps 6 --warmup 2 $J > gpurun_out/ts_ser_$TAG.log 2>&1 || { tail -20 gpurun_out/ts_ser_$TAG.log; exit 1; }
grep "phase cycles" gpurun_out/ts_ser_$TAG.log
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so FM_TS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ts_pipe_$TAG.log 2>&1 || { tail -20 gpurun_out/ts_pipe_$TAG.log; exit 1; }
grep "phase cycles" gpurun_out/ts_pipe_$TAG.log
echo "done $TAG"
