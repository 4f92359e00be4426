#!/bin/bash
# Round 4, call g: GPU suite on the current kernels (SDWA table offset + buffer loads in the pixel
# kernels, root masks in the tile labelling, the Haar frame list), then an A/B of the driver's command
# over v0 (neither), v1 (pixel changes only), v2 (both) in 3 alternating rounds, config 5 v0 / v2, and
# configs[4] with its Haar stage on the frame list.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04g}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --masks"
for round in 1 2 3; do
  for var in v0 v1 v2; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
for round in 1 2; do
  for B in 256 384 512; do
    FM_HIP_LIB=$PWD/abvar/v2/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch $B --ring $B $J > gpurun_out/ab_${TAG}_b${B}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_b${B}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_b${B}_$round.log "F v2 batch $B r$round"
  done
done
for round in 1 2; do
  for var in v0 v2; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py $C5 $J > gpurun_out/ab_${TAG}_c5_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_c5_${var}_$round.log "C5 $var r$round"
  done
done
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
grep '^{' gpurun_out/bench_${TAG}_c5h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5h', d['value'], d['ms_per_step'], d['haar_stage'])"
echo "done $TAG"
