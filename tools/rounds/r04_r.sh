#!/bin/bash
# Round 4, call r: k_pixw (configs[4] geometry) without buffer frame loads (global loads, SDWA kept)
# against the product build (both): buffer loads cost k_pix5 7.7 % (tools/r04_q.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04r}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_HIP_LIB=$PWD/abvar/pwnobuf/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "k21 or config5" > gpurun_out/parity_pwnobuf_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_pwnobuf_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_pwnobuf_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2 3; do
  for var in prod pwnobuf; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "C5 $var r$round"
  done
done
echo "done $TAG"
