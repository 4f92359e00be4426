#!/bin/bash
# Round 4, last: mode D with the pixel stream on 2 CUs (its two 16-wave workgroups) and the input stream
# on the other 254 (px2) or on all (px2all), against the product (pixel on 8 CUs, input on all).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04px2}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
for round in 1 2 3; do
  for var in prod px2 px2all; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
echo "done $TAG"
