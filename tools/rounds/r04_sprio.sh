#!/bin/bash
# Round 4, last: mode D with the small-image pixel waves at issue priority 3 / 1 (over the resize waves
# that share their CUs) against the product (0); parity of the priority-3 build first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04sprio}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_HIP_LIB=$PWD/abvar/sprio3/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "mode_d or resize" > gpurun_out/parity_sprio_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_sprio_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_sprio_$TAG.log
for round in 1 2 3; do
  for var in prod sprio1 sprio3; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
echo "done $TAG"
