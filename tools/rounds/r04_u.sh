#!/bin/bash
# Round 4, call u: mode D, the input stream's CU share: all but the pixel stream's 8 (prod), 3/4 (rs8),
# 1/2 (rs16) -- less resize bandwidth pressure on the latency-bound pixel kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04u}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'], 'hwq', d.get('hw_queues_per_process'))"; }
for round in 1 2 3; do
  for var in prod rs8 rs16; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
echo "done $TAG"
