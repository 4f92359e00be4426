#!/bin/bash
# Round 4: the driver's command at 256 (default) vs 512 frames per step, 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04t512}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
for round in 1 2 3; do
  for B in 256 512; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch $B --ring $B $J > gpurun_out/ab_${TAG}_b${B}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_b${B}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_b${B}_$round.log "F b$B r$round"
  done
done
echo "done $TAG"
