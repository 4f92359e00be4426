#!/bin/bash
# Round 5, call ae: how much of the headline the tile labelling costs (dev build ablations, results invalid):
# FM_DEBUG_SKIP 0 (dev build, as the product), 256 (tiles neither full nor simple take the empty-tile record),
# 512 (every tile that is not full does), 3 alternating rounds of the driver's 20-step command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
D=$PWD/find_motion_amd/libfm_hip_dev.so
for r in 1 2 3; do
  for v in 0 256 512; do
    o=$(FM_HIP_LIB=$D FM_DEBUG_SKIP=$v timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r skip$v $o"
  done
done
echo "done r05ae"
