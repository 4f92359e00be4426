#!/bin/bash
# Round 5, call at: max-memory-clause scheduling for fm_pix.hip (M) against the product's default (P): the
# driver's command 6 alternating rounds, configs[4]'s geometry (k_pixw) 2 rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
M=$PWD/abvar/smc/libfm_hip.so
P=$PWD/find_motion_amd/libfm_hip.so
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
for r in 1 2 3 4 5 6; do
  for v in P M; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
for r in 1 2; do
  for v in P M; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C5 $J | q) || exit 1
    echo "C5 r$r $v $o"
  done
done
echo "done r05at"
