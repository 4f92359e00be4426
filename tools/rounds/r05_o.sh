#!/bin/bash
# Round 5, call o: contour streams 2 vs 3 (dev build FM_CCL_STREAMS) on mode D (60 steps, as the side leg) and on
# the driver's command, alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], {n: v['avg_us'] for n, v in k.items() if v['launches']})"; }
V=$PWD/find_motion_amd/libfm_hip_dev.so
for r in 1 2 3; do
  for n in 2 3; do
    o=$(FM_CCL_STREAMS=$n FM_HIP_LIB=$V timeout -k 10 200 python bench.py --mode D --steps 60 $J | q) || exit 1
    echo "D r$r cs$n $o"
  done
done
for r in 1 2 3; do
  for n in 2 3; do
    o=$(FM_CCL_STREAMS=$n FM_HIP_LIB=$V timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r cs$n $o"
  done
done
echo "done r05o"
