#!/bin/bash
# Round 5, call q: batch slots per context (6 = product, 8, 10): the driver's command without side legs and mode D
# at 60 steps, 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], d.get('footprint_per_gpu', {}).get('device_bytes'))"; }
P=$PWD/find_motion_amd/libfm_hip.so
S8=$PWD/abvar/s8/libfm_hip.so
S10=$PWD/abvar/s10/libfm_hip.so
for r in 1 2 3; do
  for v in P S8 S10; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
for r in 1 2; do
  for v in P S8 S10; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D --steps 60 $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
echo "done r05q"
