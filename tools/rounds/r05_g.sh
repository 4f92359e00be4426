#!/bin/bash
# Round 5, call g: where mode D's host time goes (dev build: fm_wait blocked on the batch vs its post-pass),
# and whether more batch slots (10 vs 6) keep the input stream's resizes back to back.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'))"; }
P=$PWD/find_motion_amd/libfm_hip.so
V=$PWD/find_motion_amd/libfm_hip_dev.so
S10=$PWD/abvar/s10/libfm_hip.so
for r in 1 2; do
  for v in P V S10; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
o=$(FM_HIP_LIB=$V timeout -k 10 200 python bench.py $J | q) || exit 1
echo "F V $o"
o=$(FM_HIP_LIB=$S10 timeout -k 10 200 python bench.py $J | q) || exit 1
echo "F S10 $o"
echo "done r05g"
