#!/bin/bash
# Round 5, call af: compact tiles (one lane per run of the distinct rows, fm_ccl.hip compact_tile): the whole GPU
# suite on the product, then the driver's 20-step command A/B against the previous contour source (base), 3 rounds,
# and mode D once each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05af.log 2>&1 || { tail -40 gpurun_out/parity_r05af.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_r05af.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
B=$PWD/abvar/base/libfm_hip.so
for r in 1 2 3; do
  for v in P B; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
for v in P B; do
  lib=${!v}
  o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D --steps 60 $J | q) || exit 1
  echo "D $v $o"
done
echo "done r05af"
