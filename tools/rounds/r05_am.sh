#!/bin/bash
# Round 5, call am: k_pix5 frame loads as buffer loads through a per-frame descriptor (FM_P5_BUFLOAD=1: no per-lane 64-bit address add per load)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/abvar/bl/libfm_hip.so
FM_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05am.log 2>&1 || { tail -40 gpurun_out/parity_r05am.log; exit 1; }
echo "bufload parity: $(tail -1 gpurun_out/parity_r05am.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4; do
  for v in P V; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05am"
