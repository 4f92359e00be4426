#!/bin/bash
# Round 5, call au: k_pix5's partial last round of tap jobs on wave 4 instead of wave 0 (FM_P5_TAPLAST4=1: wave 0
# also carries four gray slots, so it set every frame's barrier) -- the parity file through it, then the
# driver's command A/B against the product, 5 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/abvar/t4/libfm_hip.so
FM_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "not jpeg" --timeout 300 --timeout-method thread > gpurun_out/parity_r05au.log 2>&1 || { tail -40 gpurun_out/parity_r05au.log; exit 1; }
echo "taplast4 parity: $(tail -1 gpurun_out/parity_r05au.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4 5; do
  for v in P V; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05au"
