#!/bin/bash
# Round 5, call ak: k_pix5 with the SDWA table offset, v_perm row pairs and no keep-mask copies without masks (the
# product now): the whole GPU suite; then the driver's command A/B against two frame bodies per iteration
# (FM_P5_UNROLL2=1: immediate LDS offsets), 4 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05ak.log 2>&1 || { tail -40 gpurun_out/parity_r05ak.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_r05ak.log)"
U=$PWD/abvar/u2/libfm_hip.so
FM_HIP_LIB=$U timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05ak_u2.log 2>&1 || { tail -40 gpurun_out/parity_r05ak_u2.log; exit 1; }
echo "u2 parity: $(tail -1 gpurun_out/parity_r05ak_u2.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4; do
  for v in P U; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05ak"
