#!/bin/bash
# Round 5, call ac: consecutive batches' resizes on two input streams (product) vs one (RS1): the resize / mode D /
# small-image / MJPEG GPU tests on the product, then mode D (60 steps) A/B 3 rounds and the headline once each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K="resize or mode_d or small or frame_contour or mjpeg or dropin or stream_group"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mjpeg_dropin.py -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/parity_r05ac.log 2>&1 || { tail -40 gpurun_out/parity_r05ac.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/parity_r05ac.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
R1=$PWD/abvar/rs1/libfm_hip.so
for r in 1 2 3; do
  for v in P R1; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D --steps 60 $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
for v in P R1; do
  lib=${!v}
  o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
  echo "F $v $o"
done
echo "done r05ac"
