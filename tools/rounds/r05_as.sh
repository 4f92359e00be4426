#!/bin/bash
# Round 5, call as: the pixel kernels built with other LLVM machine-scheduler strategies (fm_pix.hip only):
# iterative-ilp (I: 87 VGPRs, 55 waits in k_pix5 vs 78) and max-memory-clause (M: 81 VGPRs) -- the parity file
# through each, then the driver's command A/B against the product (default scheduler), 4 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
I=$PWD/abvar/sil/libfm_hip.so
M=$PWD/abvar/smc/libfm_hip.so
for v in I M; do
  lib=${!v}
  FM_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05as_$v.log 2>&1 || { tail -40 gpurun_out/parity_r05as_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/parity_r05as_$v.log)"
done
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4; do
  for v in P I M; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05as"
