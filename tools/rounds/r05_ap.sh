#!/bin/bash
# Round 5, call ap: k_pix5's gray deal 3/2 instead of 4/1 (FM_P5_GFAST=3: three frame loads per wave, 75 VGPRs)
# and the gray stores by ds_write_addtid_b32 with the slot base in M0 (FM_P5_ADDTID=1: no per-lane address
# arithmetic) -- the parity file through both, then the driver's command A/B against the product, 4 rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
G=$PWD/abvar/g3/libfm_hip.so
A=$PWD/abvar/at/libfm_hip.so
for v in G A; do
  lib=${!v}
  FM_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05ap_$v.log 2>&1 || { tail -40 gpurun_out/parity_r05ap_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/parity_r05ap_$v.log)"
done
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4; do
  for v in P G A; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05ap"
