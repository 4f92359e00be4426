#!/bin/bash
# k_pix5 stage ablations, serial (dev build; FM_DEBUG_SKIP bits 1 gray, 2 chain, 4 loads, 8 taps; results invalid)
set -o pipefail
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so} FM_SERIAL=1  # (k_pix5 runtime skips need a -DFM_DEV_SKIP build)
for sk in ${SKIPS:-0 1 2 4 8 5 13 15}; do
  FM_DEBUG_SKIP=$sk timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --steps 30 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skip $sk', d['roofline']['avg_launch_us'])" || exit 1
done
