#!/bin/bash
# Round 5, call ag: compact tiles -- the new compact-tile parity test on the product and the bounds-checked build,
# the checked build on the parity / configuration files, then kernel trace + PMC passes of the headline (the
# contour kernels' instructions per batch against r05x).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "compact or simple or full_tiles" --timeout 200 --timeout-method thread > gpurun_out/parity_r05ag.log 2>&1 || { tail -40 gpurun_out/parity_r05ag.log; exit 1; }
echo "compact: $(tail -1 gpurun_out/parity_r05ag.log)"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_r05ag_checked.log 2>&1 || { tail -40 gpurun_out/parity_r05ag_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_r05ag_checked.log)"
tools/profile.sh r05ag_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05ag_F > gpurun_out/pmc_r05ag_F.txt 2>&1
echo "done r05ag"
