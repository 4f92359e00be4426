#!/bin/bash
# Round 5, call r: ten slots -- the GPU suite, the bounds-checked build on the parity / configuration / JPEG
# suites, smoke, the default command, configs[4] legs (r05_l.sh), the multi-rank rehearsal.
set -o pipefail
TAG=${1:-r05r}
mkdir -p gpurun_out
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_jpeg.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_${TAG}_checked.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_${TAG}_checked.log)"
tools/rounds/r05_l.sh $TAG || exit 1
tools/rehearse_multi.sh > gpurun_out/rehearse_$TAG.log 2>&1 || { tail -20 gpurun_out/rehearse_$TAG.log; exit 1; }
grep -E "n_gpus" gpurun_out/rehearse_$TAG.log
