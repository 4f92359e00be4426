#!/bin/bash
# GPU box: the whole GPU parity suite against the bounds-checked library (make VARIANT=checked):
# any out-of-range index in the contour pass fails fm_wait with its FM_OOB codes.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu \
  --timeout 300 --timeout-method thread > gpurun_out/parity_checked.log 2>&1
rc=$?; tail -5 gpurun_out/parity_checked.log; exit $rc
