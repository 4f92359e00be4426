#!/bin/bash
# Round 5, call y: k_frame_contours with batch sizes that change on a slot (the slot-wide words re-armed at the
# new indices): the frame-contour, small-image and drop-in GPU tests on the product and the bounds-checked build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K="frame_contour or small or mode_d or dropin or stream_group or video_motion"
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_mjpeg_dropin.py -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/parity_r05y.log 2>&1 || { tail -40 gpurun_out/parity_r05y.log; exit 1; }
echo "product: $(tail -1 gpurun_out/parity_r05y.log)"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/parity_r05y_checked.log 2>&1 || { tail -40 gpurun_out/parity_r05y_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_r05y_checked.log)"
echo "done r05y"
