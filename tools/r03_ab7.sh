#!/bin/bash
# k_regions LDS sized to the frame's tiles: parity, then A/B (driver's 20-step command) vs the static 32 KB.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_ab7.log 2>&1 || { tail -30 gpurun_out/parity_ab7.log; exit 1; }
tail -1 gpurun_out/parity_ab7.log
for r in ${ROUNDS:-1 2 3 4}; do
  for N in "$@"; do
    FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/abd_$N.log 2>&1 || { tail -3 gpurun_out/abd_$N.log; exit 1; }
    echo "$N round $r $(tail -1 gpurun_out/abd_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
