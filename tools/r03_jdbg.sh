#!/bin/bash
# GPU JPEG parity per library variant (abvar/<name>), one pytest run each.
set -o pipefail
mkdir -p gpurun_out
for v in base "$@"; do
  if [ "$v" != base ]; then export FM_HIP_LIB=$PWD/abvar/$v/libfm_hip.so; else unset FM_HIP_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -q --timeout 120 --timeout-method thread > gpurun_out/jd_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/jd_$v.log)"
done
