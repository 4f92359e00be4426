#!/bin/bash
# Haar A/B: abvar/<name> library variants on the frontalface bench, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for k in "$@"; do
    FM_HIP_LIB=$PWD/abvar/$k/libfm_hip.so timeout -k 10 120 python tools/bench_haar.py --frontalface --frames 64 --iters 10 --cpu-frames 0 > gpurun_out/hab_$k.log 2>&1 || { tail -3 gpurun_out/hab_$k.log; exit 1; }
    echo "$k round $r $(grep '^{' gpurun_out/hab_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["device_ms_per_call"], d["resident_frames_per_s"])')"
  done
done
