#!/bin/bash
# Decode side: IDCT + colour launched in frame groups (planes kept in the Infinity Cache), A/B.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    FM_HIP_LIB=$PWD/abvar/$v/libfm_hip.so timeout -k 10 300 python3 tools/bench_mjpeg.py 192 75 > gpurun_out/jc_$v.log 2>&1 || { tail -5 gpurun_out/jc_$v.log; exit 1; }
    echo "$v round $r $(tail -1 gpurun_out/jc_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); x=d["no_restart"]; print(x["decoder_device_ms"], x["decoder_device_fps"], x["end_to_end_fps"])')"
  done
done
