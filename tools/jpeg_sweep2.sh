#!/bin/bash
# Decoder-only chunk/speculation sweep (bench_mjpeg's decoder_device_ms).  Usage: tools/jpeg_sweep2.sh "CB OV" ...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  set -- $cfg
  r=$(FM_JPEG_CB=$1 FM_JPEG_OV=$2 timeout -k 10 120 python3 tools/bench_mjpeg.py 192 75 2>/dev/null | tail -1) || exit 1
  echo "CB=$1 OV=$2 $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["no_restart"]["decoder_device_ms"], d["restart_per_mcu_row"]["decoder_device_ms"])')"
done
