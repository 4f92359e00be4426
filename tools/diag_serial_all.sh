#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Uncontended per-kernel durations (serial mode, events around every kernel) + k_pix workgroup stamps.
set -o pipefail
mkdir -p gpurun_out
FM_SERIAL=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --all-ktimes "$@" > gpurun_out/serial_all.log 2>&1 || { tail -3 gpurun_out/serial_all.log; exit 1; }
tail -1 gpurun_out/serial_all.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('serial', d['value'], {n: (v['avg_us'], v['launches']) for n, v in k.items()})"
for MODE in pipe serial; do
  E=""; [ $MODE = serial ] && E="FM_SERIAL=1"
  env $E FM_PTS=gpurun_out/pts_$MODE.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/pts_$MODE.log 2>&1 || { tail -5 gpurun_out/pts_$MODE.log; exit 1; }
  echo "== $MODE"; python tools/pts.py gpurun_out/pts_$MODE.bin 32
done
