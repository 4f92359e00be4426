#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Serial-mode (one stream) bench: uncontended per-kernel durations.
mkdir -p gpurun_out
FM_SERIAL=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > gpurun_out/serial.log 2>&1 || { tail -3 gpurun_out/serial.log; exit 1; }
tail -1 gpurun_out/serial.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('serial', d['value'], {n: v['avg_us'] for n, v in k.items()})"
