#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Pipelined and serial bench at several batch sizes (frames per stream per launch).
set -o pipefail
mkdir -p gpurun_out
for B in ${BATCHES:-32 64 128}; do
  for MODE in pipe serial; do
    E=""; [ $MODE = serial ] && E="FM_SERIAL=1"
    env $E timeout -k 10 120 python bench.py --no-cpu-baseline --batch $B --ring $((B*2)) --steps $((640/B)) --warmup 2 "$@" > gpurun_out/bb_${MODE}_$B.log 2>&1 || { tail -5 gpurun_out/bb_${MODE}_$B.log; exit 1; }
    tail -1 gpurun_out/bb_${MODE}_$B.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('batch $B $MODE', d['value'], d['kernels']['pix'])"
  done
done
