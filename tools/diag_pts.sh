#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# k_pix workgroup timing (FM_PTS) pipelined and serial, plus batch-size sweep.  Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
for MODE in pipe serial; do
  E=""; [ $MODE = serial ] && E="FM_SERIAL=1"
  env $E FM_PTS=gpurun_out/pts_$MODE.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/pts_$MODE.log 2>&1 || { tail -5 gpurun_out/pts_$MODE.log; exit 1; }
  echo "== $MODE"; python tools/pts.py gpurun_out/pts_$MODE.bin 32
done
for B in 16 64; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --batch $B --ring $((B*2)) > gpurun_out/batch_$B.log 2>&1 || { tail -5 gpurun_out/batch_$B.log; exit 1; }
  tail -1 gpurun_out/batch_$B.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('batch $B', d['value'], d['kernels']['pix'])"
done
