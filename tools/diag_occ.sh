#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# k_pix workgroup durations vs workgroups per CU (serial mode).  Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
for G in "1024 1024" "2048 1024" "2048 1536" "1920 1080"; do
  set -- $G
  FM_SERIAL=1 FM_PTS=gpurun_out/occ_$1x$2.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --width $1 --height $2 > gpurun_out/occ_$1x$2.log 2>&1 || { tail -5 gpurun_out/occ_$1x$2.log; exit 1; }
  echo "== $1x$2 pix_us $(tail -1 gpurun_out/occ_$1x$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])')"
  python tools/pts.py gpurun_out/occ_$1x$2.bin 32
done
