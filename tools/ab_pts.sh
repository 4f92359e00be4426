#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Each abvar/ variant: serial pixel-kernel time + workgroup stamp summary, then the pipelined bench value.
set -o pipefail
mkdir -p gpurun_out
for D in abvar/*/; do
  N=$(basename $D)
  FM_HIP_LIB=$PWD/$D/libfm_hip.so FM_SERIAL=1 FM_PTS=gpurun_out/pts_$N.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/ab_$N.log 2>&1 || { tail -3 gpurun_out/ab_$N.log; exit 1; }
  FM_HIP_LIB=$PWD/$D/libfm_hip.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > gpurun_out/abp_$N.log 2>&1 || { tail -3 gpurun_out/abp_$N.log; exit 1; }
  echo "== $N serial_pix $(tail -1 gpurun_out/ab_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])') pipelined $(tail -1 gpurun_out/abp_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels"]["pix"]["avg_us"])')"
  python tools/pts.py gpurun_out/pts_$N.bin 32 | sed -n 2,5p
done
