#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Each abvar/ variant: serial pixel time (modes F, D) and pipelined values (F x2, D x1).
set -o pipefail
mkdir -p gpurun_out
for D in abvar/*/; do
  N=$(basename $D); L="$N"
  for M in F D; do
    FM_HIP_LIB=$PWD/$D/libfm_hip.so FM_SERIAL=1 timeout -k 10 120 python bench.py --no-cpu-baseline --mode $M --steps 10 --warmup 2 > gpurun_out/fd_$N.log 2>&1 || { tail -3 gpurun_out/fd_$N.log; exit 1; }
    L="$L serial$M $(tail -1 gpurun_out/fd_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])')"
  done
  for M in F F D; do
    FM_HIP_LIB=$PWD/$D/libfm_hip.so timeout -k 10 120 python bench.py --no-cpu-baseline --mode $M --steps 20 --warmup 3 > gpurun_out/fd_$N.log 2>&1 || { tail -3 gpurun_out/fd_$N.log; exit 1; }
    L="$L pipe$M $(tail -1 gpurun_out/fd_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1000,1))')k"
  done
  echo "$L"
done
