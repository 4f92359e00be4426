#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Pixel-kernel stage ablations (FM_DEBUG_SKIP bits 1 gray, 2 chain, 4 raw loads, 8 raw->LDS, 16 barrier; results
# invalid), serial mode, with workgroup-duration percentiles from FM_PTS stamps.
mkdir -p gpurun_out
for M in ${MASKS:-0 4 12 1 2 3 16 15}; do
  FM_SERIAL=1 FM_DEBUG_SKIP=$M FM_PTS=gpurun_out/ablpts_$M.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/ablp_$M.log 2>&1 || { tail -3 gpurun_out/ablp_$M.log; exit 1; }
  echo "skip=$M pix $(tail -1 gpurun_out/ablp_$M.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])') $(python tools/pts.py gpurun_out/ablpts_$M.bin 32 | grep '^dur')"
done
