#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Mode D pixel-kernel time (serial) with and without raw loads (FM_DEBUG_SKIP=4: results invalid).
for M in 0 4 12 3; do
  FM_SERIAL=1 FM_DEBUG_SKIP=$M timeout -k 10 120 python bench.py --no-cpu-baseline --mode D --steps 10 --warmup 2 > gpurun_out/mds_$M.log 2>&1 || { tail -3 gpurun_out/mds_$M.log; exit 1; }
  echo "skip=$M $(tail -1 gpurun_out/mds_$M.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])')"
done
