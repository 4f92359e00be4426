#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# bench.py under a few engine modes (stderr summaries).  Usage: tools/bench_modes.sh <tag>
TAG=${1:-modes}
mkdir -p gpurun_out
for MODE in "" "FM_SERIAL=1"; do
  env $MODE timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_${TAG}_${MODE:-default}.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}_${MODE:-default}.log; exit 1; }
  echo "== ${MODE:-default}"
  tail -1 gpurun_out/bench_${TAG}_${MODE:-default}.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms/step', d['ms_per_step'])
for k,v in d['kernels'].items(): print('  ', k, v)"
done
