#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# In-tree build: GPU parity, contour phase stamps (serial), serial per-kernel times, pipelined bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_cur.log 2>&1 || { tail -30 gpurun_out/parity_cur.log; exit 1; }
tail -1 gpurun_out/parity_cur.log
FM_SERIAL=1 FM_TS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ts_cur.log 2>&1 || { tail -5 gpurun_out/ts_cur.log; exit 1; }
grep "phase cycles" gpurun_out/ts_cur.log
bash tools/diag_serial_all.sh | head -1
for i in 1 2; do timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench_cur.log 2>&1 || { tail -5 gpurun_out/bench_cur.log; exit 1; }
tail -1 gpurun_out/bench_cur.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pipelined', d['value'], d['kernels']['pix'])"; done
