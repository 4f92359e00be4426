#!/bin/bash
# FM_* developer switches are honoured only by the dev build: make -C find_motion_amd/csrc VARIANT=dev
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
# Parity tests, then serial pixel-kernel workgroup timing and the default pipelined bench line.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
FM_SERIAL=1 FM_PTS=gpurun_out/pts_$TAG.bin timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ser_$TAG.log 2>&1 || { tail -5 gpurun_out/ser_$TAG.log; exit 1; }
echo "serial pix_us $(tail -1 gpurun_out/ser_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["pix"]["avg_us"])')"
python tools/pts.py gpurun_out/pts_$TAG.bin 32
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], 'frac', d['roofline']['frac'], d['kernels'])"
