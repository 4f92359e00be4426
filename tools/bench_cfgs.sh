#!/bin/bash
# Parity of the in-tree build, then the pipelined bench at batch 32/64 (1 stream) and 8 streams (config 3).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/parity_cfg.log 2>&1 || { tail -30 gpurun_out/parity_cfg.log; exit 1; }
tail -1 gpurun_out/parity_cfg.log
run() { N=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg_$N.log 2>&1 || { tail -5 gpurun_out/cfg_$N.log; exit 1; }
  tail -1 gpurun_out/cfg_$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$N', d['value'], d['roofline']['frac'], d['kernels']['pix'])"; }
run b32 --steps 40
run b64 --batch 64 --ring 64 --steps 20
run b32_again --steps 40
run b64_again --batch 64 --ring 64 --steps 20
run s8 --streams 8 --steps 10 --ring 64
run s8b16 --streams 8 --batch 16 --steps 20 --ring 64
