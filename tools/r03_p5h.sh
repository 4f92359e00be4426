#!/bin/bash
# k_pix5h: k = 5 parity (the default library), then A/B against k_pix5 on the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_p5h.log 2>&1 || { tail -30 gpurun_out/parity_p5h.log; exit 1; }
tail -2 gpurun_out/parity_p5h.log
ROUNDS="1 2 3" tools/ab_steady.sh p5full p5h
