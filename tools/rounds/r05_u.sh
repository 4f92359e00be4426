#!/bin/bash
# Round 5, call u: the mode D bench-shape parity test; kernel traces + PMC passes of the headline and mode D on
# the round's final build (ten slots, three contour streams).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k "mode_d_bench_shape or slot_reuse" --timeout 300 --timeout-method thread > gpurun_out/parity_r05u.log 2>&1 || { tail -40 gpurun_out/parity_r05u.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/parity_r05u.log)"
tools/profile.sh r05u_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05u_F > gpurun_out/pmc_r05u_F.txt 2>&1
tools/profile.sh r05u_D --mode D --steps 60 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05u_D > gpurun_out/pmc_r05u_D.txt 2>&1
echo "done r05u"
