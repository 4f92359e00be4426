#!/bin/bash
# Each abvar/ variant: mode F and mode D pipelined bench values, plus the mode-D parity subset.
set -o pipefail
mkdir -p gpurun_out
for D in abvar/*/; do
  N=$(basename $D)
  FM_HIP_LIB=$PWD/$D/libfm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abm_par_$N.log 2>&1 || { echo "$N parity FAILED"; tail -15 gpurun_out/abm_par_$N.log; continue; }
  echo "$N parity $(tail -1 gpurun_out/abm_par_$N.log)"
  for M in F D; do
    FM_HIP_LIB=$PWD/$D/libfm_hip.so timeout -k 10 120 python bench.py --no-cpu-baseline --mode $M --steps 20 --warmup 3 > gpurun_out/abm_$N_$M.log 2>&1 || { tail -3 gpurun_out/abm_$N_$M.log; exit 1; }
    echo "$N mode $M $(tail -1 gpurun_out/abm_$N_$M.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels"]["pix"]["avg_us"])')"
  done
done
