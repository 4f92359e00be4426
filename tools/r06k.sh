#!/bin/bash
# Round 6, call k: k_hdetect with the head stages' stump records staged in LDS (product) vs their per-lane vector
# loads (lh0): the Haar GPU tests through the product, then tools/bench_haar.py --frontalface and configs[4] with its
# Haar stage, alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/find_motion_amd/libfm_hip.so; V=$PWD/abvar/lh0/libfm_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r06k_haar.log 2>&1 || { tail -40 gpurun_out/parity_r06k_haar.log; exit 1; }
echo "haar suite (product): $(tail -1 gpurun_out/parity_r06k_haar.log)"
for r in 1 2; do
  for lib in $P $V; do
    n=$(basename $(dirname $lib))
    FM_HIP_LIB=$lib timeout -k 10 300 python tools/bench_haar.py --frontalface --iters 10 > gpurun_out/r06k_bh_${n}_r$r.log 2>&1 || { tail -10 gpurun_out/r06k_bh_${n}_r$r.log; exit 1; }
    echo "bench_haar r$r $n: $(grep '^{' gpurun_out/r06k_bh_${n}_r$r.log | tail -1 | cut -c1-300)"
  done
done
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
REPS=3 ARGS="$C4 --haar" tools/ab_bench.sh lhh $P $V || exit 1
echo "done r06k"
