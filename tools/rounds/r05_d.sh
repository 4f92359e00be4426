#!/bin/bash
# Round 5, call d (call a ran k_fused everywhere: fm_create tested the work-plane size before setting it):
# the GPU suite on the product (k_pix5), on k_pixq and on the small-image path; A/B of the driver's command
# (k_pix5 / k_pixq / k_pixq PF 2) and of mode D (k_pix5 SPL / small path); the default bench line; a kernel
# trace of k_pixq.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05d}
P=$PWD/find_motion_amd/libfm_hip.so
Q=$PWD/abvar/pixq/libfm_hip.so
Q2=$PWD/abvar/pixq2/libfm_hip.so
SM=$PWD/abvar/small/libfm_hip.so
for v in P Q SM; do
  lib=${!v}
  FM_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_${TAG}_$v.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_$v.log; exit 1; }
  echo "suite $v: $(tail -1 gpurun_out/parity_${TAG}_$v.log)"
done
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], r['launch_le_step'], sorted(k))"; }
for r in 1 2 3; do
  for v in P Q Q2; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
for r in 1 2; do
  for v in P SM; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
FM_HIP_LIB=$Q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_q -o run --output-format csv -- python3 bench.py $J > gpurun_out/prof_${TAG}_q.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_q.log; exit 1; }
echo "done $TAG"
