#!/bin/bash
# Round 5, call c: mode D on the small-image path (k_small_blur + k_small_scan, fm_small.hip) -- the GPU
# suite on that library, alternating A/B rounds of mode D against the round-4 path (k_pix5 SPL on 8 CUs),
# and a kernel trace of mode D on it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05c}
SM=$PWD/abvar/small/libfm_hip.so
P=$PWD/find_motion_amd/libfm_hip.so
FM_HIP_LIB=$SM timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
J="--mode D --no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()})"; }
for r in 1 2 3; do
  for lib in $P $SM; do
    v=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "r$r $(basename $(dirname $lib)) $v"
  done
done
FM_HIP_LIB=$SM timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $J > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log | cut -c1-200
echo "done $TAG"
