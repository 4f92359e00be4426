#!/bin/bash
# A/B of library builds on the GPU box, one gpurun call:
#   [PARITY="tests/test_gpu_parity.py ..."] [REPS=4] [ARGS="..."] tools/ab_bench.sh TAG libA.so libB.so ...
# 1. if PARITY is set: the named GPU test files through every library but the first (the product);
# 2. REPS alternating rounds of the bench command (default: the driver's configs[1] line without its side legs)
#    per library: frames/s, ms per step, pixel launch average / std, roofline fraction.
# Logs under gpurun_out/ab_TAG_*; libraries are built beforehand with tools/ab_build.sh (abvar/, git-ignored).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
REPS=${REPS:-4}
ARGS=${ARGS:---steps 20 --warmup 5}
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
first=1
for lib in "$@"; do
  if [ -n "$PARITY" ] && [ $first = 0 ]; then
    n=$(basename "$(dirname "$lib")")
    FM_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest $PARITY -x -q -m gpu --timeout 300 --timeout-method thread \
      > gpurun_out/ab_${TAG}_parity_$n.log 2>&1 || { tail -40 gpurun_out/ab_${TAG}_parity_$n.log; exit 1; }
    echo "$n parity: $(tail -1 gpurun_out/ab_${TAG}_parity_$n.log)"
  fi
  first=0
done
q() { python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
for r in $(seq "$REPS"); do
  for lib in "$@"; do
    n=$(basename "$(dirname "$lib")")
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $ARGS $J > gpurun_out/ab_${TAG}_${n}_r$r.log 2>&1 \
      || { tail -20 gpurun_out/ab_${TAG}_${n}_r$r.log; exit 1; }
    echo "r$r $n $(q < gpurun_out/ab_${TAG}_${n}_r$r.log)"
  done
done
echo "done ab $TAG"
