#!/bin/bash
# Round 4, call w: k_pix5 with chain and producer waves (FM_P5_SPLIT, small work images): the parity and
# configuration suites on it, then mode D A/B against the product build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04w}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'], 'hwq', d.get('hw_queues_per_process'))"; }
FM_HIP_LIB=$PWD/abvar/spl/libfm_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_spl_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_spl_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_spl_$TAG.log
for round in 1 2 3; do
  for var in prod spl; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
echo "done $TAG"
