#!/bin/bash
# Round 4, call q: k_pix5 with the SDWA table offset alone (static LDS table) and with buffer frame loads
# alone, against the product build (the round's combined A/B measured both together at -3.4 %).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04q}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_HIP_LIB=$PWD/abvar/sdwa/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "bench_shape or k5 or threshold or tail or mask" > gpurun_out/parity_sdwa_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_sdwa_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_sdwa_$TAG.log
for round in 1 2 3; do
  for var in prod sdwa bufld; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
echo "done $TAG"
