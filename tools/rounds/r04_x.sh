#!/bin/bash
# Round 4, call x: k_pix5 with 8 chain + 4 producer waves for every image size (FM_P5_SPLIT_LARGE: 768-thread
# workgroups, 6 waves per SIMD at two per CU): parity and configuration suites, then A/B x 3 on the
# driver's command and configs[2].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04x}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'])"; }
FM_HIP_LIB=$PWD/abvar/splL/libfm_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_splL_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_splL_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_splL_$TAG.log
for round in 1 2 3; do
  for var in prod splL; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_${var}_$round.log "F $var r$round"
  done
done
for var in prod splL; do
  FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_c2_${var}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c2_${var}.log; exit 1; }
  v gpurun_out/ab_${TAG}_c2_${var}.log "C2 $var"
done
FM_HIP_LIB=$PWD/abvar/pwspl/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread -k "k21 or config5" > gpurun_out/parity_pwspl_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_pwspl_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_pwspl_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2; do
  for var in prod pwspl; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J > gpurun_out/ab_${TAG}_c5_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_c5_${var}_$round.log "C5 $var r$round"
  done
done
echo "done $TAG"
