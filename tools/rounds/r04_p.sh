#!/bin/bash
# Round 4, call p: Haar GPU suite (pipelined integral columns), then k_hdetect with two stump records in
# flight (pfd2) against one (prod): 64-frame frontalface call and configs[4] with its Haar stage.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04p}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/haar_parity_$TAG.log 2>&1 || { tail -40 gpurun_out/haar_parity_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_parity_$TAG.log
FM_HIP_LIB=$PWD/abvar/pfd2/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_haar.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/haar_parity_pfd2_$TAG.log 2>&1 || { tail -40 gpurun_out/haar_parity_pfd2_$TAG.log; exit 1; }
tail -1 gpurun_out/haar_parity_pfd2_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
for round in 1 2; do
  for var in prod pfd2; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python tools/bench_haar.py --frontalface --iters 10 --cpu-frames 0 > gpurun_out/hb_${TAG}_${var}_$round.log 2>&1 || { tail -20 gpurun_out/hb_${TAG}_${var}_$round.log; exit 1; }
    echo "HB $var r$round $(grep '^{' gpurun_out/hb_${TAG}_${var}_$round.log | cut -c100-240)"
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/ab_${TAG}_c5h_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_c5h_${var}_$round.log; exit 1; }
    grep '^{' gpurun_out/ab_${TAG}_c5h_${var}_$round.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['haar_stage']; print('C5H $var r$round', d['value'], d['ms_per_step'], h['device_ms'], h['wall_ms'])"
  done
done
echo "done $TAG"
