#!/bin/bash
# Round 4, call t: mode D at 8 hardware queues: kernel trace of the product (pixel stream on 8 CUs), and
# A/B of 16 pixel CUs (sp16) and 16 CUs + 8/16-row bands (sp16b).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04t}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'], 'hwq', d.get('hw_queues_per_process'))"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_D -o run --output-format csv -- python3 bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/tr_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/tr_${TAG}_D.log; exit 1; }
v gpurun_out/tr_${TAG}_D.log "D traced"
FM_HIP_LIB=$PWD/abvar/sp16b/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "mode_d or resize" > gpurun_out/parity_sp16b_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_sp16b_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_sp16b_$TAG.log
for round in 1 2; do
  for var in prod sp16 sp16b; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
echo "done $TAG"
