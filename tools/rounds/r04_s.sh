#!/bin/bash
# NOTE (round 5): this archived A/B predates bench.py reading FM_BENCH_HW_QUEUES; bench.py now overwrites
# GPU_MAX_HW_QUEUES, so re-running it as written measures 8 queues in both arms (use FM_BENCH_HW_QUEUES=$q).
# Round 4, call s: hardware queues per process (the box exports GPU_MAX_HW_QUEUES=4, which bench.py's
# use_hw_queues() left in place): mode D, the driver's command and the MJPEG-fed leg at 4 vs 8, alternating;
# first the parity suite and mode D with the pixel / input streams on disjoint CUs (FM_CU_SPLIT) vs shared.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04s}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
v() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'us', r['avg_launch_us'], 'hwq', d.get('hw_queues_per_process'), 'mjpeg', (d.get('mjpeg_fed_per_gpu') or {}).get('frames_per_s'))"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_split_$TAG.log 2>&1 || { tail -30 gpurun_out/parity_split_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_split_$TAG.log
for round in 1 2; do
  for var in prod nosplit; do
    FM_HIP_LIB=$PWD/abvar/$var/libfm_hip.so timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_${var}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_${var}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_${var}_$round.log "D $var r$round"
  done
done
for round in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --mode D --steps 20 --warmup 5 $J > gpurun_out/ab_${TAG}_D_q${q}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_D_q${q}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_D_q${q}_$round.log "D q$q r$round"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed > gpurun_out/ab_${TAG}_F_q${q}_$round.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_F_q${q}_$round.log; exit 1; }
    v gpurun_out/ab_${TAG}_F_q${q}_$round.log "F q$q r$round"
  done
done
echo "done $TAG"
