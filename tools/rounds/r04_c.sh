#!/bin/bash
# Round 4, call c: the new GPU tests (JPEG host fallback, large-pitch fm_submit_streams) and configs[4] with
# its Haar stage after the detector's stream went to high priority.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r04c}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mjpeg_dropin.py tests/test_gpu_configs.py tests/test_gpu_haar.py -x -v -m gpu -k "unsupported or large_pitch or submit_streams or haar or cascade or config5 or frontalface" --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
grep '^{' gpurun_out/bench_${TAG}_c5h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['haar_stage'])"
