#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP's default, vs 8): headline and MJPEG-fed figures, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed > gpurun_out/hwq_$q.log 2>&1 || { tail -5 gpurun_out/hwq_$q.log; exit 1; }
    echo "hwq $q round $r $(tail -1 gpurun_out/hwq_$q.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"], d["mjpeg_fed_per_gpu"]["frames_per_s"])')"
  done
done
