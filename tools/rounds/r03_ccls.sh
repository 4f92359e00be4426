#!/bin/bash
# Contour-stream count with 8 hardware queues per process (dev library, FM_CCL_STREAMS): the driver's
# 20-step command, alternating, order flipped each round.  "-" = the default (3 streams).
set -o pipefail
mkdir -p gpurun_out
LIB=$PWD/find_motion_amd/libfm_hip_dev.so
i=0
for r in ${ROUNDS:-1 2 3 4}; do
  if [ $((i % 2)) -eq 0 ]; then ORDER="$*"; else ORDER=$(echo "$*" | awk '{for(i=NF;i>0;i--) printf "%s ", $i}'); fi
  i=$((i+1))
  for N in $ORDER; do
    E=""; [ "$N" != "-" ] && E="FM_CCL_STREAMS=$N"
    env $E FM_HIP_LIB=$LIB timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/ccls_$N.log 2>&1 || { tail -3 gpurun_out/ccls_$N.log; exit 1; }
    echo "streams $N round $r $(tail -1 gpurun_out/ccls_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
