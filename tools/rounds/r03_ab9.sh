#!/bin/bash
# A/B of abvar variants with the driver's 20-step command, alternating (ROUNDS), order flipped each round.
set -o pipefail
mkdir -p gpurun_out
i=0
for r in ${ROUNDS:-1 2 3 4 5 6}; do
  if [ $((i % 2)) -eq 0 ]; then ORDER="$*"; else ORDER=$(echo "$*" | awk '{for(i=NF;i>0;i--) printf "%s ", $i}'); fi
  i=$((i+1))
  for N in $ORDER; do
    FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/abd_$N.log 2>&1 || { tail -3 gpurun_out/abd_$N.log; exit 1; }
    echo "$N round $r $(tail -1 gpurun_out/abd_$N.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
