#!/bin/bash
# A/B of library builds on the GPU box (dev builds, so FM_SERIAL works): for each library, the default
# bench pipelined (frames/s, pixel-kernel event average) and serial (FM_SERIAL: contour pass on the pixel
# stream, so the pixel kernel runs alone), alternating libraries, REPS rounds.
# Usage: REPS=2 tools/ab.sh libA.so libB.so ...   (build: make -C find_motion_amd/csrc VARIANT=dev OUT=... OBJDIR=...)
set -o pipefail
REPS=${REPS:-2}
ARGS=${ARGS:-}
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']), d['roofline']['avg_launch_us'])"; }
for r in $(seq $REPS); do
  for lib in "$@"; do
    p=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed $ARGS | q) || exit 1
    s=$(FM_SERIAL=1 FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed $ARGS | q) || exit 1
    echo "$(basename $(dirname $lib)) r$r pipelined $p serial $s"
  done
done
