#!/bin/bash
# Steady-state (default bench) A/B of runtime environment knobs, alternating, 2 rounds.
# Usage: tools/ab_env.sh "NAME=VAL ..." "NAME=VAL ..."   ("-" = no variable)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/abe_$i.log 2>&1 || { tail -3 gpurun_out/abe_$i.log; exit 1; }
    echo "[$E] round $r $(tail -1 gpurun_out/abe_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"])')"
  done
done
