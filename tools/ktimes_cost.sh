#!/bin/bash
for K in "--no-ktimes" "" ; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $K > gpurun_out/q.log 2>&1 || { tail -3 gpurun_out/q.log; exit 1; }
  echo "$K $(tail -1 gpurun_out/q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
tools/timeline.sh c --no-ktimes | tail -2
