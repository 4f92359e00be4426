#!/bin/bash
# Default bench N times (variance check).
for i in $(seq ${N:-3}); do
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/rep.log 2>&1 || { tail -3 gpurun_out/rep.log; exit 1; }
  tail -1 gpurun_out/rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("value", d["value"], "pix_us", d["roofline"]["avg_launch_us"] if d["roofline"] else None)'
done
