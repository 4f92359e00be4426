#!/bin/bash
# Round 5, call ar: the driver's default command twice on another fresh box (the committed build), for the spread.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r05ar_$i.log 2>&1 || { tail -20 gpurun_out/bench_r05ar_$i.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r05ar_$i.log').read().strip().splitlines()[-1]); r=d['roofline']
print('F', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], {k: round(v['value']) for k, v in d['side_configs'].items()})"
done
echo "done r05ar"
