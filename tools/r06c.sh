#!/bin/bash
# Round 6, call c: the driver's default command (with the mode D, configs[2] and configs[4] side legs), then the
# multi-rank rehearsal (incl. configs[3]'s per-rank shape at two ranks on the one card).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r06c.log 2>&1 || { tail -20 gpurun_out/bench_r06c.log; exit 1; }
echo "default command: $(( $(date +%s) - s )) s"
python3 - <<'PY'
import json; d=json.loads(open('gpurun_out/bench_r06c.log').read().strip().splitlines()[-1]); r=d['roofline']
print('F', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], r['traffic'])
for k, v in d['side_configs'].items(): print(k, round(v['value']), v['ms_per_step'], v['roofline']['avg_launch_us'], v['roofline'].get('launch_std_us'), v['roofline']['frac'], v['roofline'].get('traffic'), (v.get('haar_stage') or {}).get('share_of_step_time'))
print('cpu', d['cpu_baseline'])
PY
tools/rehearse_multi.sh > gpurun_out/rehearse_r06c.log 2>&1 || { tail -20 gpurun_out/rehearse_r06c.log; exit 1; }
grep -E "n_gpus|configs" gpurun_out/rehearse_r06c.log
echo "done r06c"
