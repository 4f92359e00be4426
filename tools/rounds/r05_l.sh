#!/bin/bash
# Round 5, call l: the committed build -- the GPU suite, smoke(), the driver's default command (with the
# 60-step mode D and configs[2] side legs), configs[4] with its Haar stage and with masks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05l}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_$TAG.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1]); r=d['roofline']
print('F', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], r['traffic'])
for k, v in d['side_configs'].items(): print(k, round(v['value']), v['ms_per_step'], v['roofline']['avg_launch_us'], v['roofline'].get('launch_std_us'), v['roofline']['frac'], v['roofline'].get('traffic'), {n: x['avg_us'] for n, x in v['kernels'].items()})
print('mjpeg', d.get('mjpeg_fed_per_gpu', d.get('mjpeg')), 'host_fed', d.get('host_fed_per_gpu'))
"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
timeout -k 10 300 python bench.py $C5 $J --masks > gpurun_out/bench_${TAG}_c5m.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5m.log; exit 1; }
for f in c5h c5m; do python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], (d.get('haar_stage') or {}).get('share_of_step_time'))"; done
echo "done $TAG"
