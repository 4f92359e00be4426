#!/bin/bash
# Round 6 close, call 1: the GPU suite on the product, the bounds-checked build on the parity / configuration / JPEG
# suites, smoke(), the driver's default command (configs[1] + the mode D / configs[2] / configs[4] side legs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06c1}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_$TAG.log)"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_jpeg.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_${TAG}_checked.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_${TAG}_checked.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 - "$TAG" <<'PY'
import json, sys; d=json.loads(open(f'gpurun_out/bench_{sys.argv[1]}.log').read().strip().splitlines()[-1]); r=d['roofline']
print('F', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], r['traffic'])
for k, v in d['side_configs'].items(): print(k, round(v['value']), v['ms_per_step'], v['roofline']['avg_launch_us'], v['roofline'].get('launch_std_us'), v['roofline']['frac'], v['roofline'].get('traffic'), (v.get('haar_stage') or {}).get('share_of_step_time'))
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], 'mjpeg', (d.get('mjpeg_fed_per_gpu') or {}).get('frames_per_s'), 'host_fed', (d.get('host_fed_per_gpu') or {}).get('frames_per_s'))
PY
echo "done $TAG"
