#!/bin/bash
# Round 5, call ai: the per-frame contour workgroup at any image size (dev switch FM_FRAME_CCL=2): the parity /
# configuration GPU files through it (first call: 120 passed), then the driver's command and configs[2] A/B
# against the kernel chain (dev build both ways), 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
D=$PWD/find_motion_amd/libfm_hip_dev.so
if [ "${PARITY:-0}" = 1 ]; then
  FM_HIP_LIB=$D FM_FRAME_CCL=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_r05ai.log 2>&1 || { tail -40 gpurun_out/parity_r05ai.log; exit 1; }
  echo "frame-ccl parity: $(tail -1 gpurun_out/parity_r05ai.log)"
fi
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernels']; print(round(d['value']), d['ms_per_step'], {n: (v.get('avg_us'), v.get('std_us')) for n, v in k.items() if v.get('launches')})"; }
for r in 1 2 3; do
  for v in 1 2; do
    o=$(FM_HIP_LIB=$D FM_FRAME_CCL=$v timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r fccl$v $o"
  done
done
for v in 1 2; do
  o=$(FM_HIP_LIB=$D FM_FRAME_CCL=$v timeout -k 10 200 python bench.py --steps 20 --streams 8 --batch 128 $J | q) || exit 1
  echo "C2 fccl$v $o"
done
echo "done r05ai"
