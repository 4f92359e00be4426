#!/bin/bash
# Round 5, call i: the per-frame contour workgroup for small work images (k_frame_contours): the GPU suite,
# the bounds-checked build on the small-image and contour tests, mode D (product, 3 runs) and its launch
# stamp pipeline (dev build), the headline once.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05i}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_$TAG.log)"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "frame_contour or small or heavy or golden or random or full_tiles or mode_d or node_pool" --timeout 300 --timeout-method thread > gpurun_out/parity_${TAG}_checked.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_${TAG}_checked.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'), d.get('contour_pass'))"; }
for r in 1 2 3; do
  o=$(timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
  echo "D r$r $o"
done
V=$PWD/find_motion_amd/libfm_hip_dev.so
FM_STAMP_DUMP=1 FM_HIP_LIB=$V timeout -k 10 200 python bench.py --mode D $J > gpurun_out/stamps_${TAG}_D.json 2> gpurun_out/stamps_${TAG}_D.txt || exit 1
python3 tools/stamp_pipeline.py gpurun_out/stamps_${TAG}_D.txt 24 | tail -8
o=$(timeout -k 10 200 python bench.py $J | q) || exit 1
echo "F $o"
echo "done $TAG"
