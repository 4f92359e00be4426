#!/bin/bash
# Round 5, call j: k_frame_contours with workgroup-scope barriers (call i's agent-scope fences wrote back
# and invalidated the L2 at every step): the small-image / contour GPU tests (product and bounds-checked),
# mode D A/B product vs the resize with the next row pair's loads in flight (RSPF), the stamp pipeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05j}
K="frame_contour or small or heavy or golden or random or full_tiles or mode_d or node_pool or selection or resize"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
echo "subset: $(tail -1 gpurun_out/parity_$TAG.log)"
FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_checked.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/parity_${TAG}_checked.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_checked.log; exit 1; }
echo "checked: $(tail -1 gpurun_out/parity_${TAG}_checked.log)"
FM_HIP_LIB=$PWD/abvar/rspf/libfm_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "resize or small or mode_d" --timeout 300 --timeout-method thread > gpurun_out/parity_${TAG}_rspf.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_rspf.log; exit 1; }
echo "rspf: $(tail -1 gpurun_out/parity_${TAG}_rspf.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'), d.get('contour_pass'))"; }
P=$PWD/find_motion_amd/libfm_hip.so
R=$PWD/abvar/rspf/libfm_hip.so
for r in 1 2 3; do
  for v in P R; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
V=$PWD/find_motion_amd/libfm_hip_dev.so
FM_STAMP_DUMP=1 FM_HIP_LIB=$V timeout -k 10 200 python bench.py --mode D $J > gpurun_out/stamps_${TAG}_D.json 2> gpurun_out/stamps_${TAG}_D.txt || exit 1
python3 tools/stamp_pipeline.py gpurun_out/stamps_${TAG}_D.txt 24 | tail -8
echo "done $TAG"
