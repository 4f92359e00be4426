#!/bin/bash
# Round 5, call h: k_small_scan's blur-byte prefetch depth (NG groups of 8 frames in flight: 2 = the old
# depth, 4, 8) on mode D, 3 alternating rounds; the small-path parity tests on the deepest variant.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'))"; }
N2=$PWD/find_motion_amd/libfm_hip.so
N4=$PWD/abvar/ng4/libfm_hip.so
N8=$PWD/abvar/ng8/libfm_hip.so
FM_HIP_LIB=$N8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "small" --timeout 120 --timeout-method thread > gpurun_out/parity_r05h_ng8.log 2>&1 || { tail -30 gpurun_out/parity_r05h_ng8.log; exit 1; }
echo "ng8 small parity: $(tail -1 gpurun_out/parity_r05h_ng8.log)"
for r in 1 2 3; do
  for v in N2 N4 N8; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
    echo "D r$r $v $o"
  done
done
V=$PWD/find_motion_amd/libfm_hip_dev.so
FM_STAMP_DUMP=1 FM_HIP_LIB=$V timeout -k 10 200 python bench.py --mode D $J > gpurun_out/stamps_r05h_D.json 2> gpurun_out/stamps_r05h_D.txt || exit 1
python3 tools/stamp_pipeline.py gpurun_out/stamps_r05h_D.txt 24
FM_STAMP_DUMP=1 FM_HIP_LIB=$V timeout -k 10 200 python bench.py $J > gpurun_out/stamps_r05h_F.json 2> gpurun_out/stamps_r05h_F.txt || exit 1
python3 tools/stamp_pipeline.py gpurun_out/stamps_r05h_F.txt 24
echo "done r05h"
