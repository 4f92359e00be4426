#!/bin/bash
# Round 5, call s: contour workgroups per frame in k_tile_ccl / k_merge / k_fold / k_emit (GW = 4 product, 3, 2):
# the driver's command without side legs, 3 alternating rounds; contour parity tests on the smallest GW.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FM_HIP_LIB=$PWD/abvar/gw2/libfm_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -k "heavy or golden or random or full_tiles or lattice or node_pool or contours_past or bench_shape" --timeout 300 --timeout-method thread > gpurun_out/parity_r05s_gw2.log 2>&1 || { tail -40 gpurun_out/parity_r05s_gw2.log; exit 1; }
echo "gw2: $(tail -1 gpurun_out/parity_r05s_gw2.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
G3=$PWD/abvar/gw3/libfm_hip.so
G2=$PWD/abvar/gw2/libfm_hip.so
for r in 1 2 3; do
  for v in P G3 G2; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05s"
