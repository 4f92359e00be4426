#!/bin/bash
# Round 5, call v: the contour pass's simple-tile path (FM_CCL_SIMPLE, abvar/simple): the contour and
# configuration GPU tests on it and on its bounds-checked build, then the driver's command A/B (3 rounds).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$PWD/abvar/simple/libfm_hip.so
SC=$PWD/abvar/simplechk/libfm_hip.so
FM_HIP_LIB=$S timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_r05v_simple.log 2>&1 || { tail -60 gpurun_out/parity_r05v_simple.log; exit 1; }
echo "simple: $(tail -1 gpurun_out/parity_r05v_simple.log)"
FM_HIP_LIB=$SC timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "simple or heavy or golden or random or full_tiles or mode_d or small" --timeout 300 --timeout-method thread > gpurun_out/parity_r05v_simplechk.log 2>&1 || { tail -40 gpurun_out/parity_r05v_simplechk.log; exit 1; }
echo "simple checked: $(tail -1 gpurun_out/parity_r05v_simplechk.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3; do
  for v in P S; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05v"
