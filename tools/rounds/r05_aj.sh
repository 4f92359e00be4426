#!/bin/bash
# Round 5, call aj: k_pix5's blur x alpha table as static LDS at address 0, its byte offset by one SDWA shift
# (FM_P5_SDWA=1: 8 fewer VALU per wave-frame), the tap jobs' row pairs packed by v_perm (FM_P5_PERMPACK=1: 4 fewer
# per job), and both -- the parity file through both, then the driver's command A/B against the product, 4
# alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/abvar/sdwapack/libfm_hip.so
S=$PWD/abvar/sdwa/libfm_hip.so
K=$PWD/abvar/pack/libfm_hip.so
FM_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r05aj.log 2>&1 || { tail -40 gpurun_out/parity_r05aj.log; exit 1; }
echo "sdwa+pack parity: $(tail -1 gpurun_out/parity_r05aj.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
for r in 1 2 3 4; do
  for v in P S K V; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05aj"
