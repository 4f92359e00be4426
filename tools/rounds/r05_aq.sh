#!/bin/bash
# Round 5, call aq: k_pixw without the keep-mask register copies when no stream has a mask (2 fewer VALU per
# wave-frame, 81 -> 79 VGPRs) -- the k = 21 / config-5 GPU tests, then configs[4]'s geometry without masks (the
# Haar leg's pixel kernel) A/B against the previous build, 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu -k "k21 or config5 or wide" --timeout 300 --timeout-method thread > gpurun_out/parity_r05aq.log 2>&1 || { tail -40 gpurun_out/parity_r05aq.log; exit 1; }
echo "k21 tests: $(tail -1 gpurun_out/parity_r05aq.log)"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
B=$PWD/abvar/prev/libfm_hip.so
for r in 1 2 3; do
  for v in P B; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $C5 $J | q) || exit 1
    echo "C5 r$r $v $o"
  done
done
echo "done r05aq"
