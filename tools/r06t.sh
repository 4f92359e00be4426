#!/bin/bash
# Round 6, call t: k_hdetect window tiles of 32 x 16, 32 x 32 and 16 x 32 windows (FM_HAAR_TW / TH: more windows
# pooled per workgroup, so each phase -- the tail above all -- packs more survivors per wave) against 16 x 16
# (r06t_base, the product). The Haar GPU tests through each variant, then configs[4] with its Haar stage,
# 3 alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/abvar/r06t_base/libfm_hip.so; P=$PWD/abvar/r06t_32x16/libfm_hip.so
V="$PWD/abvar/r06t_32x32/libfm_hip.so $PWD/abvar/r06t_16x32/libfm_hip.so"
for lib in $P $V; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/r06t_parity_$n.log 2>&1 || { tail -30 gpurun_out/r06t_parity_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/r06t_parity_$n.log)"
done
A="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --haar"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
for r in 1 2 3; do
  for lib in $B $P $V; do
    n=$(basename $(dirname $lib))
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $A $J > gpurun_out/r06t_${n}_r$r.log 2>&1 || { tail -20 gpurun_out/r06t_${n}_r$r.log; exit 1; }
    python3 - gpurun_out/r06t_${n}_r$r.log "$n" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']; h = d['haar_stage']
print(f"r{sys.argv[3]} {sys.argv[2]} {round(d['value'])} {d['ms_per_step']} pix {r['avg_launch_us']} std {r.get('launch_std_us')} "
      f"haar_dev_ms {h['device_ms']} share {h['share_of_step_time']} det {h['detections']} roi {h['roi_frames']}")
PY
  done
done
echo "done r06t"
