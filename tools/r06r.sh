#!/bin/bash
# Round 6, call r: k_hdetect's tail with GL lanes per window (FM_HAAR_GROUP; a stage's stumps dealt over the window's
# lanes, a butterfly sum -- exact in any order for order_free cascades) against the packed per-lane tail (r06r_base,
# the previous product). The Haar GPU tests through each new library (and the bounds-checked build's Haar file), then
# configs[4] with its Haar stage, 3 alternating rounds: GL = 8 (find_motion_amd), 4, 16.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/abvar/r06r_base/libfm_hip.so; P=$PWD/find_motion_amd/libfm_hip.so
V="$PWD/abvar/r06r_g4/libfm_hip.so $PWD/abvar/r06r_g16/libfm_hip.so"
for lib in $P $V; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/r06r_parity_$n.log 2>&1 || { tail -30 gpurun_out/r06r_parity_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/r06r_parity_$n.log)"
done
A="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --haar"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
for r in 1 2 3; do
  for lib in $B $P $V; do
    n=$(basename $(dirname $lib))
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $A $J > gpurun_out/r06r_${n}_r$r.log 2>&1 || { tail -20 gpurun_out/r06r_${n}_r$r.log; exit 1; }
    python3 - gpurun_out/r06r_${n}_r$r.log "$n" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']; h = d['haar_stage']
print(f"r{sys.argv[3]} {sys.argv[2]} {round(d['value'])} {d['ms_per_step']} pix {r['avg_launch_us']} std {r.get('launch_std_us')} "
      f"haar_dev_ms {h['device_ms']} share {h['share_of_step_time']} det {h['detections']} roi {h['roi_frames']}")
PY
  done
done
echo "done r06r"
