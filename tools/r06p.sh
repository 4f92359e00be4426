#!/bin/bash
# Round 6, call p: k_hdetect's phases (verdict r05 item 5) -- the survivors compacted after stages 1 and 2 as well
# as after the head (FM_HAAR_HEADC) and the last phase packed into the first waves instead of spread over four
# (FM_HAAR_TAIL_SPREAD=0). The Haar GPU tests through every new library, then configs[4] with its Haar stage,
# 3 alternating rounds: base = the previous product, find_motion_amd = both, r06p_spread = compaction with the
# spread tail, r06p_nohc = the packed tail alone.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/abvar/r06p_base/libfm_hip.so; P=$PWD/find_motion_amd/libfm_hip.so
LIBS="$B $P $PWD/abvar/r06p_spread/libfm_hip.so $PWD/abvar/r06p_nohc/libfm_hip.so"
for lib in $P $PWD/abvar/r06p_spread/libfm_hip.so $PWD/abvar/r06p_nohc/libfm_hip.so; do
  n=$(basename $(dirname $lib))
  FM_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_haar.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/r06p_parity_$n.log 2>&1 || { tail -30 gpurun_out/r06p_parity_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/r06p_parity_$n.log)"
done
A="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --haar"
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
for r in 1 2 3; do
  for lib in $LIBS; do
    n=$(basename $(dirname $lib))
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $A $J > gpurun_out/r06p_${n}_r$r.log 2>&1 || { tail -20 gpurun_out/r06p_${n}_r$r.log; exit 1; }
    python3 - gpurun_out/r06p_${n}_r$r.log "$n" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']; h = d['haar_stage']
print(f"r{sys.argv[3]} {sys.argv[2]} {round(d['value'])} {d['ms_per_step']} pix {r['avg_launch_us']} std {r.get('launch_std_us')} "
      f"haar_dev_ms {h['device_ms']} share {h['share_of_step_time']} det {h['detections']} roi {h['roi_frames']}")
PY
  done
done
echo "done r06p"
