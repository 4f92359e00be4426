#!/bin/bash
# Round 5, call m: contour streams per context (dev build FM_CCL_STREAMS = 1 / 2 / 3, the product's 3): the
# driver's command without side legs, 3 alternating rounds -- throughput and the pixel launch's spread;
# then a kernel trace of configs[4] with its Haar stage (the detector's kernels beside k_pixw).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05m}
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
V=$PWD/find_motion_amd/libfm_hip_dev.so
for r in 1 2 3; do
  for n in 1 2 3; do
    o=$(FM_CCL_STREAMS=$n FM_HIP_LIB=$V timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "F r$r cs$n $o"
  done
done
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c5h -o run --output-format csv -- python3 bench.py $C5 $J --haar > gpurun_out/prof_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c5h.log; exit 1; }
echo "done $TAG"
