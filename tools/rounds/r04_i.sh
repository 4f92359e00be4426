#!/bin/bash
# Round 4, call i: k_pix5 workgroup stamps (dev build, no phase stamps) of 25 consecutive launches of
# the driver's command, twice: are the long launches late-dispatched or slow-running workgroups?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04i}
J="--no-mjpeg --no-cpu-baseline --no-host-fed"
for r in 1 2; do
  FM_PTS=gpurun_out/pts_${TAG}_$r.bin FM_PTS_RING=25 FM_HIP_LIB=$PWD/abvar/pts/libfm_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_$r.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$r.log; exit 1; }
  grep '^{' gpurun_out/bench_${TAG}_$r.log | cut -c1-160
  python tools/pts_ring.py gpurun_out/pts_${TAG}_$r.bin 510 > gpurun_out/pts_${TAG}_$r.txt 2>&1
  cat gpurun_out/pts_${TAG}_$r.txt
done
echo "done $TAG"
