#!/bin/bash
# Decode-side ablation (results invalid): kernel times with / without the planes' HBM round trip.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in jabl0 jabl3; do
  FM_HIP_LIB=$PWD/abvar/$v/libfm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run --output-format csv -- python3 tools/bench_mjpeg.py 192 75 > gpurun_out/prof_$v.log 2>&1 || exit 1
  echo $v; find gpurun_out/prof_$v -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | grep jp
done
