#!/bin/bash
# Decoder kernel times at several frames-per-call (rocprofv3 kernel stats).  Usage: tools/jpeg_scale_prof.sh N...
set -o pipefail
export TMPDIR=/tmp
for n in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/jscale_$n -o run --output-format csv -- python3 tools/jpeg_only.py 0 3 $n 75 > gpurun_out/jscale_$n.log 2>&1 || exit 1
done
