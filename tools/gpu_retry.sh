#!/bin/bash
# Run one gpurun call, retrying (up to 8 times, 3 minutes apart) only while the pool answers that no
# box is free or the box was lost while being prepared (status=transient: nothing ran, nothing charged).
# Usage: tools/gpu_retry.sh OUTFILE TIMEOUT SCRIPT [ARGS...]
OUT=$1; TMO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  grep -q "status=transient" "$OUT" || exit 0
  sleep 180
done
