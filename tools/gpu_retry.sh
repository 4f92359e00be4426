#!/bin/bash
# Run one gpurun call, retrying (up to 8 times, 3 minutes apart) only while the pool answers that no
# box is free or the box was lost while being prepared (status=transient: nothing ran, nothing charged).
# Exits with gpurun's own status, so a failed GPU run is not reported as a pass.
# Usage: tools/gpu_retry.sh OUTFILE TIMEOUT SCRIPT [ARGS...]
OUT=$1; TMO=$2; shift 2
rc=3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  grep -q "status=transient" "$OUT" || exit $rc
  sleep 180
done
exit $rc
