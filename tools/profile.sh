#!/bin/bash
# Profile a workload on the GPU box: kernel-trace stats + PMC passes.
# Usage: tools/profile.sh <tag> [args...]   (outputs under gpurun_out/prof_<tag>/)
#   PROG=bench.py (default; the bench's side legs are turned off) or any other script, e.g.
#   PROG=tools/bench_haar.py tools/profile.sh r04_haar --frontalface --iters 10
set -o pipefail
TAG=${1:-run}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
[ -z "$GRAFT_REPO_ROOT" ] && OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PROG=${PROG:-bench.py}
if [ "$PROG" = bench.py ]; then ARGS="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side $*"; else ARGS="$*"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $PROG $ARGS > "$OUT/trace.log" 2>&1 || exit 1
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC -d "$OUT/pmc$i" -o run --output-format csv -- python3 $PROG $ARGS > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo "profile $TAG done"
