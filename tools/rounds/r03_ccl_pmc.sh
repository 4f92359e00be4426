#!/bin/bash
# Instruction counts of the contour kernels per labelling variant (abvar/<NAME>): one SQ PMC pass each
# over the bench defaults.  Usage: tools/r03_ccl_pmc.sh NAME...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in "$@"; do
  OUT=$PWD/gpurun_out/cpmc_$N
  FM_HIP_LIB=$PWD/abvar/$N/libfm_hip.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    -d "$OUT" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg > "$OUT.log" 2>&1 || { tail -5 "$OUT.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT" > gpurun_out/cpmc_$N.txt 2>&1
  echo "pmc $N done"
done
