#!/bin/bash
# LDS bank conflicts / activity of the pixel kernel per stage (dev build, serial, FM_DEBUG_SKIP stage
# ablations: 1 = no gray/horizontal stage, 2 = no chain, 9 = no gray stage and no raw->LDS stores;
# results invalid, counters only).  Prints the k_pix<5,false,false> means per dispatch.
set -o pipefail
export TMPDIR=/tmp FM_SERIAL=1
export FM_HIP_LIB=${FM_HIP_LIB:-$PWD/find_motion_amd/libfm_hip_dev.so}
for skip in ${SKIPS:-0 1 2 9}; do
  OUT=$PWD/gpurun_out/lds_${TAG:-x}_$skip; mkdir -p $OUT
  FM_DEBUG_SKIP=$skip timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES} \
     -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
  echo "== skip $skip"; python3 tools/pmc_summary.py $OUT | grep -A9 "${KNAME:-k_pix<5, false, false>}" | tail -8
done
