#!/bin/bash
# PMC passes over the Haar detector (frontalface 64-frame bench): instruction mix, waits, LDS, HBM bytes.
set -o pipefail
OUT=${1:-gpurun_out/haar_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d "$OUT/pmc$i" -o run --output-format csv -- python3 tools/bench_haar.py --frontalface --cpu-frames 0 > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo "haar pmc done"
