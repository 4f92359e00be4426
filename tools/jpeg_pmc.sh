#!/bin/bash
# PMC passes over the Huffman kernel (decoder only).  Usage: tools/jpeg_pmc.sh [restart] [out_dir]
set -o pipefail
R=${1:-0}
OUT=${2:-gpurun_out/jpeg_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-include-regex "${KREGEX:-k_jpeg_huff}" -d "$OUT/p$i" -o run --output-format csv -- python3 tools/jpeg_only.py $R 2 > "$OUT/p$i.log" 2>&1 || exit 1
done
timeout -k 10 90 python3 tools/jpeg_only.py $R 3 > "$OUT/t.log" 2>&1
