#!/bin/bash
# Quick pixel-kernel PMC pass (VALU/SALU/LDS instruction counts) on the default bench.
TAG=${1:-pp}
OUT=$PWD/gpurun_out/pp_$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d "$OUT" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/log" 2>&1 || { tail -5 "$OUT/log"; exit 1; }
python3 tools/pmc_summary.py "$OUT" | grep -A9 "k_pix<5, false, false>"
