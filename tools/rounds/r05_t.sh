#!/bin/bash
# Round 5, call t: per-phase cycles of k_tile_ccl's labelled tiles (dev build FM_TS: s_memtime at dilation,
# run count, run records, pairs, union rounds, fold, outputs), the headline workload (results of the timing
# only; the stamps' device-to-host copies in fm_wait serialise the pipeline).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 10 --warmup 3"
FM_TS=1 FM_HIP_LIB=$PWD/find_motion_amd/libfm_hip_dev.so timeout -k 10 300 python bench.py $J > gpurun_out/ts_r05t.json 2> gpurun_out/ts_r05t.log || { tail -20 gpurun_out/ts_r05t.log; exit 1; }
grep -iE "phase|cycles|[0-9]:[0-9]" gpurun_out/ts_r05t.log | tail -5
echo "done r05t"
