#!/bin/bash
# Round 5, call ah: where k_tile_ccl's instructions go now (dev build ablations, results invalid: 0 = as the product,
# 256 = compact / general tiles take the empty record, 512 = simple ones too), one PMC pass each; then the
# driver's command, compact tiles (product) vs the previous contour source, 3 more alternating rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --warmup 5"
D=$PWD/find_motion_amd/libfm_hip_dev.so
for v in 0 256 512; do
  FM_HIP_LIB=$D FM_DEBUG_SKIP=$v timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmc_ah_$v -o run --output-format csv -- python3 bench.py --steps 20 $J > gpurun_out/pmc_ah_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - gpurun_out/pmc_ah_$v/run_counter_collection.csv $v <<'PY'
import csv, sys, collections
s = collections.defaultdict(float); n = collections.Counter()
for row in csv.DictReader(open(sys.argv[1])):
    k = row["Kernel_Name"]
    if "k_tile_ccl" not in k and "k_frame" not in k: continue
    s[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
print("skip", sys.argv[2], {c: round(s[c] / max(n[c], 1) / 1e6, 3) for c in s}, "dispatches", n.get("SQ_INSTS_VALU"))
PY
done
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'])"; }
P=$PWD/find_motion_amd/libfm_hip.so
B=$PWD/abvar/base/libfm_hip.so
for r in 1 2 3; do
  for v in P B; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
echo "done r05ah"
