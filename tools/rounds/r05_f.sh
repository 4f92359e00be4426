#!/bin/bash
# Round 5, call f: is mode D's loop host-bound? (host time in fm_submit / fm_wait per step beside the
# stamped resize); the headline's trace + PMC passes without the side legs (tools/profile.sh --no-side).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05f}
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()}, d.get('host_us_per_step'))"; }
for r in 1 2; do
  o=$(timeout -k 10 200 python bench.py --mode D $J | q) || exit 1
  echo "D r$r $o"
  o=$(timeout -k 10 200 python bench.py $J | q) || exit 1
  echo "F r$r $o"
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/prof_${TAG}_Dapi -o run --output-format csv -- python3 bench.py --mode D $J > gpurun_out/prof_${TAG}_Dapi.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_Dapi.log; exit 1; }
tools/profile.sh ${TAG}_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_F > gpurun_out/pmc_${TAG}_F.txt 2>&1
echo "done $TAG"
