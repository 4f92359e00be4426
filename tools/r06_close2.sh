#!/bin/bash
# Round 6 close, call 2: kernel trace + PMC passes (tools/profile.sh) of the named workloads on the final build, each
# bench line beside its profile for tools/traffic.py; then (with "default") the driver's default command.
#   tools/r06_close2.sh TAG F c2 default      tools/r06_close2.sh TAG c4h c4m
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side"
C4="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
run() {  # name, args
  local n=$1; shift
  tools/profile.sh ${TAG}_$n "$@" || { echo "profile $n failed"; exit 1; }
  timeout -k 10 300 python bench.py "$@" $J > gpurun_out/bench_${TAG}_$n.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/bench_${TAG}_$n.log | cut -c1-160)"
}
for w in "$@"; do
  case $w in
    F) run F --steps 20 --warmup 5 ;;
    c2) run c2 --streams 8 --batch 128 --steps 60 --warmup 5 ;;
    c4h) run c4h $C4 --haar ;;
    c4m) run c4m $C4 --masks ;;
    default)
      timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_default.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_default.log; exit 1; }
      python3 - "$TAG" <<'PY'
import json, sys; d=json.loads(open(f'gpurun_out/bench_{sys.argv[1]}_default.log').read().strip().splitlines()[-1]); r=d['roofline']
print('F', round(d['value']), d['ms_per_step'], r['avg_launch_us'], r.get('launch_std_us'), r['frac'], r['traffic'])
for k, v in d['side_configs'].items(): print(k, round(v['value']), v['ms_per_step'], v['roofline']['avg_launch_us'], v['roofline'].get('launch_std_us'), v['roofline']['frac'], v['roofline'].get('traffic'), (v.get('haar_stage') or {}).get('share_of_step_time'))
PY
      ;;
  esac
done
echo "done $TAG"
