#!/bin/bash
# Round 5, call e: the product with the small-image path on by default (mode D) and without k_pix5's split
# variant: the GPU suite, the default bench line (mode D and configs[2] legs), A/B of k_pix5 with fewer
# scalar instructions (branch-free flag word, frame pointers by increment), configs[4] with the overlapped
# Haar stage on frames with faces, kernel traces of mode D and the headline, the headline's PMC passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05e}
P=$PWD/find_motion_amd/libfm_hip.so
L=$PWD/abvar/lean/libfm_hip.so
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_$TAG.log)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels']; print(round(d['value']), d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], r['launch_le_step'], {n: v['avg_us'] for n, v in k.items()}, d.get('haar_stage'))"; }
for r in 1 2 3; do
  for v in P L; do
    lib=${!v}
    o=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "F r$r $v $o"
  done
done
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10"
o=$(timeout -k 10 300 python bench.py $C5 $J --haar | q) || exit 1
echo "C5 haar $o"
o=$(timeout -k 10 300 python bench.py $C5 $J --masks | q) || exit 1
echo "C5 masks $o"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_D -o run --output-format csv -- python3 bench.py --mode D $J > gpurun_out/prof_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_D.log; exit 1; }
tools/profile.sh ${TAG}_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_F > gpurun_out/pmc_${TAG}_F.txt 2>&1
echo "done $TAG"
