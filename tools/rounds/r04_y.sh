#!/bin/bash
# Round 4, call y (as call h, final): the GPU suite on the committed kernels, smoke, the driver's bench line, mode D,
# configs[2], configs[4] (Haar stage / masks), then kernel traces + PMC passes (HBM bytes) of the
# headline, configs[4] geometry and mode D for profiles/traffic.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04y}
J="--no-mjpeg --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 $J --no-host-fed > gpurun_out/bench_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_D.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_D.log | cut -c1-300
timeout -k 10 300 python bench.py --streams 8 --batch 128 --steps 20 --warmup 5 $J > gpurun_out/bench_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c2.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c2.log | cut -c1-300
C5="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --no-host-fed"
timeout -k 10 300 python bench.py $C5 $J --haar > gpurun_out/bench_${TAG}_c5h.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5h.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c5h.log | cut -c1-300
timeout -k 10 300 python bench.py $C5 $J --masks > gpurun_out/bench_${TAG}_c5m.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_c5m.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c5m.log | cut -c1-300
tools/profile.sh ${TAG}_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_F > gpurun_out/pmc_${TAG}_F.txt 2>&1
tools/profile.sh ${TAG}_c5 $C5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_c5 > gpurun_out/pmc_${TAG}_c5.txt 2>&1
echo "done $TAG"
