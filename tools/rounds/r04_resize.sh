#!/bin/bash
# Round 4: the register-resident INTER_AREA kernel (k_resize_area_nt): parity, mode-D bench, kernel stats + PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04rs}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_haar.py -x -v -m gpu -k "resize or mode_d or fast_area or haar or frontalface or detect" --timeout 300 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -3 gpurun_out/parity_$TAG.log
timeout -k 10 300 python bench.py --mode D --steps 20 --warmup 5 --no-mjpeg --no-host-fed --no-cpu-baseline > gpurun_out/bench_${TAG}_D.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_D.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_D.log | cut -c1-1800
tools/profile.sh ${TAG}_D --mode D --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_D > gpurun_out/pmc_${TAG}_D.txt 2>&1
grep -A12 -i resize gpurun_out/pmc_${TAG}_D.txt | head -40 || true
timeout -k 10 300 python tools/bench_haar.py --frontalface > gpurun_out/haar_${TAG}.log 2>&1 || { tail -20 gpurun_out/haar_${TAG}.log; exit 1; }
tail -5 gpurun_out/haar_${TAG}.log
