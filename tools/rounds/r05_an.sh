#!/bin/bash
# Round 5, call an: kernel trace + PMC passes of the headline on the final k_pix5 (SDWA table offset, v_perm row
# pairs) and compact tiles -- the traffic.json entry and the profile the bench line's roofline cites.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/profile.sh r05an_F --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05an_F > gpurun_out/pmc_r05an_F.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --no-mjpeg --no-side > gpurun_out/bench_r05an_F.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r05an_F.log | cut -c1-300
echo "done r05an"
