#!/bin/bash
# Round 5, call n: the committed build with two contour streams -- r05_l.sh (GPU suite, smoke, the default
# command, configs[4] with Haar and with masks), then the multi-rank rehearsal on the one GPU.
set -o pipefail
TAG=${1:-r05n}
tools/rounds/r05_l.sh $TAG || exit 1
tools/rehearse_multi.sh > gpurun_out/rehearse_$TAG.log 2>&1 || { tail -20 gpurun_out/rehearse_$TAG.log; exit 1; }
grep -E "n_gpus" gpurun_out/rehearse_$TAG.log
