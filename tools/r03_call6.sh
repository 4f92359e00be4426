#!/bin/bash
# Round close with the labelling gate (r03i: suite, smoke, bench, rocprof stats + PMC, config 5), then the
# workgroups-per-frame / contour-stream A/B.
set -o pipefail
bash tools/r03_final.sh r03i || exit 1
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh cur gw4 gw6 s4 || exit 1
