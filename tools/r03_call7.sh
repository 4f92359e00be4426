#!/bin/bash
# Round close with 4 contour workgroups per frame (r03j), then 3 vs 4 contour streams on top of it.
set -o pipefail
bash tools/r03_final.sh r03j || exit 1
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh cur s4 || exit 1
