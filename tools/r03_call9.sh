#!/bin/bash
# Round close with 6 batch slots (r03k), then 4 vs 6 slots again.
set -o pipefail
bash tools/r03_final.sh r03k || exit 1
ROUNDS="1 2 3 4" bash tools/r03_ab9.sh sl4 sl6 || exit 1
