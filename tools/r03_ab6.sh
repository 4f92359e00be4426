#!/bin/bash
# k_regions with the tile flags staged in LDS: contour/config parity, then the driver's command x4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_ab6.log 2>&1 || { tail -30 gpurun_out/parity_ab6.log; exit 1; }
tail -1 gpurun_out/parity_ab6.log
bash tools/r03_drv.sh 4
