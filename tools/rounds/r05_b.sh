#!/bin/bash
# Round 5, call b: k_pixq (no frame barrier, wave-private gray/taps) against k_pix5 -- the GPU suite on the
# k_pixq library, then alternating A/B rounds of the driver's bench command, then a kernel trace + the SQ
# pass of k_pixq.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05b}
Q=$PWD/abvar/pixq/libfm_hip.so
P=$PWD/find_motion_amd/libfm_hip.so
Q2=$PWD/abvar/pixq2/libfm_hip.so
FM_HIP_LIB=$Q timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
tail -2 gpurun_out/parity_$TAG.log
FM_HIP_LIB=$Q2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/parity_${TAG}_pf2.log 2>&1 || { tail -40 gpurun_out/parity_${TAG}_pf2.log; exit 1; }
tail -2 gpurun_out/parity_${TAG}_pf2.log
J="--no-cpu-baseline --no-host-fed --no-mjpeg --no-side --steps 20 --warmup 5"
q() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['avg_launch_us'], r['frac'], r['launch_le_step'])"; }
for r in 1 2 3; do
  for lib in $P $Q $Q2; do
    v=$(FM_HIP_LIB=$lib timeout -k 10 200 python bench.py $J | q) || exit 1
    echo "r$r $(basename $(dirname $lib)) $v"
  done
done
FM_HIP_LIB=$Q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $J > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log | cut -c1-200
FM_HIP_LIB=$Q timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/prof_${TAG}_pmc1 -o run --output-format csv -- python3 bench.py $J > gpurun_out/prof_${TAG}_pmc1.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_pmc1.log; exit 1; }
FM_HIP_LIB=$Q timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof_${TAG}_pmc2 -o run --output-format csv -- python3 bench.py $J > gpurun_out/prof_${TAG}_pmc2.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_pmc2.log; exit 1; }
echo "done $TAG"
