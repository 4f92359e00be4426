set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_r06b.log 2>&1 || { tail -40 gpurun_out/parity_r06b.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/parity_r06b.log)"
P=$PWD/find_motion_amd/libfm_hip.so; O=$PWD/abvar/r5/libfm_hip.so
REPS=2 ARGS="--streams 2 --steps 20 --warmup 5" tools/ab_bench.sh s2 $P $O || exit 1
REPS=2 ARGS="--streams 4 --batch 128 --steps 30 --warmup 5" tools/ab_bench.sh s4 $P $O || exit 1
REPS=2 ARGS="--streams 8 --batch 128 --steps 60 --warmup 5" tools/ab_bench.sh c2 $P $O || exit 1
REPS=2 ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 20 --warmup 10 --masks" tools/ab_bench.sh c4 $P $O || exit 1
