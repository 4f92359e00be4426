#!/bin/bash
# N>1 rehearsal on the box's one GPU (every rank pinned to device 0 over gloo; RCCL refuses two
# ranks on one device): bench.py's own rank spawning at --gpus 2 and 4, and the driver's
# torch.distributed.run form at 2 ranks.  Checks that rank 0 prints one line with n_gpus = N.
set -o pipefail
mkdir -p gpurun_out
export FM_BENCH_DEVICE=0 FM_BENCH_BACKEND=gloo
check() { grep '^{' "$1" | python -c "import json,sys; L=sys.stdin.read().splitlines(); assert len(L)==1, L; d=json.loads(L[0]); assert d['n_gpus']==$2, d['n_gpus']; print('$1', 'n_gpus', d['n_gpus'], 'value', d['value'], 'ms/step', d['ms_per_step'])"; }
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-host-fed --no-mjpeg > gpurun_out/n2_spawn.log 2>&1 || { tail -20 gpurun_out/n2_spawn.log; exit 1; }
check gpurun_out/n2_spawn.log 2 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/n2_torchrun.log 2>&1 || { tail -20 gpurun_out/n2_torchrun.log; exit 1; }
check gpurun_out/n2_torchrun.log 2 || exit 1
# four processes on the ONE card: 4 x 8 hardware queues (bench.py's default per process) oversubscribe the
# card's queue slots and the ranks time-share (133 k aggregate, round 5); at 4 queues per process they fit.
# (On a real node every rank has a card of its own and keeps its 8 queues.)
FM_BENCH_HW_QUEUES=4 timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/n4_spawn.log 2>&1 || { tail -20 gpurun_out/n4_spawn.log; exit 1; }
check gpurun_out/n4_spawn.log 4 || exit 1
# configs[3]'s per-rank shape (8 x 1080p streams per rank, 128 frames per step, a 12.7 GB ring per rank) at two
# ranks on the one card: the line must read "configs[3] family: 8 streams per GPU x 2 GPUs", world_size_seen 2
FM_BENCH_HW_QUEUES=4 timeout -k 10 400 python bench.py --gpus 2 --streams 8 --batch 128 --steps 20 --warmup 3 --no-cpu-baseline --no-host-fed --no-mjpeg > gpurun_out/n2_c3.log 2>&1 || { tail -20 gpurun_out/n2_c3.log; exit 1; }
check gpurun_out/n2_c3.log 2 || exit 1
grep '^{' gpurun_out/n2_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); w=d['config']['workload']; assert w.startswith('configs[3] family'), w; assert d['ranks']['world_size_seen'] == 2; print('configs[3] family', d['value'], d['ranks'])"
