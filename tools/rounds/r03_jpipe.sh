#!/bin/bash
# Decoder with two device sets / streams: GPU JPEG tests, decoder bench, and the bench's MJPEG-fed figure.
set -o pipefail
mkdir -p gpurun_out
bash tools/r03_jpeg.sh jp2 || exit 1
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed > gpurun_out/bench_jp2.log 2>&1 || { tail -5 gpurun_out/bench_jp2.log; exit 1; }
tail -1 gpurun_out/bench_jp2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("value", d["value"], "mjpeg_fed", d["mjpeg_fed_per_gpu"])'
done
