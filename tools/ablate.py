#!/usr/bin/env python3
"""Time the fused kernel with stages skipped (FM_DEBUG_SKIP bitmask; results invalid).
bits: 1 gray, 2 horizontal taps, 4 vertical+chain, 8 dilate+mask out, 16 raw load/store."""
import os
import subprocess
import sys

masks = [int(m) for m in sys.argv[1:]] or [0, 1, 2, 4, 8, 16, 1 | 2, 1 | 2 | 4, 1 | 2 | 4 | 8, 31]
for m in masks:
    env = dict(os.environ, FM_DEBUG_SKIP=str(m))
    out = subprocess.run([sys.executable, "bench.py", "--no-cpu-baseline", "--steps", "10", "--warmup", "2"],
                         env=env, capture_output=True, text=True).stdout.strip().splitlines()[-1]
    import json
    d = json.loads(out)
    print(f"skip={m:3d} fused_us={d['kernels']['fused']['avg_us']:9.2f}", flush=True)
