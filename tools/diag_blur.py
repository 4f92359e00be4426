#!/usr/bin/env python3
"""Diagnostic: where the GPU blur plane differs from the oracle (small mode-Fast case)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import oracle
from find_motion_amd import MotionEngine, make_gaussian
from find_motion_amd._native import PLANE_BLUR, PLANE_GRAY
from find_motion_amd.synthetic import batch

W, H, box, bs = [int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (160, 120, 80, 20))]
k = make_gaussian(box, bs)
for rep in range(3):
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=3, keep_planes=True)
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k, thresh=12, alpha=0.1)
    orc = oracle.OracleStream(cfg, None)
    fr = batch(W, H, 1, 0, 3)
    eng.submit(fr); eng.wait()
    for t in range(3):
        ref = orc.step(fr[t, 0])
        b = eng.plane(PLANE_BLUR, t, 0)
        g = eng.plane(PLANE_GRAY, t, 0)
        bad = np.argwhere(b != ref["blur"])
        print(f"rep {rep} frame {t}: gray bad {int((g != ref['gray']).sum())} blur bad {len(bad)}", bad[:12].tolist())
    eng.close()
