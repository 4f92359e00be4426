#!/usr/bin/env python3
"""Contour-pass workload of the bench ring (CPU, oracle): per frame the candidate
tiles (64x64 tiles whose dilated mask is non-empty), runs per candidate, components.
Diagnostic only (uses oracle/, test infrastructure)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as O
from find_motion_amd.synthetic import SyntheticVideo

W, H, k, T, A = 1920, 1080, 5, 12, 0.1
ring = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 2
v = SyntheticVideo(W, H, 0)
frames = [v.frame(i) for i in range(ring)]
bg = None
tot_c, tot_r = [], []
for n in range(ring * cycles):
    fr = frames[n % ring]
    blur = O.gauss_blur(O.bgr2gray(fr), k)
    if bg is None:
        bg = blur.astype(np.float64)
    _, th = O.diff_thresh(blur, bg, T)
    O.accumulate(blur, bg, A)
    m = O.dilate5(th) > 0
    nty, ntx = (H + 63) // 64, (W + 63) // 64
    mp = np.zeros((nty * 64, ntx * 64), bool)
    mp[:H, :W] = m
    t = mp.reshape(nty, 64, ntx, 64).transpose(0, 2, 1, 3)
    cand = t.any(axis=(2, 3))
    starts = np.zeros_like(t)
    starts[..., 0] = True
    starts[..., 1:] = t[..., 1:] != t[..., :-1]
    runs = starts.sum(axis=(2, 3))[cand]
    full = t.all(axis=(2, 3)).sum()
    tot_c.append(cand.sum()); tot_r.extend(runs.tolist())
    if n % 8 == 0 or n % ring == 0:
        print(f"frame {n:4d}: candidates {cand.sum():4d} full {full:4d} runs/cand mean {runs.mean() if len(runs) else 0:7.1f} max {runs.max() if len(runs) else 0}")
print("mean candidates/frame", np.mean(tot_c[ring:]) if cycles > 1 else np.mean(tot_c), "mean runs/cand", np.mean(tot_r))
