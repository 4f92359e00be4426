#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference (find_motion/find_motion.py) ships no tests, fixtures or sample
videos, and OpenCV -- where its arithmetic lives -- is not
installed here, so these vectors come from the oracle in
oracle/ (C restatement, cross-checked against the numpy restatement and the
analytic known-answer tests of tests/test_oracle_kat.py).  They pin:

* the oracle itself against regressions (tests/test_golden.py, CPU), and
* the HIP path through the C ABI (tests/test_gpu_parity.py::test_golden_*).

Each pixel-chain case stores its INPUT frames (BGR u8, [T][H][W][3]) and keep
mask, the parameters, and per frame the gray / blur / frame_delta / dilated
threshold planes, the external-contour count, bounding boxes and border start
points, plus the final float64 background.  Contour cases store a binary mask
and what findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) returns for it.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from find_motion_amd.synthetic import SyntheticVideo  # noqa: E402

# (name, W, H, box, ksize, T, thresh, alpha, rects (keep-mask zero boxes in work coords))
CHAIN_CASES = [
    ("modeF_k5_masked", 96, 64, 96, 5, 6, 12, 0.1, [(0, 0, 20, 12), (70, 40, 95, 63)]),
    ("modeD_area_general", 230, 130, 100, 5, 4, 12, 0.1, []),
    ("area_fast_2x", 128, 96, 64, 3, 4, 12, 0.1, []),
    ("k21_reflect101", 40, 30, 40, 21, 4, 7, 0.1, [(5, 5, 9, 9)]),
    ("tiny_scalar_tails", 7, 5, 7, 3, 4, 3, 0.25, []),
]


def keep_from_rects(h, w, rects):
    keep = np.ones((h, w), np.uint8)
    for (x0, y0, x1, y1) in rects:
        keep[y0:y1 + 1, x0:x1 + 1] = 0
    return keep


def chain_case(name, W, H, box, k, T, thresh, alpha, rects):
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k, thresh=thresh, alpha=alpha)
    keep = keep_from_rects(cfg.h, cfg.w, rects) if rects else None
    st = oracle.OracleStream(cfg, keep)
    vid = SyntheticVideo(W, H, stream=3, seed=2024)
    frames = vid.frames(90, T)  # frames 94-96 carry the full-frame flash
    out = {k_: [] for k_ in ("gray", "blur", "delta", "mask", "count")}
    boxes, origins = [], []
    for t in range(T):
        r = st.step(frames[t])
        for k_ in ("gray", "blur", "delta", "mask"):
            out[k_].append(r[k_])
        out["count"].append(r["count"])
        boxes.extend([(t,) + b for b in r["boxes"]])
        origins.extend([(t,) + o for o in r["origins"]])
    np.savez_compressed(
        os.path.join(HERE, f"chain_{name}.npz"),
        params=np.array([W, H, box, k, T, thresh], np.int64), alpha=np.float64(alpha),
        frames=frames, keep=keep if keep is not None else np.ones((cfg.h, cfg.w), np.uint8),
        has_keep=np.int64(keep is not None),
        gray=np.stack(out["gray"]), blur=np.stack(out["blur"]), delta=np.stack(out["delta"]),
        mask=np.stack(out["mask"]), count=np.array(out["count"], np.int32),
        boxes=np.array(boxes, np.int32).reshape(-1, 5), origins=np.array(origins, np.int32).reshape(-1, 3),
        bg=st.bg)


def contour_patterns():
    """Binary masks exercising RETR_EXTERNAL (fm.py:269-272): nesting, diagonals, borders."""
    pats = {}
    m = np.zeros((20, 24), np.uint8)
    m[2:18, 2:18] = 255; m[4:16, 4:16] = 0; m[8:12, 8:12] = 255            # blob inside a ring's hole
    pats["ring_with_inner_blob"] = m
    m = np.zeros((10, 10), np.uint8)
    m[3, 3] = m[4, 4] = 255                                                 # 8-connected diagonal
    pats["diagonal_pair"] = m
    m = np.zeros((12, 12), np.uint8)
    m[0:12, 0:6] = 255; m[3:9, 2:4] = 0; m[5, 2] = 255                      # ring touching the border
    pats["border_ring"] = m
    m = np.zeros((16, 16), np.uint8)
    m[1:15, 1:15] = 255; m[2:14, 2:14] = 0; m[3:13, 3:13] = 255; m[4:12, 4:12] = 0; m[6:10, 6:10] = 255
    pats["three_nested"] = m
    m = np.zeros((9, 9), np.uint8)
    m[::2, ::2] = 255                                                        # isolated dots
    pats["dot_lattice"] = m
    m = np.zeros((8, 8), np.uint8)
    m[2:6, 2:6] = 255; m[3:5, 3:5] = 0; m[3, 4] = 255                       # hole 4-split by a diagonal gap
    pats["hole_diag_gap"] = m
    m = np.full((6, 7), 255, np.uint8)                                       # everything foreground
    pats["full"] = m
    pats["empty"] = np.zeros((5, 5), np.uint8)
    rng = np.random.default_rng(11)
    pats["random_35pct"] = ((rng.random((40, 48)) < 0.35) * 255).astype(np.uint8)
    pats["random_dilated"] = oracle.dilate5(((rng.random((48, 40)) < 0.04) * 255).astype(np.uint8))
    return pats


def contour_cases():
    rows = {}
    for name, m in contour_patterns().items():
        cs = oracle.find_contours_ext(m)
        rows[name + "__mask"] = m
        rows[name + "__boxes"] = np.array([c["bbox"] for c in cs], np.int32).reshape(-1, 4)
        rows[name + "__origins"] = np.array([c["origin"] for c in cs], np.int32).reshape(-1, 2)
        rows[name + "__areas"] = np.array([c["area"] for c in cs], np.float64)
    np.savez_compressed(os.path.join(HERE, "contours_external.npz"), **rows)


def main():
    oracle.build()
    for c in CHAIN_CASES:
        chain_case(*c)
    contour_cases()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f"{f:40s} {os.path.getsize(os.path.join(HERE, f)):8d} B")


if __name__ == "__main__":
    main()
