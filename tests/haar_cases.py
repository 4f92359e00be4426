"""Synthetic HAAR cascades and ROI images for the object-ROI stage tests.

The reference's cascade files are not available on the GPU box (and no cascade
in them has a detection fixture), so parity runs on generated cascades of the
same format: stage 0 is a centre-surround stump that fires on bright squares,
later stages are random stumps or depth-2 trees over random upright (and,
optionally, tilted) features, with thresholds that pass a fraction of windows.
"""
from __future__ import annotations

import numpy as np

from find_motion_amd.cascade import THRESHOLD_EPS, Cascade


def _rand_rect(rng, W, H, tilted):
    while True:
        if not tilted:
            w, h = int(rng.integers(1, W // 2 + 1)), int(rng.integers(1, H // 2 + 1))
            x, y = int(rng.integers(0, W - w + 1)), int(rng.integers(0, H - h + 1))
            return [x, y, w, h]
        w, h = int(rng.integers(1, W // 3 + 1)), int(rng.integers(1, H // 3 + 1))
        if w + h > H or h > W - w:
            continue
        x = int(rng.integers(h, W - w + 1))
        y = int(rng.integers(0, H - w - h + 1))
        return [x, y, w, h]


def make_cascade(seed=0, win=(20, 20), stages=4, trees=5, depth=1, tilted=False, tight=0.35) -> Cascade:
    rng = np.random.default_rng(seed)
    W, H = win
    rects, wts, tl = [], [], []

    def add_feature(rs, ws, t=0):
        r = np.zeros((3, 4), np.int32)
        w = np.zeros(3, np.float32)
        for j, (a, b) in enumerate(zip(rs, ws)):
            r[j] = a
            w[j] = b
        rects.append(r)
        wts.append(w)
        tl.append(t)
        return len(rects) - 1

    # stage 0: centre-surround on a bright square
    f0 = add_feature([[0, 0, W, H], [W // 4, H // 4, W // 2, H // 2]], [-1.0, 4.0])
    ntrees, sthr, tnodes = [1], [np.float32(np.float32(0.0) - THRESHOLD_EPS)], [1]
    left, right, feat, nthr, leaves = [0], [-1], [f0], [np.float32(0.3)], [np.float32(-1.0), np.float32(1.0)]
    for _ in range(stages - 1):
        lo = hi = 0.0
        for _ in range(trees):
            nn = depth
            fids = []
            for _ in range(nn):
                t = int(tilted and rng.random() < 0.5)
                k = int(rng.integers(2, 4))
                rs = [_rand_rect(rng, W, H, bool(t)) for _ in range(k)]
                ws = [float(np.float32(rng.choice([-1.0, 2.0, 3.0, -2.0]))) for _ in range(k)]
                fids.append(add_feature(rs, ws, t))
            if nn == 1:
                left.append(0)
                right.append(-1)
            else:  # node 0 -> node 1 on the left, leaf on the right
                left += [1, -1]
                right += [0, -2]
            feat += fids
            nthr += [np.float32(rng.normal(0, 0.02)) for _ in range(nn)]
            lv = [np.float32(rng.uniform(-1, 1)) for _ in range(nn + 1)]
            leaves += lv
            tnodes.append(nn)
            lo += float(min(lv))
            hi += float(max(lv))
        ntrees.append(trees)
        sthr.append(np.float32(np.float32(lo + tight * (hi - lo)) - THRESHOLD_EPS))
    return Cascade(W, H, np.asarray(ntrees, np.int32), np.asarray(sthr, np.float32), np.asarray(tnodes, np.int32),
                   np.asarray(left, np.int32), np.asarray(right, np.int32), np.asarray(feat, np.int32),
                   np.asarray(nthr, np.float32), np.asarray(leaves, np.float32), np.stack(rects),
                   np.stack(wts).astype(np.float32), np.asarray(tl, np.uint8))


def make_image(seed=0, w=300, h=169, squares=4, channels=3) -> np.ndarray:
    """Dark noisy background with bright squares (the ROI frame: imutils.resize(raw, width=300))."""
    rng = np.random.default_rng(seed)
    img = rng.integers(30, 46, (h, w), dtype=np.int32)  # sigma < 10: flat windows are rejected
    for _ in range(squares):
        s = int(rng.integers(18, min(h, w) // 2))
        x, y = int(rng.integers(0, w - s)), int(rng.integers(0, h - s))
        img[y:y + s, x:x + s] = rng.integers(190, 206, (s, s))
    img = img.astype(np.uint8)
    if channels == 1:
        return img
    return np.stack([img, np.clip(img.astype(np.int32) + rng.integers(-8, 9, img.shape), 0, 255).astype(np.uint8),
                     img], -1)


def draw_faces(img: np.ndarray, faces, bg: int = 110, noise: int = 6, seed: int = 0) -> np.ndarray:
    """A gray BGR image (H, W, 3) of cartoon frontal faces: (cx, cy, r) each an ellipse of skin tone with
    dark eyes and brows, a light nose bridge and a dark mouth, over a flat background with uniform noise.
    The reference's haarcascade_frontalface_default.xml detects them (tests/golden/make_golden_cascade.py)."""
    H, W = img.shape[:2]
    g = np.full((H, W), bg, np.int16)
    yy, xx = np.mgrid[:H, :W]
    for cx, cy, r in faces:
        g[((xx - cx) / (0.8 * r)) ** 2 + ((yy - cy) / r) ** 2 <= 1] = 175
        for ex in (-0.38, 0.38):
            g[((xx - (cx + ex * r)) / (0.2 * r)) ** 2 + ((yy - (cy - 0.22 * r)) / (0.09 * r)) ** 2 <= 1] = 50
            g[(np.abs(xx - (cx + ex * r)) < 0.25 * r) & (np.abs(yy - (cy - 0.42 * r)) < 0.05 * r)] = 70
        g[(np.abs(xx - cx) < 0.07 * r) & (yy > cy - 0.15 * r) & (yy < cy + 0.2 * r)] = 150
        g[((xx - cx) / (0.32 * r)) ** 2 + ((yy - (cy + 0.45 * r)) / (0.08 * r)) ** 2 <= 1] = 80
    rng = np.random.default_rng(seed)
    g = np.clip(g + rng.integers(-noise, noise + 1, g.shape), 0, 255).astype(np.uint8)
    img[...] = g[..., None]
    return img


# 3840x2160 frames of config 5 (find_motion.py:703-731 resizes them to width 300 for the cascades)
FACE_FRAMES_4K = [
    dict(faces=[(1024, 1024, 576), (2688, 1152, 448)], seed=1),
    dict(faces=[(1900, 1000, 700)], seed=2),
    dict(faces=[(700, 900, 420), (2000, 1100, 420), (3200, 1000, 420)], seed=3),
    dict(faces=[], seed=4),
]


def face_frame_4k(i: int) -> np.ndarray:
    c = FACE_FRAMES_4K[i]
    return draw_faces(np.empty((2160, 3840, 3), np.uint8), c["faces"], seed=c["seed"])


PLATE_SEEDS = [0, 9, 22, 36]


def plate_image(seed: int, w: int = 300, h: int = 169) -> np.ndarray:
    """A ROI-sized frame with three light, dark-framed rectangles holding dark bars (number-plate
    like), for the reference's licence_plate_rus_16stages cascade (64x16 window)."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w, 3), int(rng.integers(60, 140)), np.uint8) + rng.integers(0, 10, (h, w, 3), dtype=np.uint8)
    for _ in range(3):
        pw = int(rng.integers(64, 160))
        ph = max(16, pw * int(rng.integers(20, 30)) // 100)
        x, y = int(rng.integers(0, w - pw)), int(rng.integers(0, h - ph))
        img[y:y + ph, x:x + pw] = int(rng.integers(200, 250))
        b = int(rng.integers(1, 4))
        img[y:y + b, x:x + pw] = 20
        img[y + ph - b:y + ph, x:x + pw] = 20
        img[y:y + ph, x:x + b] = 20
        img[y:y + ph, x + pw - b:x + pw] = 20
        n = int(rng.integers(6, 10))
        cw = pw // (n + 2)
        for k in range(n):
            cx = x + cw + k * cw + int(rng.integers(0, 2))
            img[y + ph // 4:y + ph - ph // 4, cx:cx + max(1, cw * int(rng.integers(40, 70)) // 100)] = int(rng.integers(10, 50))
    return img
