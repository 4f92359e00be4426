"""Deterministic synthetic video: the input of tests and bench.

No video files or decoders are available offline, so streams are generated:
a static per-stream gradient background, U[-3,3] per-pixel noise, four
bouncing filled rectangles, a +-2 level illumination drift over 120 frames
and a 3-frame full-frame flash every 97 frames (frames 94-96 mod 97).  Frames are BGR uint8
HWC C-contiguous, the layout cv2.VideoCapture.read returns (fm.py:501).
Any frame can be generated independently (random access by index).
"""
from __future__ import annotations

import numpy as np


def _bounce(p0: float, v: float, t: int, span: float) -> int:
    if span <= 0:
        return 0
    m = (p0 + v * t) % (2 * span)
    return int(m if m <= span else 2 * span - m)


class SyntheticVideo:
    def __init__(self, width: int, height: int, stream: int = 0, n_objects: int = 4, seed: int = 1000):
        self.W, self.H = int(width), int(height)
        self.stream = int(stream)
        self.seed = int(seed) + self.stream
        rng = np.random.Generator(np.random.PCG64(self.seed))
        off = rng.integers(0, 64)
        gx = np.linspace(0, 120, self.W, dtype=np.float32)[None, :]
        gy = np.linspace(0, 80, self.H, dtype=np.float32)[:, None]
        base = 40 + off + gx + gy
        tint = rng.integers(-20, 21, size=3)
        self.background = np.clip(base[..., None] + tint[None, None, :], 0, 255).astype(np.int16)
        scale = self.W / 1920.0
        self.objects = []
        for _ in range(n_objects):
            ow = max(1, int(rng.uniform(0.05, 0.15) * self.W))
            oh = max(1, int(rng.uniform(0.05, 0.15) * self.W))
            oh = min(oh, self.H)
            col = rng.integers(0, 256, size=3).astype(np.int16)
            x0, y0 = rng.uniform(0, max(1, self.W - ow)), rng.uniform(0, max(1, self.H - oh))
            vx = rng.uniform(2, 8) * scale * rng.choice([-1, 1])
            vy = rng.uniform(2, 8) * scale * rng.choice([-1, 1])
            self.objects.append((ow, oh, col, x0, y0, vx, vy))

    def frame(self, i: int) -> np.ndarray:
        rng = np.random.Generator(np.random.PCG64([self.seed, int(i)]))
        img = self.background.copy()
        drift = int(round(2 * np.sin(2 * np.pi * i / 120.0)))
        img += drift
        if i % 97 >= 94:  # frames 94-96, 191-193, ...: 3-frame flash every 97 frames
            img += 60
        for (ow, oh, col, x0, y0, vx, vy) in self.objects:
            x = _bounce(x0, vx, i, self.W - ow)
            y = _bounce(y0, vy, i, self.H - oh)
            img[y:y + oh, x:x + ow] = col
        img += rng.integers(-3, 4, size=img.shape, dtype=np.int16)
        np.clip(img, 0, 255, out=img)
        return img.astype(np.uint8)

    def frames(self, start: int, n: int) -> np.ndarray:
        return np.stack([self.frame(start + k) for k in range(n)])


def batch(width: int, height: int, n_streams: int, start: int, n: int, seed: int = 1000) -> np.ndarray:
    """[n][n_streams][H][W][3] block of frames, the fm_submit layout."""
    vids = [SyntheticVideo(width, height, s, seed=seed) for s in range(n_streams)]
    out = np.empty((n, n_streams, height, width, 3), np.uint8)
    for t in range(n):
        for s, v in enumerate(vids):
            out[t, s] = v.frame(start + t)
    return out
