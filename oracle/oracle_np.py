"""Independent numpy/scipy restatement of the motion chain.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Written separately from
fm_oracle.c so the two restatements check each other:

* pixel ops are vectorised numpy, following the same OpenCV 4.x semantics;
* external contours use the *topological* definition (8-connected foreground
  components whose outer border faces the 4-connected background region that
  touches the 1-px zero pad) via scipy.ndimage.label, instead of the literal
  Suzuki-Abe scan in fm_oracle.c.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage


def reflect101_index(n: int, lo: int, hi: int) -> np.ndarray:
    """OpenCV borderInterpolate(BORDER_REFLECT_101) for indices lo..hi-1."""
    idx = np.arange(lo, hi)
    if n == 1:
        return np.zeros_like(idx)
    period = 2 * (n - 1)
    m = np.mod(idx, period)
    return np.where(m < n, m, period - m)


def area_tab(ssize: int, dsize: int):
    """computeResizeAreaTab restated: per destination index, (src idx, weight f32) in order."""
    inv = dsize / ssize
    scale = 1.0 / inv
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cw = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        ent = []
        if sx1 - fsx1 > 1e-3:
            ent.append((sx1 - 1, np.float32((sx1 - fsx1) / cw)))
        for sx in range(sx1, sx2):
            ent.append((sx, np.float32(1.0 / cw)))
        if fsx2 - sx2 > 1e-3:
            ent.append((sx2, np.float32(min(min(fsx2 - sx2, 1.0), cw) / cw)))
        tab.append(ent)
    return tab


def resize_area_bgr(src: np.ndarray, w: int) -> np.ndarray:
    H, W, cn = src.shape
    h = int(H * (w / float(W)))
    if (h, w) == (H, W):
        return src.copy()
    sx, sy = 1.0 / (w / W), 1.0 / (h / H)
    assert sx >= 1 and sy >= 1
    isx, isy = int(round(sx)), int(round(sy))
    if abs(sx - isx) < np.finfo(float).eps and abs(sy - isy) < np.finfo(float).eps:
        blk = src[: h * isy, : w * isx].reshape(h, isy, w, isx, cn).astype(np.int64).sum(axis=(1, 3))
        if isx == 2 and isy == 2:
            return ((blk + 2) >> 2).astype(np.uint8)
        v = np.rint(blk.astype(np.float32) * np.float32(1.0 / np.float32(isx * isy)))
        return np.clip(v, 0, 255).astype(np.uint8)
    xt, yt = area_tab(W, w), area_tab(H, h)
    nmax = max(len(e) for e in xt)
    # pad each destination's entry list with zero-weight taps (x + 0.0f == x)
    xi = np.zeros((w, nmax), np.int64)
    xa = np.zeros((w, nmax), np.float32)
    for d, ent in enumerate(xt):
        for k, (s, a) in enumerate(ent):
            xi[d, k], xa[d, k] = s, a
    out = np.empty((h, w, cn), np.uint8)
    for dy, ent in enumerate(yt):
        acc = None
        for (s_row, beta) in ent:
            row = src[s_row].astype(np.float32)  # (W, cn)
            buf = np.zeros((w, cn), np.float32)
            for k in range(nmax):
                buf = buf + row[xi[:, k]] * xa[:, k : k + 1]
            term = np.float32(beta) * buf
            acc = term if acc is None else acc + term
        out[dy] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    return out


def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    b, g, r = (bgr[..., i].astype(np.int32) for i in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def fma(a: float, b: float, c: float) -> float:
    """a * b + c rounded once, as C's fma (fm_oracle.c, OpenCV's mulAdd): math.fma where Python has it (3.13+),
    else the exact rational result rounded to the nearest double (float(Fraction) rounds correctly)."""
    if hasattr(math, "fma"):
        return math.fma(a, b, c)
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def gauss_coeffs(k: int) -> np.ndarray:
    tables = {
        1: [1.0],
        3: [0.25, 0.5, 0.25],
        5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
        7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125],
        9: [v / 256.0 for v in (4, 13, 30, 51, 60, 51, 30, 13, 4)],
    }
    if k in tables:
        kd = tables[k]
    else:
        sigma = fma(k, 0.15, 0.35)
        s2 = -0.125 / (sigma * sigma)
        n2 = (k - 1) // 2
        vals = [math.exp(float(x * x) * s2) for x in range(1 - k, 1 - k + 2 * n2, 2)]
        tot = 0.0
        for v in vals:
            tot += v
        tot = tot * 2.0 + 1.0
        kd = [v / tot for v in vals] + [1.0 / tot] + [v / tot for v in vals[::-1]]
    n2 = k // 2
    out = [0] * k
    err, s = 0.0, 0
    for i in range(n2):
        adj = kd[i] * 256.0 + err
        v0 = round(adj)  # Python round: half to even == cvRound
        err = adj - v0
        out[i] = out[k - 1 - i] = v0
        s += v0
    out[n2] = 256 - 2 * s
    return np.array(out, np.int64)


def gauss_blur(gray: np.ndarray, k: int) -> np.ndarray:
    h, w = gray.shape
    kx = 1 if w == 1 else k
    ky = 1 if h == 1 else k
    cx, cy = gauss_coeffs(kx), gauss_coeffs(ky)
    rx, ry = kx // 2, ky // 2
    g = gray.astype(np.int64)
    xs = reflect101_index(w, -rx, w + rx)
    gp = g[:, xs]
    H = sum(cx[i] * gp[:, i : i + w] for i in range(kx))
    ys = reflect101_index(h, -ry, h + ry)
    Hp = H[ys, :]
    V = sum(cy[i] * Hp[i : i + h, :] for i in range(ky))
    return ((V + 32768) >> 16).astype(np.uint8)


def diff_thresh(blur: np.ndarray, bg: np.ndarray, t: int):
    if bg.size >= 16:
        q = np.rint(np.abs(bg.astype(np.float32))).astype(np.int32)
    else:
        q = np.rint(np.abs(bg)).astype(np.int32)
    q = np.clip(q, 0, 255)
    delta = np.abs(blur.astype(np.int32) - q).astype(np.uint8)
    return delta, np.where(delta > t, 255, 0).astype(np.uint8)


def accumulate_nofma(blur: np.ndarray, bg: np.ndarray, alpha: float) -> np.ndarray:
    """accumulateWeighted without fusing (equal to the fused form within 1 ulp)."""
    return blur.astype(np.float64) * alpha + bg * (1.0 - alpha)


def dilate5(th: np.ndarray) -> np.ndarray:
    return ndimage.maximum_filter(th, size=5, mode="constant", cval=0)


def external_components(mask: np.ndarray):
    """Topological RETR_EXTERNAL: list of (origin(x,y), bbox(x,y,w,h)) sorted by origin raster order."""
    h, w = mask.shape
    fg = np.zeros((h + 2, w + 2), bool)
    fg[1:-1, 1:-1] = mask != 0
    flab, nf = ndimage.label(fg, structure=np.ones((3, 3), int))
    blab, _ = ndimage.label(~fg, structure=np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]]))
    outer = blab[0, 0]
    out = []
    if nf == 0:
        return out
    # raster-first pixel of each fg component
    flat = flab.ravel()
    idx = np.flatnonzero(flat)
    labs = flat[idx]
    first = np.full(nf + 1, -1, np.int64)
    order = np.argsort(labs, kind="stable")
    ls, ids = labs[order], idx[order]
    starts = np.r_[0, np.flatnonzero(np.diff(ls)) + 1]
    first[ls[starts]] = ids[starts]
    objs = ndimage.find_objects(flab)
    for lab in range(1, nf + 1):
        p = first[lab]
        y, x = divmod(int(p), w + 2)
        if blab[y, x - 1] != outer:
            continue
        sl = objs[lab - 1]
        out.append(((x - 1, y - 1), (sl[1].start - 1, sl[0].start - 1,
                                       sl[1].stop - sl[1].start, sl[0].stop - sl[0].start)))
    out.sort(key=lambda t: (t[0][1], t[0][0]))
    return out
