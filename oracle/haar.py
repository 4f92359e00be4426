"""CPU restatement of cv2.CascadeClassifier.detectMultiScale for HAAR cascades.

TEST INFRASTRUCTURE ONLY (the checker for fm_haar_*): only tests/, smoke() and
bench.py's cpu_baseline may import this.  Parity unpinned: OpenCV is not
installed here and the reference holds no detection fixtures; this restates
OpenCV 4.x objdetect/imgproc semantics at the reference's call site
(find_motion.py:722-731: `detectMultiScale(frame.resized, scaleFactor=1.1,
minNeighbors=5)`, flags 0, minSize/maxSize default):

* detectMultiScale -> detectMultiScaleNoGrouping + groupRectangles(eps 0.2)
  (cascadedetect.cpp);
* the scale list: factor *= scaleFactor in double while cvRound(win*factor)
  fits the image, kept as float; min/max object size filter on
  cvRound(win * (float)factor);
* per scale: BGR->gray (fixed point, as oracle_np.bgr2gray), resize to
  (cvRound(W/s), cvRound(H/s)) with INTER_LINEAR_EXACT (resize.cpp
  resize_bitExact: softdouble tap positions, 8-bit fixed-point taps, 16-bit
  horizontal values, (v + 2^15) >> 16), then integral sum / squared sum in
  int32 (wrapping) and, for cascades with tilted features, the tilted sum
  T(X,Y) = sum_{y<Y, |x-X+1| <= Y-y-1} I(x,y);
* windows on a ystep grid (2 below scale 2, else 1), rows limited by the
  invoker's stripes (nstripes = ceil(working width of scale 0 / 32)), a
  window rejected by stage 0 skips the next x position;
* HaarEvaluator::setWindow: norm rect (1,1,W-2,H-2), nf = area*sqsum - sum^2
  in double, window kept only if nf > 0 and area/sqrt(nf) < 0.1 (float
  1/sqrt); feature = (w0*s0 + w1*s1 [+ w2*s2]) * (float)(1/nf) in float32
  without FMA; trees walked with `value < threshold` (double compare), leaves
  summed in double, stage fails if sum < stage threshold;
* candidate rect (cvRound(x*s), cvRound(y*s), cvRound(W*s), cvRound(H*s)) in
  float; groupRectangles: partition by SimilarRects, class mean with
  cvRound(sum * (1.f/n)), keep n > minNeighbors, drop rects inside a
  stronger class.
"""
from __future__ import annotations

import math

import numpy as np

from .oracle_np import bgr2gray


def _rne(x) -> int:
    """cvRound: round half to even (lrint / lrintf under the default rounding mode)."""
    return int(np.rint(x))


# ----------------------------------------------------------------------------- scales
def scale_list(img_w, img_h, win_w, win_h, scale_factor=1.1, min_size=(0, 0), max_size=(0, 0)):
    """cascadedetect.cpp detectMultiScaleNoGrouping: the float scales kept."""
    if max_size[0] == 0 or max_size[1] == 0:
        max_size = (img_w, img_h)
    if img_h < win_h or img_w < win_w:
        return []
    allsc = []
    factor = 1.0
    while True:
        ww, wh = _rne(win_w * factor), _rne(win_h * factor)
        if ww > img_w or wh > img_h:
            break
        allsc.append(np.float32(factor))
        factor *= scale_factor
    out = []
    for s in allsc:
        ww, wh = _rne(np.float32(win_w) * s), _rne(np.float32(win_h) * s)
        if ww > max_size[0] or wh > max_size[1]:
            break
        if ww < min_size[0] or wh < min_size[1]:
            continue
        out.append(s)
    return out


def scale_geometry(img_w, img_h, win_w, win_h, scales):
    """Per scale: resized size, ystep, working size, row limit (stripes)."""
    geo = []
    for s in scales:
        sw, sh = _rne(np.float32(img_w) / s), _rne(np.float32(img_h) / s)
        ystep = 1 if s >= np.float32(2) else 2
        geo.append(dict(scale=s, sw=sw, sh=sh, ystep=ystep,
                        ww=max(sw + 1 - win_w, 0), wh=max(sh + 1 - win_h, 0)))
    if geo:
        nstripes = math.ceil(geo[0]["ww"] / 32.0)
        for g in geo:
            stripe = max((g["wh"] // g["ystep"] + nstripes - 1) // nstripes, 1) * g["ystep"] if nstripes else 0
            g["ylim"] = min(nstripes * stripe, g["wh"])
    return geo


# ----------------------------------------------------------------------------- resize
def linear_exact_tab(ssize: int, dsize: int):
    """interpolationLinear<uint8_t> (resize.cpp): per dst index the source offset and
    the 8-bit fixed-point taps; indices < lo take src[0], >= hi take src[ssize-1]."""
    inv = dsize / ssize
    scale = 1.0 / inv
    ofs = np.zeros(dsize, np.int64)
    c1 = np.zeros(dsize, np.int64)
    lo, hi = 0, dsize
    for d in range(dsize):
        f = scale * (d + 0.5) - 0.5
        i = math.floor(f)
        if i >= 0 and ssize > 1:
            if i < ssize - 1:
                ofs[d] = i
                c1[d] = _rne((f - i) * 256.0)
            else:
                ofs[d] = ssize - 1
                hi = min(hi, d)
        else:
            lo = max(lo, d + 1)
    return ofs, c1, lo, hi


def resize_linear_exact(g: np.ndarray, dw: int, dh: int) -> np.ndarray:
    sh, sw = g.shape
    if (sw, sh) == (dw, dh):
        return g.copy()
    xo, xc, xlo, xhi = linear_exact_tab(sw, dw)
    yo, yc, ylo, yhi = linear_exact_tab(sh, dh)
    src = g.astype(np.int64)
    # horizontal: 16-bit fixed point (8 fractional bits)
    hl = np.empty((sh, dw), np.int64)
    xs = np.arange(dw)
    mid = (xs >= xlo) & (xs < xhi)
    hl[:, mid] = src[:, xo[mid]] * (256 - xc[mid]) + src[:, np.minimum(xo[mid] + 1, sw - 1)] * xc[mid]
    hl[:, xs < xlo] = src[:, :1] * 256
    if xhi < dw:
        hl[:, xs >= xhi] = src[:, xo[dw - 1]:xo[dw - 1] + 1] * 256
    out = np.empty((dh, dw), np.uint8)
    for d in range(dh):
        if d < ylo:
            out[d] = (hl[0] + 128) >> 8
        elif d >= yhi:
            out[d] = (hl[sh - 1] + 128) >> 8
        else:
            v = hl[yo[d]] * (256 - yc[d]) + hl[yo[d] + 1] * yc[d]
            out[d] = np.minimum((v + (1 << 15)) >> 16, 255)
    return out


# ----------------------------------------------------------------------------- integrals
def integrals(img: np.ndarray, tilted: bool):
    """cv::integral(img, sum, sqsum[, tilted], CV_32S, CV_32S): (h+1, w+1) int32 (wrapping)."""
    h, w = img.shape
    v = img.astype(np.int64)
    s = np.zeros((h + 1, w + 1), np.int64)
    q = np.zeros((h + 1, w + 1), np.int64)
    s[1:, 1:] = v.cumsum(0).cumsum(1)
    q[1:, 1:] = (v * v).cumsum(0).cumsum(1)
    wrap = lambda a: ((a + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int32)  # noqa: E731
    t = None
    if tilted:
        # T(X,Y) = sum_{y<Y} rowprefix(y, min(w, X+Y-1-y)) - rowprefix(y, max(0, X-Y+y))
        rp = np.zeros((h, w + 1), np.int64)
        rp[:, 1:] = v.cumsum(1)
        t = np.zeros((h + 1, w + 1), np.int64)
        X = np.arange(w + 1)[None, :]
        for Y in range(1, h + 1):
            ys = np.arange(Y)[:, None]
            hi_ = np.clip(X + Y - 1 - ys, 0, w)
            lo_ = np.clip(X - Y + ys, 0, w)
            t[Y] = np.where(hi_ > lo_, rp[ys, hi_] - rp[ys, lo_], 0).sum(0)
        t = wrap(t)
    return wrap(s), wrap(q), t


# ----------------------------------------------------------------------------- evaluation
def _rect_sum(I, x, y, r, tilted):
    """CALC_SUM_OFS with CV_SUM_OFS / CV_TILTED_OFS corners, int32 wrapping; x, y arrays."""
    rx, ry, rw, rh = (int(v) for v in r)
    if not tilted:
        p0 = I[y + ry, x + rx]
        p1 = I[y + ry, x + rx + rw]
        p2 = I[y + ry + rh, x + rx]
        p3 = I[y + ry + rh, x + rx + rw]
    else:
        p0 = I[y + ry, x + rx]
        p1 = I[y + ry + rh, x + rx - rh]
        p2 = I[y + ry + rw, x + rx + rw]
        p3 = I[y + ry + rw + rh, x + rx + rw - rh]
    with np.errstate(over="ignore"):
        return (p0.astype(np.int32) - p1 - p2 + p3).astype(np.int32)


def eval_windows(cs, S, Q, T, xs, ys):
    """Result per window: 1 accepted, 0 rejected by stage 0, -k rejected by stage k,
    -1 also for a flat window (setWindow false)."""
    W, H = cs.win_w, cs.win_h
    n = len(xs)
    area = float((W - 2) * (H - 2))
    nr = (1, 1, W - 2, H - 2)
    vs = _rect_sum(S, xs, ys, nr, False).astype(np.int64)
    vq = _rect_sum(Q, xs, ys, nr, False).astype(np.int64) & 0xFFFFFFFF  # (unsigned)
    nf = area * vq.astype(np.float64) - vs.astype(np.float64) * vs.astype(np.float64)
    ok = nf > 0
    vnf = np.ones(n, np.float32)
    vnf[ok] = (1.0 / np.sqrt(nf[ok])).astype(np.float32)
    ok &= area * vnf.astype(np.float64) < 1e-1
    res = np.full(n, -1, np.int64)
    alive = np.nonzero(ok)[0]
    fcache = {}

    def fval(fi, idx):
        key = (fi,)
        if key not in fcache:
            tl = bool(cs.feat_tilted[fi])
            I = T if tl else S
            acc = None
            for j in range(3):
                wj = cs.feat_weights[fi, j]
                if j == 2 and wj == 0:
                    continue
                sj = _rect_sum(I, xs, ys, cs.feat_rects[fi, j], tl).astype(np.float32)
                term = (np.float32(wj) * sj).astype(np.float32)
                acc = term if acc is None else (acc + term).astype(np.float32)
            fcache[key] = (acc * vnf).astype(np.float32)
        return fcache[key][idx]

    ti = ni = li = 0
    for si in range(cs.n_stages):
        tot = np.zeros(len(alive), np.float64)
        for _ in range(int(cs.stage_ntrees[si])):
            nn = int(cs.tree_nodes[ti])
            idx = np.zeros(len(alive), np.int64)
            cur = np.ones(len(alive), bool)
            while cur.any():
                k = np.nonzero(cur)[0]
                nd = ni + idx[k]
                nxt = np.empty(len(k), np.int64)
                for u in np.unique(nd):
                    m = nd == u
                    val = fval(int(cs.node_feature[u]), alive[k[m]]).astype(np.float64)
                    nxt[m] = np.where(val < np.float64(cs.node_threshold[u]), cs.node_left[u], cs.node_right[u])
                idx[k] = nxt
                cur[k] = nxt > 0
            tot += cs.leaves[li - idx].astype(np.float64)
            ti += 1
            ni += nn
            li += nn + 1
        fail = tot < np.float64(cs.stage_threshold[si])
        res[alive[fail]] = -si
        alive = alive[~fail]
        if len(alive) == 0:
            # advance the tree/node/leaf cursors is not needed any more
            break
    res[alive] = 1
    return res


def detect_candidates(cs, bgr: np.ndarray, scale_factor=1.1, min_size=(0, 0), max_size=(0, 0)):
    """detectMultiScaleNoGrouping: candidate rects in scale, row, column order."""
    g = bgr2gray(bgr) if bgr.ndim == 3 else bgr
    h, w = g.shape
    scales = scale_list(w, h, cs.win_w, cs.win_h, scale_factor, min_size, max_size)
    cands = []
    for geo in scale_geometry(w, h, cs.win_w, cs.win_h, scales):
        if geo["ww"] == 0 or geo["ylim"] <= 0:
            continue
        img = resize_linear_exact(g, geo["sw"], geo["sh"])
        S, Q, T = integrals(img, cs.has_tilted)
        st = geo["ystep"]
        gy, gx = np.meshgrid(np.arange(0, geo["ylim"], st), np.arange(0, geo["ww"], st), indexing="ij")
        res = eval_windows(cs, S, Q, T, gx.ravel(), gy.ravel()).reshape(gy.shape)
        s = geo["scale"]
        wsz = (_rne(np.float32(cs.win_w) * s), _rne(np.float32(cs.win_h) * s))
        for r in range(gy.shape[0]):
            c = 0
            while c < gy.shape[1]:
                v = res[r, c]
                if v > 0:
                    cands.append((_rne(np.float32(gx[r, c]) * s), _rne(np.float32(gy[r, c]) * s), wsz[0], wsz[1]))
                c += 2 if v == 0 else 1
    return cands


def _similar(a, b, eps):
    delta = eps * (min(a[2], b[2]) + min(a[3], b[3])) * 0.5
    return (abs(a[0] - b[0]) <= delta and abs(a[1] - b[1]) <= delta and
            abs(a[0] + a[2] - b[0] - b[2]) <= delta and abs(a[1] + a[3] - b[1] - b[3]) <= delta)


def partition(rects, eps):
    """cv::partition with SimilarRects: class labels numbered by first appearance."""
    n = len(rects)
    parent = [-1] * n
    rank = [0] * n

    def root(i):
        while parent[i] >= 0:
            i = parent[i]
        return i

    R = np.asarray(rects, np.int64).reshape(-1, 4)
    for i in range(n):
        r = root(i)
        # SimilarRects of i against every j (vectorised; the merge loop below stays sequential)
        delta = eps * (np.minimum(R[i, 2], R[:, 2]) + np.minimum(R[i, 3], R[:, 3])) * 0.5
        sim = ((np.abs(R[i, 0] - R[:, 0]) <= delta) & (np.abs(R[i, 1] - R[:, 1]) <= delta) &
               (np.abs(R[i, 0] + R[i, 2] - R[:, 0] - R[:, 2]) <= delta) &
               (np.abs(R[i, 1] + R[i, 3] - R[:, 1] - R[:, 3]) <= delta))
        sim[i] = False
        for j in np.nonzero(sim)[0].tolist():
            r2 = root(j)
            if r2 != r:
                if rank[r] > rank[r2]:
                    parent[r2] = r
                else:
                    parent[r] = r2
                    rank[r2] += rank[r] == rank[r2]
                    r = r2
                k = j
                while parent[k] >= 0:
                    p = parent[k]
                    parent[k] = r
                    k = p
                k = i
                while parent[k] >= 0:
                    p = parent[k]
                    parent[k] = r
                    k = p
    labels, ncls = [0] * n, 0
    lab = {}
    for i in range(n):
        r = root(i)
        if r not in lab:
            lab[r] = ncls
            ncls += 1
        labels[i] = lab[r]
    return labels, ncls


def group_rectangles(rects, group_threshold, eps=0.2):
    if group_threshold <= 0 or not rects:
        return list(rects)
    labels, ncls = partition(rects, eps)
    acc = [[0, 0, 0, 0] for _ in range(ncls)]
    cnt = [0] * ncls
    for r, l in zip(rects, labels):
        for k in range(4):
            acc[l][k] += r[k]
        cnt[l] += 1
    avg = []
    for l in range(ncls):
        s = np.float32(1.0) / np.float32(cnt[l])
        avg.append(tuple(_rne(np.float32(np.float32(acc[l][k]) * s)) for k in range(4)))
    out = []
    for i in range(ncls):
        r1, n1 = avg[i], cnt[i]
        if n1 <= group_threshold:
            continue
        inside = False
        for j in range(ncls):
            n2 = cnt[j]
            if j == i or n2 <= group_threshold:
                continue
            r2 = avg[j]
            dx, dy = _rne(r2[2] * eps), _rne(r2[3] * eps)
            if (r1[0] >= r2[0] - dx and r1[1] >= r2[1] - dy and r1[0] + r1[2] <= r2[0] + r2[2] + dx and
                    r1[1] + r1[3] <= r2[1] + r2[3] + dy and (n2 > max(3, n1) or n1 < 3)):
                inside = True
                break
        if not inside:
            out.append(r1)
    return out


def detect_multiscale(cs, bgr, scale_factor=1.1, min_neighbors=5, min_size=(0, 0), max_size=(0, 0)):
    return group_rectangles(detect_candidates(cs, bgr, scale_factor, min_size, max_size), min_neighbors, 0.2)
