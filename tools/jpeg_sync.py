#!/usr/bin/env python3
"""How fast does a JPEG Huffman decode started at a random bit, in state (block 0 of the MCU,
coefficient 0), fall into step with the true decode?  This sets k_jpeg_huff's speculation length
(fm_jpeg.hip).  CPU only (oracle/jpeg.py's tables); the state compared is
(bit position, block of the MCU, coefficient index) at symbol boundaries.

Usage: tools/jpeg_sync.py [width height quality subsampling noise_sigma trials]
"""
import io
import os
import sys

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from find_motion_amd.synthetic import SyntheticVideo  # noqa: E402
from oracle import jpeg as oj  # noqa: E402

W, H, Q, SUB, SIGMA, TRIALS = (int(a) for a in (sys.argv[1:] + ["1920", "1080", "75", "2", "0", "300"][len(sys.argv) - 1:]))
f = SyntheticVideo(W, H, 0).frame(37).astype(np.float32)
f = np.clip(f + np.random.default_rng(1).normal(0, SIGMA, f.shape), 0, 255).astype(np.uint8)
b = io.BytesIO()
Image.fromarray(np.ascontiguousarray(f[..., ::-1])).save(b, "JPEG", quality=Q, subsampling=SUB)
j = oj.parse(b.getvalue())
seg = j["scan"]["data"]
u8 = bytearray()
i = 0
while i < len(seg):  # stuffing removed (no restart markers in these frames)
    u8.append(seg[i])
    i += 2 if seg[i] == 0xFF else 1
bits = np.unpackbits(np.frombuffer(bytes(u8) + b"\0" * 8, np.uint8))
nbits = len(u8) * 8
comps = j["frame"]["comps"]
sel = {cid: (td, ta) for cid, td, ta in j["scan"]["sel"]}
tabs = [(oj.huff_lookup(*j["ht"][(0, sel[c["id"]][0])]), oj.huff_lookup(*j["ht"][(1, sel[c["id"]][1])])) for c in comps]
ucomp = [ci for ci, c in enumerate(comps) for _ in range(c["h"] * c["v"])]
bpm = len(ucomp)


def huff(p, tab):
    code = 0
    for ln in range(1, 17):
        code = (code << 1) | int(bits[p + ln - 1])
        if (ln, code) in tab:
            return tab[(ln, code)], p + ln
    return 0, p + 16


def step(p, u, k):
    ci = ucomp[u]
    if k == 0:
        s, p = huff(p, tabs[ci][0])
        p += s
        k = 1
    else:
        rs, p = huff(p, tabs[ci][1])
        r, s = rs >> 4, rs & 15
        if s:
            k += r + 1
            p += s
        elif r == 15:
            k += 16
        else:
            k = 64
    if k >= 64:
        k, u = 0, (u + 1) % bpm
    return p, u, k


truth = {}
p, u, k, nsym = 0, 0, 0, 0
while p < nbits - 8:
    truth[p] = (u, k)
    p, u, k = step(p, u, k)
    nsym += 1
rng = np.random.default_rng(0)
dist = []
for _ in range(TRIALS):
    p0 = int(rng.integers(0, max(1, nbits - 20000)))
    p, u, k = p0, 0, 0
    while truth.get(p) != (u, k) and p - p0 < 200000:
        p, u, k = step(p, u, k)
    dist.append(p - p0)
d = np.array(dist)
print({"bytes": len(u8), "symbols": nsym, "bits_per_symbol": round(nbits / nsym, 2),
       "in_step_within": {ov: round(float((d <= ov).mean()), 3) for ov in (256, 512, 1024, 2048, 4096)},
       "median_bits": float(np.median(d)), "p99_bits": float(np.percentile(d, 99)), "max_bits": int(d.max())})
