"""CPU restatement of the decode side for MJPEG frames -- TEST INFRASTRUCTURE.

What the reference calls: cv2.VideoCapture.read (fm.py:413, 497-506) on an MJPEG stream, i.e. one
baseline JPEG per frame decoded by libjpeg(-turbo) with its defaults (JDCT_ISLOW integer IDCT,
fancy upsampling, integer YCbCr->RGB tables) and returned as BGR u8 HWC.  libjpeg-turbo is not the
reference and OpenCV is absent here; Pillow (which bundles libjpeg-turbo) IS importable, so this
restatement -- and the GPU decoder -- are pinned bit for bit against Pillow's decode of the same
bytes (tests/test_jpeg_host.py, tests/test_gpu_jpeg.py).  Algorithms restated (libjpeg-turbo
sources, not present in this image, cited by file): jdhuff.c (Huffman + DC prediction + restart
intervals), jidctint.c (jpeg_idct_islow, CONST_BITS 13 / PASS1_BITS 2, zero-column and zero-row
shortcuts), jdmaster.c (prepare_range_limit_table), jdsample.c (h2v1/h2v2_fancy_upsample),
jdmainct.c (edge-replicated context rows), jdcolor.c (build_ycc_rgb_table / ycc_rgb_convert).

Pure Python/numpy, for small images only.  Nothing in the product imports this module.
"""
from __future__ import annotations

import numpy as np

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
                   6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38,
                   31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], np.int32)  # zigzag index -> natural index


class JpegError(ValueError):
    pass


def parse(data: bytes) -> dict:
    """Markers of one baseline JPEG: quant tables (natural order), Huffman tables, frame, scan, DRI and
    the entropy-coded segment (bytes between the SOS header and EOI, restart markers included)."""
    if data[:2] != b"\xff\xd8":
        raise JpegError("no SOI")
    qt, ht, frame, scan, dri = {}, {}, None, None, 0
    i = 2
    while i < len(data):
        if data[i] != 0xFF:
            raise JpegError(f"marker expected at {i}")
        while data[i] == 0xFF:
            i += 1
        m = data[i]
        i += 1
        if m == 0xD9:
            break
        ln = (data[i] << 8) | data[i + 1]
        seg = data[i + 2:i + ln]
        if m == 0xDB:  # DQT
            p = 0
            while p < len(seg):
                pq, tq = seg[p] >> 4, seg[p] & 15
                p += 1
                if pq:
                    v = np.frombuffer(seg[p:p + 128], ">u2").astype(np.int32)
                    p += 128
                else:
                    v = np.frombuffer(seg[p:p + 64], np.uint8).astype(np.int32)
                    p += 64
                nat = np.zeros(64, np.int32)
                nat[ZIGZAG] = v
                qt[tq] = nat
        elif m == 0xC4:  # DHT
            p = 0
            while p < len(seg):
                tc, th = seg[p] >> 4, seg[p] & 15
                bits = list(seg[p + 1:p + 17])
                n = sum(bits)
                vals = list(seg[p + 17:p + 17 + n])
                ht[(tc, th)] = (bits, vals)
                p += 17 + n
        elif m == 0xC0 or m == 0xC1:  # SOF0 / SOF1 (baseline / extended sequential Huffman)
            if seg[0] != 8:
                raise JpegError("only 8-bit samples")
            H, W, nc = (seg[1] << 8) | seg[2], (seg[3] << 8) | seg[4], seg[5]
            comps = []
            for c in range(nc):
                cid, hv, tq = seg[6 + 3 * c], seg[7 + 3 * c], seg[8 + 3 * c]
                comps.append({"id": cid, "h": hv >> 4, "v": hv & 15, "tq": tq})
            frame = {"H": H, "W": W, "comps": comps}
        elif m in (0xC2, 0xC3, 0xC5, 0xC6, 0xC7, 0xC9, 0xCA, 0xCB, 0xCD, 0xCE, 0xCF):
            raise JpegError(f"unsupported SOF {m:#x} (progressive / lossless / arithmetic)")
        elif m == 0xDD:  # DRI
            dri = (seg[0] << 8) | seg[1]
        elif m == 0xDA:  # SOS: the entropy-coded data follows the header
            ns = seg[0]
            sel = [(seg[1 + 2 * k], seg[2 + 2 * k] >> 4, seg[2 + 2 * k] & 15) for k in range(ns)]
            scan = {"sel": sel}
            j = i + ln
            k = j
            # the scan ends at the first marker that is neither FF 00 nor RSTn; a run of 0xFF fill bytes
            # may precede any marker (T.81 B.1.1.2; libjpeg's next_marker skips them)
            while k < len(data):
                if data[k] != 0xFF:
                    k += 1
                    continue
                q = k + 1
                while q < len(data) and data[q] == 0xFF:
                    q += 1
                if q < len(data) and (data[q] == 0 or 0xD0 <= data[q] <= 0xD7):
                    k = q + 1
                    continue
                break
            scan["data"] = data[j:k]
            i = k
            continue
        i += ln
    if frame is None or scan is None:
        raise JpegError("no frame or scan")
    if len(scan["sel"]) != len(frame["comps"]):
        raise JpegError("multi-scan (non-interleaved) JPEG not supported")
    for key, tab in STD_HUFF.items():  # jstdhuff.c std_huff_tables: slots 0 and 1 the stream left undefined
        ht.setdefault(key, tab)
    return {"qt": qt, "ht": ht, "frame": frame, "scan": scan, "dri": dri}


def _std_ac(bits: list[int], head: list[int]) -> tuple:
    """An Annex K AC table: its irregular head, then every other (run, size) symbol, size 1..10, in order."""
    tail = [rs for rs in range(256) if 1 <= (rs & 15) <= 10 and rs not in head]
    return bits, head + tail


# T.81 Annex K.3 (libjpeg-turbo jstdhuff.c): what MJPEG frames without a DHT segment are decoded with
STD_HUFF = {
    (0, 0): ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12))),
    (0, 1): ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12))),
    (1, 0): _std_ac([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d],
                    [0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
                     0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
                     0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16]),
    (1, 1): _std_ac([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77],
                    [0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
                     0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
                     0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1]),
}


def huff_lookup(bits: list[int], vals: list[int]) -> dict:
    """Canonical code table: {(length, code): symbol}."""
    out, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            out[(ln, code)] = vals[k]
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    """MSB-first bit reader over an entropy-coded segment (0xFF00 stuffing removed; at a marker the
    reader returns zeros, as libjpeg's fill_bit_buffer does)."""

    def __init__(self, seg: bytes):
        self.b, self.p, self.acc, self.n = seg, 0, 0, 0

    def _fill(self):
        while self.n <= 24:
            byte = 0
            if self.p < len(self.b):
                byte = self.b[self.p]
                if byte == 0xFF:  # fill_bit_buffer: skip 0xFF fill bytes; FF 00 is a data 0xFF
                    q = self.p + 1
                    while q < len(self.b) and self.b[q] == 0xFF:
                        q += 1
                    if q < len(self.b) and self.b[q] == 0:
                        self.p = q + 1
                    else:  # a marker: feed zeros, do not consume it
                        byte = 0
                else:
                    self.p += 1
            self.acc = (self.acc << 8) | byte
            self.n += 8

    def get(self, k: int) -> int:
        if k == 0:
            return 0
        self._fill()
        v = (self.acc >> (self.n - k)) & ((1 << k) - 1)
        self.n -= k
        return v

    def huff(self, tab: dict) -> int:
        code = 0
        for ln in range(1, 17):
            code = (code << 1) | self.get(1)
            if (ln, code) in tab:
                return tab[(ln, code)]
        raise JpegError("bad Huffman code")

    def restart(self):
        """Discard the partial byte and skip the RSTn marker (jdhuff.c process_restart)."""
        self.acc, self.n = 0, 0
        while self.p < len(self.b) - 1 and not (self.b[self.p] == 0xFF and 0xD0 <= self.b[self.p + 1] <= 0xD7):
            self.p += 1
        if self.p < len(self.b) - 1:
            self.p += 2


def _extend(v: int, s: int) -> int:
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def decode_coefficients(j: dict) -> list[np.ndarray]:
    """Dequantized coefficients (natural order) per component: array [by][bx][64] int32 over the
    MCU-padded block grid, as libjpeg's coefficient buffer holds them."""
    fr = j["frame"]
    comps = fr["comps"]
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    mcux = -(-fr["W"] // (8 * hmax))
    mcuy = -(-fr["H"] // (8 * vmax))
    sel = {cid: (td, ta) for cid, td, ta in j["scan"]["sel"]}
    tabs = []
    out = []
    for c in comps:
        td, ta = sel[c["id"]]
        tabs.append((huff_lookup(*j["ht"][(0, td)]), huff_lookup(*j["ht"][(1, ta)]), j["qt"][c["tq"]]))
        out.append(np.zeros((mcuy * c["v"], mcux * c["h"], 64), np.int32))
    if len(comps) == 1:  # a non-interleaved scan: one block per MCU over the component's own grid
        c = comps[0]
        bw, bh = -(-fr["W"] * c["h"] // (8 * hmax)), -(-fr["H"] * c["v"] // (8 * vmax))
        order = [[(0, by, bx)] for by in range(bh) for bx in range(bw)]
    else:
        order = []
        for my in range(mcuy):
            for mx in range(mcux):
                mcu = []
                for ci, c in enumerate(comps):
                    for v in range(c["v"]):
                        for h in range(c["h"]):
                            mcu.append((ci, my * c["v"] + v, mx * c["h"] + h))
                order.append(mcu)
    br = _Bits(j["scan"]["data"])
    pred = [0] * len(comps)
    dri = j["dri"]
    for n, mcu in enumerate(order):
        if dri and n and n % dri == 0:
            br.restart()
            pred = [0] * len(comps)
        for ci, by, bx in mcu:
            dc_t, ac_t, q = tabs[ci]
            blk = np.zeros(64, np.int32)
            s = br.huff(dc_t)
            pred[ci] += _extend(br.get(s), s)
            blk[0] = pred[ci] * q[0]
            k = 1
            while k < 64:
                rs = br.huff(ac_t)
                r, s = rs >> 4, rs & 15
                if s:
                    k += r
                    z = ZIGZAG[k]
                    blk[z] = _extend(br.get(s), s) * q[z]
                    k += 1
                elif r == 15:
                    k += 16
                else:
                    break
            out[ci][by, bx] = blk
    return out


# jidctint.c constants (CONST_BITS 13)
F0_298, F0_390, F0_541, F0_765 = 2446, 3196, 4433, 6270
F0_899, F1_175, F1_501, F1_847 = 7373, 9633, 12299, 15137
F1_961, F2_053, F2_562, F3_072 = 16069, 16819, 20995, 25172


def _idct_1d(v0, v1, v2, v3, v4, v5, v6, v7):
    """The even/odd butterflies shared by both passes; returns the 8 undescaled sums."""
    z1 = (v2 + v6) * F0_541
    tmp2 = z1 - v6 * F1_847
    tmp3 = z1 + v2 * F0_765
    tmp0 = (v0 + v4) << 13
    tmp1 = (v0 - v4) << 13
    t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    o0, o1, o2, o3 = v7, v5, v3, v1
    z1, z2, z3, z4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
    z5 = (z3 + z4) * F1_175
    o0 *= F0_298
    o1 *= F2_053
    o2 *= F3_072
    o3 *= F1_501
    z1 *= -F0_899
    z2 *= -F2_562
    z3 = z3 * -F1_961 + z5
    z4 = z4 * -F0_390 + z5
    o0 += z1 + z3
    o1 += z2 + z4
    o2 += z2 + z3
    o3 += z1 + z4
    return (t10 + o3, t11 + o2, t12 + o1, t13 + o0, t13 - o0, t12 - o1, t11 - o2, t10 - o3)


def _range_limit_idct(x: int) -> int:
    """IDCT_range_limit(cinfo)[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)."""
    v = x & 1023
    return v + 128 if v < 128 else 255 if v < 512 else 0 if v < 896 else v - 896


def idct_islow(c: np.ndarray) -> np.ndarray:
    """jpeg_idct_islow of one dequantized block (natural order, int) -> 8x8 u8 samples."""
    c = [int(x) for x in c]
    ws = [0] * 64
    for col in range(8):
        if all(c[8 * r + col] == 0 for r in range(1, 8)):
            dc = c[col] << 2
            for r in range(8):
                ws[8 * r + col] = dc
            continue
        o = _idct_1d(*[c[8 * r + col] for r in range(8)])
        for r in range(8):
            ws[8 * r + col] = (o[r] + (1 << 10)) >> 11
    out = np.zeros((8, 8), np.uint8)
    for row in range(8):
        w = ws[8 * row:8 * row + 8]
        if all(x == 0 for x in w[1:]):
            out[row, :] = _range_limit_idct((w[0] + 16) >> 5)
            continue
        o = _idct_1d(*w)
        for k in range(8):
            out[row, k] = _range_limit_idct((o[k] + (1 << 17)) >> 18)
    return out


def _fancy_h2(row: np.ndarray, n: int) -> np.ndarray:
    """h2v1_fancy_upsample of the first n > 2 samples of a row (jdsample.c)."""
    r = row.astype(np.int32)
    out = np.zeros(2 * n, np.int32)
    out[0] = r[0]
    out[1] = (r[0] * 3 + r[1] + 2) >> 2
    for i in range(1, n - 1):
        out[2 * i] = (r[i] * 3 + r[i - 1] + 1) >> 2
        out[2 * i + 1] = (r[i] * 3 + r[i + 1] + 2) >> 2
    out[2 * n - 2] = (r[n - 1] * 3 + r[n - 2] + 1) >> 2
    out[2 * n - 1] = r[n - 1]
    return out.astype(np.uint8)


def _fancy_h2v2(plane: np.ndarray, h: int, n: int) -> np.ndarray:
    """h2v2_fancy_upsample over the first h x n (n > 2) samples of a component: context rows past the
    image repeat its first / last row (jdmainct.c)."""
    p = plane.astype(np.int32)
    out = np.zeros((2 * h, 2 * n), np.int32)
    for y in range(h):
        for v in range(2):
            far = p[max(y - 1, 0)] if v == 0 else p[min(y + 1, h - 1)]
            cs = p[y] * 3 + far
            o = out[2 * y + v]
            o[0] = (cs[0] * 4 + 8) >> 4
            o[1] = (cs[0] * 3 + cs[1] + 7) >> 4
            for i in range(1, n - 1):
                o[2 * i] = (cs[i] * 3 + cs[i - 1] + 8) >> 4
                o[2 * i + 1] = (cs[i] * 3 + cs[i + 1] + 7) >> 4
            o[2 * n - 2] = (cs[n - 1] * 3 + cs[n - 2] + 8) >> 4
            o[2 * n - 1] = (cs[n - 1] * 4 + 7) >> 4
    return out[:, :2 * n].astype(np.uint8)


def _ycc_tables():
    x = np.arange(256, dtype=np.int64) - 128
    fix = lambda v: int(v * 65536 + 0.5)
    cr_r = (fix(1.40200) * x + 32768) >> 16
    cb_b = (fix(1.77200) * x + 32768) >> 16
    cr_g = -fix(0.71414) * x
    cb_g = -fix(0.34414) * x + 32768
    return cr_r, cb_b, cr_g, cb_g


def decode(data: bytes) -> np.ndarray:
    """One JPEG -> BGR u8 (H, W, 3), or (H, W) for a grayscale JPEG."""
    j = parse(data)
    fr = j["frame"]
    H, W = fr["H"], fr["W"]
    comps = fr["comps"]
    coefs = decode_coefficients(j)
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    planes = []
    for c, cf in zip(comps, coefs):
        by, bx = cf.shape[:2]
        pl = np.zeros((by * 8, bx * 8), np.uint8)
        for y in range(by):
            for x in range(bx):
                pl[8 * y:8 * y + 8, 8 * x:8 * x + 8] = idct_islow(cf[y, x])
        dw, dh = -(-W * c["h"] // hmax), -(-H * c["v"] // vmax)
        if (c["h"], c["v"]) == (hmax, vmax):
            up = pl[:dh, :dw]
        elif dw <= 2 and (hmax // c["h"], vmax // c["v"]) in ((2, 1), (2, 2)):
            # jdsample.c jinit_upsampler: fancy upsampling only when downsampled_width > 2, else
            # h2v1_upsample / h2v2_upsample (each sample replicated)
            up = np.repeat(np.repeat(pl[:dh, :dw], vmax // c["v"], axis=0), 2, axis=1)
        elif (hmax // c["h"], vmax // c["v"]) == (2, 1):
            up = np.stack([_fancy_h2(r, dw) for r in pl[:dh]])
        elif (hmax // c["h"], vmax // c["v"]) == (2, 2):
            up = _fancy_h2v2(pl, dh, dw)
        else:
            raise JpegError(f"sampling {c['h']}x{c['v']} of {hmax}x{vmax} not supported")
        planes.append(up[:H, :W].astype(np.int64))
    if len(planes) == 1:
        return planes[0].astype(np.uint8)
    y, cb, cr = planes
    cr_r, cb_b, cr_g, cb_g = _ycc_tables()
    r = np.clip(y + cr_r[cr], 0, 255)
    g = np.clip(y + ((cb_g[cb] + cr_g[cr]) >> 16), 0, 255)
    b = np.clip(y + cb_b[cb], 0, 255)
    return np.stack([b, g, r], axis=-1).astype(np.uint8)
