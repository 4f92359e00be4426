"""JPEG test inputs for the decode side (§8(f)-3): frames encoded by Pillow (libjpeg-turbo), decoded by Pillow
as the reference decode.  That is libjpeg-turbo's default decode, i.e. cv2.imdecode and OpenCV's built-in
MJPEG reader (CAP_OPENCV_MJPEG); cv2.VideoCapture's default FFmpeg backend decodes with libavcodec + swscale
instead, which nothing here can pin (neither is in the image)."""
from __future__ import annotations

import io

import numpy as np

try:
    from PIL import Image
except ImportError:  # pragma: no cover - Pillow is in the image; the tests skip without it
    Image = None

# (name, encoder keyword arguments): 4:2:0 / 4:2:2 / 4:4:4, qualities, restart intervals
ENCODINGS = [
    ("420_q75", dict(quality=75)),
    ("420_q30", dict(quality=30)),
    ("444_q95", dict(quality=95, subsampling=0)),
    ("422_q50", dict(quality=50, subsampling=1)),
    ("420_rst3", dict(quality=80, restart_marker_blocks=3)),
    ("422_rstrow", dict(quality=70, subsampling=1, restart_marker_rows=1)),
]


def image(H: int, W: int, kind: str, seed: int = 1) -> np.ndarray:
    """BGR u8 test image: noise (every coefficient busy) or a noisy gradient (typical video)."""
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
    y, x = np.mgrid[0:H, 0:W]
    img = np.stack([(x * 255 // max(W - 1, 1)), (y * 255 // max(H - 1, 1)), ((x + y) * 7) % 256], -1)
    return (img + rng.integers(-20, 21, img.shape)).clip(0, 255).astype(np.uint8)


def encode(bgr: np.ndarray, **kw) -> bytes:
    """BGR (or gray) u8 -> JPEG bytes (Pillow, libjpeg-turbo)."""
    arr = bgr[..., ::-1] if bgr.ndim == 3 else bgr
    b = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(arr)).save(b, "JPEG", **kw)
    return b.getvalue()


def reference_decode(data: bytes) -> np.ndarray:
    """Pillow's libjpeg-turbo decode -> BGR u8 (gray replicated to three channels, as cap.read returns)."""
    im = Image.open(io.BytesIO(data))
    a = np.asarray(im)
    if a.ndim == 2:
        return np.repeat(a[..., None], 3, axis=2)
    return np.ascontiguousarray(a[..., ::-1])


def segments(data: bytes):
    """(marker, start, end) of every marker segment before the scan data (SOI excluded)."""
    out, i = [], 2
    while i + 4 <= len(data) and data[i] == 0xFF:
        m = data[i + 1]
        ln = (data[i + 2] << 8) | data[i + 3]
        out.append((m, i, i + 2 + ln))
        if m == 0xDA:
            break
        i += 2 + ln
    return out


def strip_dht(data: bytes) -> bytes:
    """The same JPEG without its DHT segments (the AVI1 Motion-JPEG form many cameras write: the decoder
    supplies the T.81 Annex K tables, which are exactly what libjpeg-turbo encodes with by default)."""
    out, last = bytearray(data[:2]), 2
    for m, a, b in segments(data):
        out += data[last:a]
        if m != 0xC4:
            out += data[a:b]
        last = b
    return bytes(out + data[last:])


def fill_before_markers(data: bytes, n: int = 2) -> bytes:
    """Insert n 0xFF fill bytes before every RSTn marker and the EOI of the scan (T.81 B.1.1.2 allows any
    number; libjpeg skips them)."""
    sos = [s for s in segments(data) if s[0] == 0xDA][0]
    head, scan = data[:sos[2]], data[sos[2]:]
    out, k = bytearray(), 0
    while k < len(scan):
        c = scan[k]
        if c == 0xFF and k + 1 < len(scan) and (0xD0 <= scan[k + 1] <= 0xD7 or scan[k + 1] == 0xD9):
            out += b"\xff" * n
        out.append(c)
        k += 1
    return bytes(head + out)
