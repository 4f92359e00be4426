"""Frame sources and sinks for the host side of the motion loop.

The reference reads with cv2.VideoCapture (fm.py:413, 501) and writes the
motion frames with cv2.VideoWriter (fm.py:447-475).  Decode/encode stay on
the host (BASELINE.json north_star), so this module only adapts what is
available:

* OpenCV, when importable: cv2.VideoCapture / cv2.VideoWriter, as the
  reference does;
* otherwise (this image has no cv2): uncompressed RIFF AVI (BI_RGB, 24-bit
  BGR, bottom-up rows), read and written here -- the container OpenCV itself
  writes for fourcc 'DIB ' and reads through FFmpeg's rawvideo decoder;
* MJPEG AVI (fourcc 'MJPG', one baseline JPEG per '00dc' chunk): with OpenCV
  present, cv2.VideoCapture reads it as the reference does (fm.py:413) unless
  the caller opts in to the GPU decoder (gpu_decode=True, CLI --gpu-decode);
  without OpenCV it is read here.  MjpegAviCapture.read_jpeg() hands the
  compressed frames to the GPU decoder (find_motion_amd.MJpegDecoder /
  fm_submit_jpeg), so only compressed bytes cross PCIe.
  That decode is bit-exact to libjpeg-turbo's default decode, i.e. to
  cv2.imdecode and OpenCV's built-in MJPEG reader (CAP_OPENCV_MJPEG) -- not to
  cv2.VideoCapture's default FFmpeg backend (libavcodec's IDCT and swscale's
  colour conversion), whose frames may differ by a few levels (that parity is
  unpinned: neither FFmpeg nor OpenCV is in this image).  A stream the GPU
  decoder does not take (progressive, 12-bit, 4:1:1 ...) is decoded on the host
  instead (cv2.imdecode, else Pillow: libjpeg-turbo either way).
  MjpegAviWriter writes such files: the 'MJPG' output of an MJPEG input keeps
  the source's JPEG bytes (write_jpeg); write() encodes a BGR frame with
  Pillow;
* in-memory sources for tests, benchmarks and embedding: ArrayCapture over a
  [N][H][W][3] uint8 array and SyntheticCapture over the deterministic
  synthetic video of find_motion_amd.synthetic.

Every capture implements the subset of the cv2.VideoCapture protocol the
reference uses: isOpened(), read() -> (ok, frame), get(CAP_PROP_*), release().
"""
from __future__ import annotations

import logging
import os
import struct

import numpy as np

log = logging.getLogger("find_motion_amd.videoio")

try:  # pragma: no cover - OpenCV is not installed in the build image
    import cv2  # type: ignore
except Exception:  # noqa: BLE001
    cv2 = None

# cv2.CAP_PROP_* values (videoio.hpp)
CAP_PROP_FPS = 5
CAP_PROP_FRAME_WIDTH = 3
CAP_PROP_FRAME_HEIGHT = 4
CAP_PROP_FRAME_COUNT = 7


class ArrayCapture:
    """VideoCapture protocol over an in-memory uint8 array [N][H][W][3] (BGR)."""

    def __init__(self, frames, fps: float = 30.0):
        self._frames = frames
        self._i = 0
        self._open = True
        self._fps = float(fps)

    def isOpened(self) -> bool:  # noqa: N802 (cv2 protocol)
        return self._open

    def read(self):
        if not self._open or self._i >= len(self._frames):
            return False, None
        f = np.ascontiguousarray(self._frames[self._i], dtype=np.uint8)
        self._i += 1
        return True, f

    def get(self, prop: int) -> float:
        n = len(self._frames)
        if prop == CAP_PROP_FRAME_COUNT:
            return float(n)
        if n == 0:
            return 0.0
        shape = self._frames[0].shape
        if prop == CAP_PROP_FRAME_WIDTH:
            return float(shape[1])
        if prop == CAP_PROP_FRAME_HEIGHT:
            return float(shape[0])
        if prop == CAP_PROP_FPS:
            return self._fps
        return 0.0

    def release(self) -> None:
        self._open = False


class JpegListCapture:
    """VideoCapture protocol over in-memory JPEG frames (an MJPEG stream already split into frames):
    read_jpeg() hands them to the GPU decoder like MjpegAviCapture; width/height from the first frame."""

    def __init__(self, jpegs, fps: float = 30.0):
        self._jpegs = list(jpegs)
        self._i = 0
        self._open = True
        self.fps = float(fps)
        self.w = self.h = 0
        if self._jpegs:
            self.h, self.w = _jpeg_size(self._jpegs[0])
        self._dec = None

    def isOpened(self) -> bool:  # noqa: N802 (cv2 protocol)
        return self._open

    def read_jpeg(self):
        if not self._open or self._i >= len(self._jpegs):
            return False, None
        j = self._jpegs[self._i]
        self._i += 1
        return True, j

    def peek_jpeg(self):
        return self._jpegs[self._i] if self._open and self._i < len(self._jpegs) else None

    def read(self):
        ok, j = self.read_jpeg()
        if not ok:
            return False, None
        if self._dec is None:
            from ._native import MJpegDecoder
            self._dec = MJpegDecoder(self.w, self.h, max_frames=1)
        return True, decode_one(self._dec, j)

    def get(self, prop: int) -> float:
        return {CAP_PROP_FRAME_COUNT: float(len(self._jpegs)), CAP_PROP_FRAME_WIDTH: float(self.w),
                CAP_PROP_FRAME_HEIGHT: float(self.h), CAP_PROP_FPS: self.fps}.get(prop, 0.0)

    def release(self) -> None:
        self._open = False
        if self._dec is not None:
            self._dec.close()
            self._dec = None


def jpeg_layout(data: bytes):
    """(height, width, ((h, v) sampling factors per component)) from a JPEG's SOF marker: frames of one
    GPU decode call must share it."""
    i = 2
    while i + 9 < len(data):
        if data[i] != 0xFF:
            raise ValueError("not a JPEG marker stream")
        m = data[i + 1]
        if 0xC0 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            nc = data[i + 9]
            comps = tuple((data[i + 11 + 3 * c] >> 4, data[i + 11 + 3 * c] & 15) for c in range(nc))
            return (data[i + 5] << 8) | data[i + 6], (data[i + 7] << 8) | data[i + 8], comps
        i += 2 + ((data[i + 2] << 8) | data[i + 3])
    raise ValueError("no SOF marker")


def jpeg_gpu_supported(data: bytes) -> bool:
    """Whether the GPU decoder takes this JPEG's layout (fm_jpeg.hip parse_jpeg / setup_geometry):
    SOF0/SOF1 Huffman, 8-bit, one component or three with Cb, Cr at 1x1 and Y at 1x1, 2x1 or 2x2,
    one interleaved scan: the first SOS names every component of the frame (a file whose components
    come in separate scans is refused by parse_jpeg)."""
    try:
        i = 2
        if data[:2] != b"\xff\xd8":
            return False
        nc = None
        while i + 4 <= len(data):
            if data[i] != 0xFF:
                return False
            while i < len(data) and data[i] == 0xFF:
                i += 1
            m = data[i]
            i += 1
            if m == 0xD9 or m == 0x01 or 0xD0 <= m <= 0xD7:
                continue
            ln = (data[i] << 8) | data[i + 1]
            seg = data[i + 2:i + ln]
            if 0xC0 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
                if m not in (0xC0, 0xC1) or seg[0] != 8:
                    return False
                nc = seg[5]
                hv = [(seg[7 + 3 * c] >> 4, seg[7 + 3 * c] & 15) for c in range(nc)]
                ok = (1 <= hv[0][0] <= 4 and 1 <= hv[0][1] <= 4) if nc == 1 else \
                    (nc == 3 and hv[1] == hv[2] == (1, 1) and hv[0] in ((1, 1), (2, 1), (2, 2)))
                if not ok:
                    return False
            if m == 0xDA:  # the first scan: interleaved over every component of the frame
                return nc is not None and len(seg) >= 1 and seg[0] == nc
            i += ln
    except IndexError:
        return False
    return False


def decode_one(dec, data: bytes) -> np.ndarray:
    """One frame through a one-frame GPU decoder, or on the host when the GPU decoder refuses this frame's
    layout (FM_ENOTSUP: a later frame of a stream whose first frame it took may be coded differently)."""
    from ._native import FM_ENOTSUP, FMError
    try:
        return dec.decode([data])[0]
    except FMError as e:
        if e.code != FM_ENOTSUP:
            raise
        log.info("JPEG frame not supported by the GPU decoder (%s); decoding it on the host", e)
        return host_decode_jpeg(data)


def host_decode_jpeg(data: bytes) -> np.ndarray:
    """One JPEG -> BGR u8 on the host with libjpeg-turbo: cv2.imdecode when OpenCV exists, else Pillow."""
    if cv2 is not None:
        return cv2.imdecode(np.frombuffer(data, np.uint8), cv2.IMREAD_COLOR)
    import io

    from PIL import Image
    im = Image.open(io.BytesIO(data))
    im = im.convert("RGB") if im.mode != "RGB" else im
    return np.ascontiguousarray(np.asarray(im)[..., ::-1])


def _jpeg_size(data: bytes):
    """(height, width) from a JPEG's SOF0/SOF1/SOF2 marker."""
    i = 2
    while i + 9 < len(data):
        if data[i] != 0xFF:
            raise ValueError("not a JPEG marker stream")
        m = data[i + 1]
        if m in (0xC0, 0xC1, 0xC2):
            return (data[i + 5] << 8) | data[i + 6], (data[i + 7] << 8) | data[i + 8]
        i += 2 + ((data[i + 2] << 8) | data[i + 3])
    raise ValueError("no SOF marker")


class SyntheticCapture(ArrayCapture):
    """The seeded synthetic stream of find_motion_amd.synthetic as a capture (frames made on demand)."""

    def __init__(self, width: int, height: int, n_frames: int, stream: int = 0, seed: int = 1000, start: int = 0):
        from .synthetic import SyntheticVideo

        self.video = SyntheticVideo(width, height, stream, seed=seed)
        self.n_frames, self.start = int(n_frames), int(start)

        class _Lazy:
            def __len__(s):  # noqa: N805
                return self.n_frames

            def __getitem__(s, i):  # noqa: N805
                return self.video.frame(self.start + i)

            @property
            def shape(s):  # noqa: N805
                return (self.n_frames, height, width, 3)

        super().__init__(_Lazy())
        self._first_shape = (height, width, 3)

    def get(self, prop: int) -> float:
        if prop == CAP_PROP_FRAME_COUNT:
            return float(self.n_frames)
        if prop == CAP_PROP_FRAME_WIDTH:
            return float(self._first_shape[1])
        if prop == CAP_PROP_FRAME_HEIGHT:
            return float(self._first_shape[0])
        return super().get(prop)


# ---------------------------------------------------------------------------
# uncompressed AVI

def _fourcc(s: str) -> bytes:
    return s.encode("ascii")[:4].ljust(4, b" ")


class RawAviWriter:
    """Uncompressed 24-bit BGR AVI (RIFF, one video stream, idx1 index)."""

    def __init__(self, path: str, fps: float, size):
        self.path = path
        self.w, self.h = int(size[0]), int(size[1])
        self.fps = max(1, int(round(fps)))
        self.row = (self.w * 3 + 3) & ~3
        self.frame_bytes = self.row * self.h
        self.n = 0
        self.index = []
        self.f = open(path, "wb")
        self._write_headers()

    def _write_headers(self):
        f = self.f
        f.write(b"RIFF" + struct.pack("<I", 0) + b"AVI ")
        hdrl = bytearray()
        avih = struct.pack("<IIIIIIIIII16x", 1000000 // self.fps, self.frame_bytes * self.fps, 0, 0x10, 0, 0, 1,
                           self.frame_bytes, self.w, self.h)
        hdrl += b"avih" + struct.pack("<I", len(avih)) + avih
        strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", b"DIB ", 0, 0, 0, 0, 1, self.fps, 0, 0, self.frame_bytes,
                           0xFFFFFFFF, 0, 0, 0, self.w, self.h)
        strf = struct.pack("<IiiHHIIiiII", 40, self.w, self.h, 1, 24, 0, self.frame_bytes, 0, 0, 0, 0)
        strl = b"strl" + b"strh" + struct.pack("<I", len(strh)) + strh + b"strf" + struct.pack("<I", len(strf)) + strf
        hdrl += b"LIST" + struct.pack("<I", len(strl)) + strl
        f.write(b"LIST" + struct.pack("<I", len(hdrl) + 4) + b"hdrl" + hdrl)
        self._avih_frames_at = 12 + 8 + 4 + 8 + 16  # RIFF hdr, LIST hdr, 'hdrl', 'avih' hdr, 4 dwords
        self._strh_len_at = 12 + 8 + 4 + 8 + len(avih) + 8 + 4 + 8 + 32
        self._movi_at = f.tell()
        f.write(b"LIST" + struct.pack("<I", 0) + b"movi")

    def isOpened(self) -> bool:  # noqa: N802
        return self.f is not None

    def write(self, frame: np.ndarray) -> None:
        frame = np.asarray(frame, dtype=np.uint8)
        if frame.shape != (self.h, self.w, 3):
            raise ValueError(f"frame shape {frame.shape} != ({self.h}, {self.w}, 3)")
        buf = np.zeros((self.h, self.row), np.uint8)
        buf[:, : self.w * 3] = frame[::-1].reshape(self.h, self.w * 3)  # bottom-up rows
        off = self.f.tell() - (self._movi_at + 8)
        self.f.write(b"00db" + struct.pack("<I", self.frame_bytes))
        self.f.write(buf.tobytes())
        self.index.append(off)
        self.n += 1

    def release(self) -> None:
        if self.f is None:
            return
        f = self.f
        movi_end = f.tell()
        f.write(b"idx1" + struct.pack("<I", 16 * len(self.index)))
        for off in self.index:
            f.write(b"00db" + struct.pack("<III", 0x10, off, self.frame_bytes))
        end = f.tell()
        f.seek(4)
        f.write(struct.pack("<I", end - 8))
        f.seek(self._movi_at + 4)
        f.write(struct.pack("<I", movi_end - self._movi_at - 8))
        f.seek(self._avih_frames_at)
        f.write(struct.pack("<I", self.n))
        f.seek(self._strh_len_at)
        f.write(struct.pack("<I", self.n))
        f.close()
        self.f = None


class RawAviCapture:
    """Reader for uncompressed 24-bit AVI (what RawAviWriter and OpenCV's 'DIB ' writer produce)."""

    def __init__(self, path: str):
        self.path = path
        self._offsets = []
        self.w = self.h = 0
        self.fps = 30.0
        self._i = 0
        self._open = False
        try:
            self._parse()
            self._open = self.w > 0 and self.h > 0
        except (OSError, ValueError, struct.error) as e:
            log.error("cannot read %s as uncompressed AVI: %s", path, e)

    def _parse(self):
        with open(self.path, "rb") as f:
            data = f.read(12)
            if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"AVI ":
                raise ValueError("not a RIFF AVI file")
            size = os.path.getsize(self.path)
            self._walk(f, 12, size, depth=0)
        self._mm = np.memmap(self.path, dtype=np.uint8, mode="r")

    def _walk(self, f, start, end, depth):
        pos = start
        while pos + 8 <= end:
            f.seek(pos)
            ck, ln = struct.unpack("<4sI", f.read(8))
            body = pos + 8
            if ck == b"LIST" or (ck == b"RIFF" and depth == 0):
                # RIFF 'AVIX': the OpenDML continuation of a file past 1 GB, more 'movi' data
                kind = f.read(4)
                if kind in (b"hdrl", b"strl", b"movi", b"rec ", b"AVIX") and depth < 4:
                    self._walk(f, body + 4, min(body + ln, end), depth + 1)
            elif ck == b"avih":
                vals = struct.unpack("<10I", f.read(40))
                if vals[0]:
                    self.fps = 1e6 / vals[0]
            elif ck == b"strf" and not self.w:
                bi = struct.unpack("<IiiHHI", f.read(20))
                if bi[4] != 24 or bi[5] != 0:
                    raise ValueError(f"only uncompressed 24-bit BGR AVI is readable without OpenCV "
                                     f"(bitcount {bi[4]}, compression {bi[5]})")
                self.w, self.h = bi[1], bi[2]
                self._bottom_up = self.h > 0
                self.h = abs(self.h)
                self.row = (self.w * 3 + 3) & ~3
            elif ck[2:] in (b"db", b"dc") and ln > 0:
                self._offsets.append((body, ln))
            pos = body + ln + (ln & 1)

    def isOpened(self) -> bool:  # noqa: N802
        return self._open

    def read(self):
        if not self._open or self._i >= len(self._offsets):
            return False, None
        off, ln = self._offsets[self._i]
        self._i += 1
        if ln < self.row * self.h:
            return False, None
        rows = np.asarray(self._mm[off: off + self.row * self.h]).reshape(self.h, self.row)[:, : self.w * 3]
        if self._bottom_up:
            rows = rows[::-1]
        return True, np.ascontiguousarray(rows).reshape(self.h, self.w, 3)

    def get(self, prop: int) -> float:
        return {CAP_PROP_FRAME_COUNT: float(len(self._offsets)), CAP_PROP_FRAME_WIDTH: float(self.w),
                CAP_PROP_FRAME_HEIGHT: float(self.h), CAP_PROP_FPS: self.fps}.get(prop, 0.0)

    def release(self) -> None:
        self._open = False
        self._mm = None


FOURCC_MJPG = b"MJPG"


class MjpegAviCapture(RawAviCapture):
    """MJPEG AVI reader: read_jpeg() -> (ok, JPEG bytes) for the GPU decoder; read() -> (ok, BGR frame).

    gpu_decode (True unless the caller turns it off or the first frame's layout is one the GPU decoder
    does not take, jpeg_gpu_supported): read() decodes on the GPU (a one-frame MJpegDecoder on `device`,
    created on first use) and BatchFeeder hands the compressed frames to fm_submit_jpeg; otherwise
    read() decodes on the host (host_decode_jpeg) and the feeder copies decoded frames."""

    def __init__(self, path: str, device: int = 0, gpu_decode: bool = True):
        self._device = int(device)
        self._dec = None
        super().__init__(path)
        first = self.peek_jpeg()
        self.gpu_decode = bool(gpu_decode) and (first is None or jpeg_gpu_supported(first))
        if gpu_decode and not self.gpu_decode:
            log.info("%s: JPEG layout not supported by the GPU decoder; decoding on the host", path)

    def _walk(self, f, start, end, depth):
        pos = start
        while pos + 8 <= end:
            f.seek(pos)
            ck, ln = struct.unpack("<4sI", f.read(8))
            body = pos + 8
            if ck == b"LIST" or (ck == b"RIFF" and depth == 0):
                # RIFF 'AVIX': the OpenDML continuation of a file past 1 GB, more 'movi' data
                kind = f.read(4)
                if kind in (b"hdrl", b"strl", b"movi", b"rec ", b"AVIX") and depth < 4:
                    self._walk(f, body + 4, min(body + ln, end), depth + 1)
            elif ck == b"avih":
                vals = struct.unpack("<10I", f.read(40))
                if vals[0]:
                    self.fps = 1e6 / vals[0]
            elif ck == b"strf" and not self.w:
                bi = struct.unpack("<IiiHH4s", f.read(20))
                if bi[5] != FOURCC_MJPG:
                    raise ValueError(f"not an MJPEG AVI (compression {bi[5]!r})")
                self.w, self.h = bi[1], abs(bi[2])
            elif ck[2:] == b"dc" and ln > 0:
                self._offsets.append((body, ln))
            pos = body + ln + (ln & 1)

    def read_jpeg(self):
        if not self._open or self._i >= len(self._offsets):
            return False, None
        off, ln = self._offsets[self._i]
        self._i += 1
        return True, bytes(self._mm[off: off + ln])

    def peek_jpeg(self):
        """The next frame's JPEG bytes without consuming it (None at the end)."""
        if not self._open or self._i >= len(self._offsets):
            return None
        off, ln = self._offsets[self._i]
        return bytes(self._mm[off: off + ln])

    def read(self):
        ok, j = self.read_jpeg()
        if not ok:
            return False, None
        if not self.gpu_decode:
            return True, host_decode_jpeg(j)
        if self._dec is None:
            from ._native import MJpegDecoder
            self._dec = MJpegDecoder(self.w, self.h, max_frames=1, device=self._device)
        return True, decode_one(self._dec, j)

    def release(self) -> None:
        super().release()
        if self._dec is not None:
            self._dec.close()
            self._dec = None


class MjpegAviWriter(RawAviWriter):
    """MJPEG AVI writer: frames encoded by Pillow (libjpeg-turbo) at `quality` (default 95, OpenCV's MJPG
    default), one '00dc' chunk per frame."""

    def __init__(self, path: str, fps: float, size, quality: int = 95, **jpeg_kw):
        self.quality = int(quality)
        self.jpeg_kw = jpeg_kw
        self.sizes = []
        super().__init__(path, fps, size)

    def _write_headers(self):
        f = self.f
        f.write(b"RIFF" + struct.pack("<I", 0) + b"AVI ")
        mx = self.w * self.h * 3
        hdrl = bytearray()
        avih = struct.pack("<IIIIIIIIII16x", 1000000 // self.fps, mx * self.fps, 0, 0x10, 0, 0, 1, mx, self.w, self.h)
        hdrl += b"avih" + struct.pack("<I", len(avih)) + avih
        strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", FOURCC_MJPG, 0, 0, 0, 0, 1, self.fps, 0, 0, mx,
                           0xFFFFFFFF, 0, 0, 0, self.w, self.h)
        strf = struct.pack("<IiiHH4sIiiII", 40, self.w, self.h, 1, 24, FOURCC_MJPG, mx, 0, 0, 0, 0)
        strl = b"strl" + b"strh" + struct.pack("<I", len(strh)) + strh + b"strf" + struct.pack("<I", len(strf)) + strf
        hdrl += b"LIST" + struct.pack("<I", len(strl)) + strl
        f.write(b"LIST" + struct.pack("<I", len(hdrl) + 4) + b"hdrl" + hdrl)
        self._avih_frames_at = 12 + 8 + 4 + 8 + 16
        self._strh_len_at = 12 + 8 + 4 + 8 + len(avih) + 8 + 4 + 8 + 32
        self._movi_at = f.tell()
        f.write(b"LIST" + struct.pack("<I", 0) + b"movi")

    def write_jpeg(self, data: bytes) -> None:
        off = self.f.tell() - (self._movi_at + 8)
        self.f.write(b"00dc" + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b""))
        self.index.append(off)
        self.sizes.append(len(data))
        self.n += 1

    def write(self, frame: np.ndarray) -> None:
        import io

        from PIL import Image
        frame = np.asarray(frame, dtype=np.uint8)
        if frame.shape != (self.h, self.w, 3):
            raise ValueError(f"frame shape {frame.shape} != ({self.h}, {self.w}, 3)")
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(frame[..., ::-1])).save(b, "JPEG", quality=self.quality, **self.jpeg_kw)
        self.write_jpeg(b.getvalue())

    def release(self) -> None:
        if self.f is None:
            return
        f = self.f
        movi_end = f.tell()
        f.write(b"idx1" + struct.pack("<I", 16 * len(self.index)))
        for off, ln in zip(self.index, self.sizes):
            f.write(b"00dc" + struct.pack("<III", 0x10, off, ln))
        end = f.tell()
        f.seek(4)
        f.write(struct.pack("<I", end - 8))
        f.seek(self._movi_at + 4)
        f.write(struct.pack("<I", movi_end - self._movi_at - 8))
        f.seek(self._avih_frames_at)
        f.write(struct.pack("<I", self.n))
        f.seek(self._strh_len_at)
        f.write(struct.pack("<I", self.n))
        f.close()
        self.f = None


def is_mjpeg_avi(path) -> bool:
    """An AVI whose video stream is MJPG (read by MjpegAviCapture, decoded on the GPU)."""
    try:
        with open(path, "rb") as f:
            head = f.read(4096)
    except (OSError, TypeError):
        return False
    return head[:4] == b"RIFF" and head[8:12] == b"AVI " and FOURCC_MJPG in head


def open_capture(source, device: int = 0, gpu_decode: bool | None = None):
    """cv2.VideoCapture(source) when OpenCV exists (fm.py:413); otherwise the readers above.

    gpu_decode: MJPEG AVI files go to MjpegAviCapture (GPU decode, libjpeg-turbo-exact) when True, or
    when None (the default) and OpenCV is absent.  With OpenCV present and gpu_decode not True the
    reference's own capture is returned, whatever the codec.  gpu_decode=False without OpenCV still
    reads MJPEG AVIs with MjpegAviCapture, decoding on the host.

    `source` may also be an object that already speaks the capture protocol,
    a uint8 array [N][H][W][3], or "synthetic:WxH:N[:stream]".
    """
    if hasattr(source, "read") and hasattr(source, "isOpened"):
        return source
    if isinstance(source, np.ndarray):
        return ArrayCapture(source)
    if isinstance(source, str) and source.startswith("synthetic:"):
        parts = source.split(":")
        w, h = (int(v) for v in parts[1].lower().split("x"))
        return SyntheticCapture(w, h, int(parts[2]), int(parts[3]) if len(parts) > 3 else 0)
    if isinstance(source, str) and source.endswith(".npy"):
        return ArrayCapture(np.load(source, mmap_mode="r", allow_pickle=False))
    if isinstance(source, str) and is_mjpeg_avi(source) and (cv2 is None or gpu_decode):
        cap = MjpegAviCapture(source, device, gpu_decode=gpu_decode is not False)
        if cap.isOpened() and (cap.gpu_decode or cv2 is None):
            return cap  # compressed frames to the GPU decoder (§8(f)-3), or host decode without cv2
        cap.release()  # opted in, but the layout needs the host: the reference's capture
    if cv2 is not None:
        return cv2.VideoCapture(source)
    if isinstance(source, int):
        raise OSError(f"camera {source}: camera capture needs OpenCV, which is not installed")
    return RawAviCapture(str(source))


def open_writer(path: str, codec: str, fps: float, size, jpeg: bool = False):
    """cv2.VideoWriter(path, fourcc(codec), fps, size) (fm.py:468-470), else an uncompressed AVI.
    jpeg: the frames come from an MJPEG source -- an 'MJPG' output is then an MjpegAviWriter that
    stores the source's JPEG bytes as they are (write_jpeg), with or without cv2."""
    if jpeg and codec == "MJPG":
        return MjpegAviWriter(path, fps, size)
    if cv2 is not None:
        return cv2.VideoWriter(path, cv2.VideoWriter_fourcc(*codec), fps, size)
    if codec not in ("DIB ", "RGB ", "raw ", None):
        log.debug("OpenCV absent: writing %s as uncompressed AVI instead of codec %s", path, codec)
    return RawAviWriter(path, fps, size)
