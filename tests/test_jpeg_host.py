"""Decode side, CPU: the restatement oracle/jpeg.py against Pillow's libjpeg-turbo.

libjpeg-turbo's default decode is what cv2.imdecode and OpenCV's built-in MJPEG reader (CAP_OPENCV_MJPEG) run
on MJPEG frames.  It is NOT what cv2.VideoCapture.read (fm.py:413, 497-506) runs by default: stock OpenCV builds
open AVI files with the FFmpeg backend (libavcodec IDCT, swscale), whose parity is unpinned here.
Pillow bundles libjpeg-turbo, so the restatement of jdhuff / jidctint (islow) / jdsample (fancy upsampling) / jdcolor
is pinned bit for bit here, on every sampling layout, odd sizes (partial MCUs, one-column chroma), restart
intervals and grayscale.  The committed fixtures (tests/golden/jpeg_cases.npz, tests/golden/make_golden_jpeg.py)
keep the same check on a machine whose Pillow differs."""
import os

import numpy as np
import pytest

from oracle import jpeg
from jpeg_cases import ENCODINGS, Image, encode, fill_before_markers, image, reference_decode, segments, strip_dht

pytestmark = pytest.mark.skipif(Image is None, reason="Pillow not importable")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jpeg_cases.npz")


def _bgr(a):
    return np.repeat(a[..., None], 3, axis=2) if a.ndim == 2 else a


@pytest.mark.parametrize("name,kw", ENCODINGS)
@pytest.mark.parametrize("H,W", [(16, 16), (37, 53), (8, 9), (24, 40), (61, 33), (9, 2), (5, 4), (3, 7), (1, 1)])
@pytest.mark.parametrize("kind", ["noise", "smooth"])
def test_restatement_equals_libjpeg(name, kw, H, W, kind):
    data = encode(image(H, W, kind), **kw)
    assert np.array_equal(_bgr(jpeg.decode(data)), reference_decode(data))


@pytest.mark.parametrize("H,W", [(16, 16), (37, 53)])
def test_grayscale(H, W):
    data = encode(image(H, W, "smooth")[..., 1], quality=75)
    assert np.array_equal(_bgr(jpeg.decode(data)), reference_decode(data))


def test_parse_reports_layout_and_restart_interval():
    j = jpeg.parse(encode(image(32, 48, "smooth"), quality=80, restart_marker_blocks=3))
    assert (j["frame"]["H"], j["frame"]["W"]) == (32, 48)
    assert [(c["h"], c["v"]) for c in j["frame"]["comps"]] == [(2, 2), (1, 1), (1, 1)]
    assert j["dri"] > 0
    assert set(j["ht"]) == {(0, 0), (1, 0), (0, 1), (1, 1)}


def test_progressive_is_refused():
    data = encode(image(16, 16, "smooth"), quality=75, progressive=True)
    with pytest.raises(jpeg.JpegError):
        jpeg.parse(data)


def test_golden_fixtures():
    z = np.load(GOLDEN)
    n = int(z["n"])
    for i in range(n):
        data = z[f"jpeg{i}"].tobytes()
        assert np.array_equal(_bgr(jpeg.decode(data)), z[f"bgr{i}"]), i


def test_mjpeg_avi_round_trip(tmp_path):
    """videoio.MjpegAviWriter -> MjpegAviCapture: chunk bytes, count, size and rate survive; open_capture
    picks the MJPEG reader (the GPU decode path) and open_writer(jpeg=True) the passthrough writer."""
    from find_motion_amd import videoio
    W, H = 72, 40
    jp = [encode(image(H, W, "smooth", seed=s), quality=70 + s) for s in range(5)]  # odd and even lengths
    p = str(tmp_path / "m.avi")
    w = videoio.open_writer(p, "MJPG", 25, (W, H), jpeg=True)
    assert isinstance(w, videoio.MjpegAviWriter)
    for j in jp[:4]:
        w.write_jpeg(j)
    w.write(reference_decode(jp[4]))  # a BGR frame, Pillow-encoded
    w.release()
    assert videoio.is_mjpeg_avi(p) and not videoio.is_mjpeg_avi(str(tmp_path / "none.avi"))
    cap = videoio.open_capture(p) if videoio.cv2 is None else videoio.open_capture(p, gpu_decode=True)
    assert isinstance(cap, videoio.MjpegAviCapture)
    assert (cap.get(videoio.CAP_PROP_FRAME_COUNT), cap.get(videoio.CAP_PROP_FRAME_WIDTH),
            cap.get(videoio.CAP_PROP_FRAME_HEIGHT)) == (5, W, H)
    assert abs(cap.fps - 25) < 0.01
    got = []
    while True:
        ok, j = cap.read_jpeg()
        if not ok:
            break
        got.append(j)
    assert got[:4] == jp[:4] and len(got) == 5
    assert reference_decode(got[4]).shape == (H, W, 3)
    cap.release()
    raw = str(tmp_path / "r.avi")
    videoio.RawAviWriter(raw, 25, (W, H)).release()
    assert not videoio.is_mjpeg_avi(raw)
    assert not videoio.MjpegAviCapture(raw).isOpened()  # cv2-like: a capture that failed to open


def test_mjpeg_avi_opendml_continuation(tmp_path):
    """Frames in an OpenDML 'RIFF AVIX' continuation (files past 1 GB) are read after the first RIFF's."""
    import struct

    from find_motion_amd import videoio
    W, H = 32, 16
    jp = [encode(image(H, W, "smooth", seed=s), quality=80) for s in range(5)]
    p = str(tmp_path / "big.avi")
    w = videoio.MjpegAviWriter(p, 30, (W, H))
    for j in jp[:3]:
        w.write_jpeg(j)
    w.release()
    movi = b"movi" + b"".join(b"00dc" + struct.pack("<I", len(j)) + j + (b"\0" if len(j) & 1 else b"") for j in jp[3:])
    avix = b"AVIX" + b"LIST" + struct.pack("<I", len(movi)) + movi
    with open(p, "ab") as f:
        f.write(b"RIFF" + struct.pack("<I", len(avix)) + avix)
    cap = videoio.MjpegAviCapture(p)
    got = []
    while True:
        ok, j = cap.read_jpeg()
        if not ok:
            break
        got.append(j)
    assert got == jp


def test_jpeg_layout():
    from find_motion_amd import videoio
    assert videoio.jpeg_layout(encode(image(24, 40, "smooth"), quality=75)) == (24, 40, ((2, 2), (1, 1), (1, 1)))
    assert videoio.jpeg_layout(encode(image(24, 40, "smooth"), quality=75, subsampling=1))[2] == ((2, 1), (1, 1), (1, 1))
    assert videoio.jpeg_layout(encode(image(24, 40, "smooth")[..., 0], quality=75)) == (24, 40, ((1, 1),))
    cap = videoio.JpegListCapture([encode(image(24, 40, "smooth"), quality=75)])
    assert cap.peek_jpeg() is not None and cap.read_jpeg()[0] and cap.peek_jpeg() is None


def test_standard_huffman_tables_are_the_ones_libjpeg_encodes_with():
    """oracle STD_HUFF (T.81 Annex K.3, libjpeg-turbo jstdhuff.c) == the DHT Pillow writes without optimize."""
    j = jpeg.parse(encode(image(16, 16, "noise"), quality=75))
    for key in ((0, 0), (0, 1), (1, 0), (1, 1)):
        bits, vals = j["ht"][key]
        assert (list(bits), list(vals)) == (list(jpeg.STD_HUFF[key][0]), list(jpeg.STD_HUFF[key][1])), key
    assert [len(jpeg.STD_HUFF[k][1]) for k in ((0, 0), (0, 1), (1, 0), (1, 1))] == [12, 12, 162, 162]


@pytest.mark.parametrize("name,kw", ENCODINGS[:5])
def test_frame_without_dht_decodes_with_the_standard_tables(name, kw):
    """AVI1 Motion-JPEG: no DHT segment; libjpeg-turbo (std_huff_tables) and the restatement supply Annex K."""
    data = encode(image(37, 53, "smooth"), **kw)
    bare = strip_dht(data)
    assert not any(m == 0xC4 for m, _, _ in segments(bare)) and len(bare) < len(data)
    want = reference_decode(data)
    assert np.array_equal(reference_decode(bare), want)  # libjpeg-turbo itself accepts the bare frame
    assert np.array_equal(_bgr(jpeg.decode(bare)), want)


@pytest.mark.parametrize("n", [1, 3])
def test_fill_bytes_before_restart_markers(n):
    """0xFF fill bytes before RSTn / EOI (T.81 B.1.1.2) are skipped, as libjpeg does."""
    data = encode(image(40, 56, "noise"), quality=80, restart_marker_blocks=2)
    filled = fill_before_markers(data, n)
    assert len(filled) > len(data)
    want = reference_decode(data)
    assert np.array_equal(reference_decode(filled), want)
    assert np.array_equal(_bgr(jpeg.decode(filled)), want)


def test_jpeg_gpu_supported_layouts():
    from find_motion_amd import videoio
    ok = [encode(image(24, 40, "smooth"), quality=75, subsampling=s) for s in (0, 1, 2)]
    ok.append(encode(image(24, 40, "smooth")[..., 0], quality=75))
    ok.append(strip_dht(ok[0]))
    assert all(videoio.jpeg_gpu_supported(j) for j in ok)
    assert not videoio.jpeg_gpu_supported(encode(image(24, 40, "smooth"), quality=75, progressive=True))
    assert not videoio.jpeg_gpu_supported(b"not a jpeg")


def _marker_stream(ns, nc=3):
    """SOI, SOF0 (8-bit, 16x16, nc components at 1x1), SOS naming ns of them: the markers only."""
    sof = bytes([8, 0, 16, 0, 16, nc]) + b"".join(bytes([c + 1, 0x11, 0]) for c in range(nc))
    sos = bytes([ns]) + b"".join(bytes([c + 1, 0]) for c in range(ns)) + bytes([0, 63, 0])
    seg = lambda m, body: bytes([0xFF, m]) + (len(body) + 2).to_bytes(2, "big") + body  # noqa: E731
    return b"\xff\xd8" + seg(0xC0, sof) + seg(0xDA, sos) + b"\x00" * 8 + b"\xff\xd9"


def test_jpeg_gpu_supported_needs_one_interleaved_scan():
    """A frame whose components come in separate scans (first SOS with Ns < Nf) is refused up front, as
    parse_jpeg (fm_jpeg.hip) would refuse it (the advisor's round-3 finding)."""
    from find_motion_amd import videoio
    assert videoio.jpeg_gpu_supported(_marker_stream(3))
    assert not videoio.jpeg_gpu_supported(_marker_stream(1))
    assert not videoio.jpeg_gpu_supported(_marker_stream(2))
    assert videoio.jpeg_gpu_supported(_marker_stream(1, nc=1))


class _StubCv2:
    """Just enough of cv2 for open_capture's choice: VideoCapture records what it was opened on."""

    class VideoCapture:
        def __init__(self, src):
            self.src = src

        def isOpened(self):  # noqa: N802
            return True

    IMREAD_COLOR = 1


def _mjpeg_avi(tmp_path, **kw):
    from find_motion_amd import videoio
    p = str(tmp_path / "m.avi")
    w = videoio.MjpegAviWriter(p, 25, (40, 24))
    for s in range(3):
        w.write_jpeg(encode(image(24, 40, "smooth", seed=s), quality=75, **kw))
    w.release()
    return p


def test_open_capture_keeps_the_reference_capture_when_cv2_imports(tmp_path, monkeypatch):
    """fm.py:413: cv2.VideoCapture(filename) whenever OpenCV exists, MJPEG included; the GPU decoder only on
    opt-in (gpu_decode=True), and never for a layout it does not take."""
    from find_motion_amd import videoio
    p = _mjpeg_avi(tmp_path)
    monkeypatch.setattr(videoio, "cv2", _StubCv2)
    cap = videoio.open_capture(p)
    assert isinstance(cap, _StubCv2.VideoCapture) and cap.src == p
    assert isinstance(videoio.open_capture(p, gpu_decode=False), _StubCv2.VideoCapture)
    cap = videoio.open_capture(p, gpu_decode=True)
    assert isinstance(cap, videoio.MjpegAviCapture) and cap.gpu_decode
    q = str(tmp_path / "p.avi")
    w = videoio.MjpegAviWriter(q, 25, (40, 24))
    w.write_jpeg(encode(image(24, 40, "smooth"), quality=75, progressive=True))
    w.release()
    assert isinstance(videoio.open_capture(q, gpu_decode=True), _StubCv2.VideoCapture)
    raw = str(tmp_path / "r.avi")
    videoio.RawAviWriter(raw, 25, (40, 24)).release()
    assert isinstance(videoio.open_capture(raw), _StubCv2.VideoCapture)


def test_open_capture_without_cv2(tmp_path, monkeypatch):
    """No OpenCV: MJPEG AVIs are read here -- GPU decode for supported layouts (the default), host decode
    (Pillow, libjpeg-turbo) for the rest or on gpu_decode=False; BatchFeeder's JPEG mode only for the former."""
    from find_motion_amd import videoio
    monkeypatch.setattr(videoio, "cv2", None)
    p = _mjpeg_avi(tmp_path)
    cap = videoio.open_capture(p)
    assert isinstance(cap, videoio.MjpegAviCapture) and cap.gpu_decode
    cap = videoio.open_capture(p, gpu_decode=False)
    assert isinstance(cap, videoio.MjpegAviCapture) and not cap.gpu_decode
    ok, fr = cap.read()
    assert ok and np.array_equal(fr, reference_decode(encode(image(24, 40, "smooth", seed=0), quality=75)))
    q = str(tmp_path / "p.avi")
    w = videoio.MjpegAviWriter(q, 25, (40, 24))
    pj = encode(image(24, 40, "smooth"), quality=75, progressive=True)
    w.write_jpeg(pj)
    w.release()
    cap = videoio.open_capture(q, gpu_decode=True)
    assert isinstance(cap, videoio.MjpegAviCapture) and not cap.gpu_decode
    ok, fr = cap.read()
    assert ok and np.array_equal(fr, reference_decode(pj))
