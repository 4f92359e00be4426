"""Decode side, CPU: the restatement oracle/jpeg.py against Pillow's libjpeg-turbo.

libjpeg-turbo's default decode is what cv2.VideoCapture.read / imdecode run on MJPEG frames (fm.py:497-506);
Pillow bundles it, so the restatement of jdhuff / jidctint (islow) / jdsample (fancy upsampling) / jdcolor
is pinned bit for bit here, on every sampling layout, odd sizes (partial MCUs, one-column chroma), restart
intervals and grayscale.  The committed fixtures (tests/golden/jpeg_cases.npz, tests/golden/make_golden_jpeg.py)
keep the same check on a machine whose Pillow differs."""
import os

import numpy as np
import pytest

from oracle import jpeg
from jpeg_cases import ENCODINGS, Image, encode, image, reference_decode

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
    cap = videoio.open_capture(p)
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
