"""Decode side on the GPU: fm_mjpeg_* / fm_submit_jpeg against Pillow's libjpeg-turbo.

The reference gets frames from cv2.VideoCapture.read (fm.py:413, 497-506).  The GPU decoder reproduces
libjpeg-turbo's default decode -- cv2.imdecode / OpenCV's built-in MJPEG reader -- not the FFmpeg backend
cv2.VideoCapture picks by default (that parity is unpinned; videoio keeps cv2.VideoCapture whenever OpenCV
exists unless the caller opts in).  Every case here is bit-exact against Pillow's decode of the same
bytes (the CPU restatement oracle/jpeg.py is pinned to it in tests/test_jpeg_host.py), and the whole path
from JPEG bytes to contours equals the path from the reference-decoded frames."""
import numpy as np
import pytest

from find_motion_amd import FMError, MJpegDecoder, MotionEngine
from find_motion_amd.synthetic import SyntheticVideo
from jpeg_cases import ENCODINGS, Image, encode, fill_before_markers, image, reference_decode, strip_dht

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(Image is None, reason="Pillow not importable")]


@pytest.mark.parametrize("name,kw", ENCODINGS)
@pytest.mark.parametrize("H,W", [(16, 16), (37, 53), (8, 9), (61, 33), (9, 2), (5, 4), (1, 1)])
def test_decoder_equals_libjpeg(name, kw, H, W):
    frames = [encode(image(H, W, kind, seed=s), **kw) for s, kind in enumerate(["noise", "smooth", "smooth"])]
    dec = MJpegDecoder(W, H, max_frames=4)
    got = dec.decode(frames)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f)), (name, H, W, i)
    dec.close()


@pytest.mark.parametrize("name,kw", ENCODINGS)
def test_wide_frames_without_the_fused_y_idct(name, kw):
    """3840 px wide: the colour kernel's LDS budget leaves bands of 4 rows, narrower than a block
    row, so k_jpeg_idct transforms every block (Y too) and the colour kernel reads the Y plane --
    the path the fused Y IDCT replaced for 1080p.  Two calls: the coefficient buffer and the piece
    masks must come back zeroed from both kernels."""
    H, W = 19, 3840
    frames = [encode(image(H, W, kind, seed=s), **kw) for s, kind in enumerate(["noise", "smooth"])]
    dec = MJpegDecoder(W, H, max_frames=2)
    for _ in range(2):
        got = dec.decode(frames)
        for i, f in enumerate(frames):
            assert np.array_equal(got[i], reference_decode(f)), (name, i)
        frames = frames[::-1]
    dec.close()


def test_grayscale_frames_come_out_bgr():
    frames = [encode(image(37, 53, "smooth", seed=s)[..., 1], quality=75) for s in range(3)]
    dec = MJpegDecoder(53, 37, max_frames=3)
    got = dec.decode(frames)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f))
    # and 3840 wide (k_jpeg_idct on every block, not fused into the colour kernel)
    frames = [encode(image(11, 3840, "noise", seed=s)[..., 1], quality=75) for s in range(2)]
    dec = MJpegDecoder(3840, 11, max_frames=2)
    got = dec.decode(frames)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f))


@pytest.mark.parametrize("kw", [dict(quality=75), dict(quality=90, restart_marker_rows=1),
                                dict(quality=60, subsampling=1)])
def test_1080p_synthetic_video(kw):
    v = SyntheticVideo(1920, 1080, 0)
    frames = [encode(v.frame(t), **kw) for t in (0, 1, 95, 96)]
    dec = MJpegDecoder(1920, 1080, max_frames=8)
    got = dec.decode(frames)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f)), i
    # a second call reuses the (re-zeroed) coefficient buffer
    got2 = dec.decode(frames[::-1])
    for i, f in enumerate(frames[::-1]):
        assert np.array_equal(got2[i], reference_decode(f)), i
    assert dec.last_ms() > 0


def test_decode_into_device_memory():
    torch = pytest.importorskip("torch")
    frames = [encode(image(64, 96, "smooth", seed=s), quality=80) for s in range(4)]
    dec = MJpegDecoder(96, 64, max_frames=4)
    out = torch.zeros((4, 64, 96, 3), dtype=torch.uint8, device="cuda")
    dec.decode_device(frames, out.data_ptr())
    got = out.cpu().numpy()
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f))


def test_refusals():
    dec = MJpegDecoder(16, 16, max_frames=2)
    with pytest.raises(FMError):  # progressive
        dec.decode([encode(image(16, 16, "smooth"), quality=75, progressive=True)])
    with pytest.raises(FMError):  # size differs from the decoder's
        dec.decode([encode(image(16, 24, "smooth"), quality=75)])
    with pytest.raises(FMError):  # more frames than max_frames
        dec.decode([encode(image(16, 16, "smooth"), quality=75)] * 3)
    with pytest.raises(FMError):  # not a JPEG
        dec.decode([b"\x00" * 64])
    dec.close()
    dec = MJpegDecoder(16, 16, max_frames=2)  # per-frame optimized Huffman tables: decoded run by run
    fr = [encode(image(16, 16, "noise", seed=s), quality=75, optimize=True) for s in range(2)]
    got = dec.decode(fr)
    assert all(np.array_equal(got[i], reference_decode(fr[i])) for i in range(2))


def test_submit_jpeg_equals_submit_of_decoded_frames():
    """The path from compressed frames (fm_submit_jpeg) == fm_submit of the libjpeg-decoded frames."""
    W, H, S, T = 320, 240, 2, 4
    vids = [SyntheticVideo(W, H, s) for s in range(S)]
    kw = dict(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    a, b = MotionEngine(**kw), MotionEngine(**kw)
    dec = MJpegDecoder(W, H, max_frames=T * S)
    for bi in range(3):
        jp = [encode(vids[s].frame(bi * T + t), quality=85) for t in range(T) for s in range(S)]
        frames = np.stack([reference_decode(j) for j in jp]).reshape(T, S, H, W, 3)
        a.submit_jpeg(dec, jp)
        b.submit(frames)
        a.wait()
        b.wait()
        assert np.array_equal(a.counts(), b.counts())
        for t in range(T):
            for s in range(S):
                assert [c.bbox for c in a.contours(t, s)] == [c.bbox for c in b.contours(t, s)]
                assert np.array_equal(a.mask(t, s), b.mask(t, s))
    for s in range(S):
        assert np.array_equal(a.background(s), b.background(s))
    a.close()
    b.close()


@pytest.mark.parametrize("cb,ov", [(64, 0), (64, 48), (200, 1000), (4096, 0), (1024, 512)])
def test_chunking_and_lookback(cb, ov):
    """The parallel Huffman decode cut into tiny chunks (many tiles per segment, entry states mostly
    mis-speculated, long look-back chains) and into chunks longer than whole segments: all bit-exact."""
    v = SyntheticVideo(640, 360, 3)
    groups = [  # one decoder per sampling (a decoder keeps its first frame's geometry)
        [encode(v.frame(0), quality=75), encode(v.frame(1), quality=95),
         encode(v.frame(2), quality=90, restart_marker_rows=1), encode(v.frame(5), quality=80, restart_marker_blocks=7),
         encode(image(360, 640, "noise", seed=0), quality=50), encode(image(360, 640, "noise", seed=1), quality=92)],
        [encode(v.frame(3), quality=60, subsampling=1), encode(v.frame(6), quality=97, subsampling=1)],
        [encode(v.frame(4), quality=85, subsampling=0), encode(image(360, 640, "noise", seed=2), quality=88, subsampling=0)],
    ]
    for frames in groups:
        dec = MJpegDecoder(640, 360, max_frames=len(frames), chunk_bits=cb, spec_bits=ov)
        got = dec.decode(frames)
        for i, f in enumerate(frames):
            assert np.array_equal(got[i], reference_decode(f)), i
        dec.close()
    g = MJpegDecoder(96, 64, max_frames=2, chunk_bits=cb, spec_bits=ov)  # grayscale, same chunking
    gj = [encode(image(64, 96, "noise", seed=s)[..., 0], quality=70) for s in range(2)]
    out = g.decode(gj)
    for i, f in enumerate(gj):
        assert np.array_equal(out[i], reference_decode(f)), i


def test_corrupt_and_truncated_frames_do_not_fault():
    """Damaged camera frames: entropy data cut short or overwritten.  The decode must stay inside its
    buffers (values are unspecified, as libjpeg's are after its corrupt-data warnings) and the decoder
    must still decode the next, valid call bit-exactly."""
    v = SyntheticVideo(320, 240, 5)
    good = [encode(v.frame(t), quality=q, **kw) for t, (q, kw) in
            enumerate([(75, {}), (90, {}), (85, dict(restart_marker_rows=1)), (60, {})])]
    rng = np.random.default_rng(7)
    bad = []
    for i, j in enumerate(good):
        b = bytearray(j)
        sos = b.find(b"\xff\xda")
        body = sos + 2 + ((b[sos + 2] << 8) | b[sos + 3])
        if i % 2 == 0:  # truncated scan (cut at 40 %), EOI appended
            b = b[:body + (len(b) - body) * 2 // 5] + b"\xff\xd9"
        else:  # random bytes over the middle of the scan (no 0xFF, so no fake markers)
            n = (len(b) - body) // 3
            b[body + n:body + 2 * n] = bytes(rng.integers(0, 255, n, dtype=np.uint8))
        bad.append(bytes(b))
    for cb, ov in ((1024, 512), (64, 0)):
        dec = MJpegDecoder(320, 240, max_frames=4, chunk_bits=cb, spec_bits=ov)
        for j in bad:  # one call each: a frame whose restart markers no longer cover the image is refused
            try:
                assert dec.decode([j]).shape == (1, 240, 320, 3)
            except FMError:
                pass
        out = dec.decode([bad[1], bad[3]])
        assert out.shape == (2, 240, 320, 3)
        got = dec.decode(good)
        for i, f in enumerate(good):
            assert np.array_equal(got[i], reference_decode(f)), (cb, i)
        dec.close()


def test_per_frame_optimized_huffman_tables():
    """Frames with their own (optimized) Huffman tables, mixed with standard-table frames and with a
    4:2:0 stream whose chroma use table id 1: decoded per run of frames sharing one table set."""
    v = SyntheticVideo(320, 240, 9)
    frames = [encode(v.frame(0), quality=75), encode(v.frame(1), quality=75),            # standard tables: one run
              encode(v.frame(2), quality=80, optimize=True), encode(v.frame(3), quality=80, optimize=True),
              encode(v.frame(4), quality=75), encode(image(240, 320, "noise", seed=3), quality=90, optimize=True)]
    for cb in (512, 64):
        dec = MJpegDecoder(320, 240, max_frames=len(frames), chunk_bits=cb)
        got = dec.decode(frames)
        for i, f in enumerate(frames):
            assert np.array_equal(got[i], reference_decode(f)), (cb, i)
        dec.close()


def test_frames_without_dht_use_the_standard_tables():
    """AVI1 Motion-JPEG (no DHT segment, as many webcams / IP cameras write): decoded with the T.81 Annex K
    tables libjpeg-turbo installs (std_huff_tables), alone and mixed with frames that carry the same tables."""
    v = SyntheticVideo(320, 240, 11)
    full = [encode(v.frame(t), quality=q) for t, q in enumerate((75, 90, 60, 85))]
    full.append(encode(v.frame(4), quality=80, restart_marker_rows=1))
    bare = [strip_dht(j) for j in full]
    for cb in (512, 64):
        dec = MJpegDecoder(320, 240, max_frames=len(full) * 2, chunk_bits=cb)
        got = dec.decode(bare + full[::-1])
        want = [reference_decode(j) for j in full]
        for i in range(len(full)):
            assert np.array_equal(got[i], want[i]), (cb, i)
            assert np.array_equal(got[len(full) + i], want[len(full) - 1 - i]), (cb, i)
        dec.close()
    g = [encode(image(37, 53, "smooth", seed=s)[..., 0], quality=70) for s in range(2)]  # grayscale, table 0 only
    dec = MJpegDecoder(53, 37, max_frames=2)
    out = dec.decode([strip_dht(j) for j in g])
    assert all(np.array_equal(out[i], reference_decode(g[i])) for i in range(2))


@pytest.mark.parametrize("n", [1, 2, 5])
def test_fill_bytes_before_markers(n):
    """0xFF fill bytes before every RSTn and the EOI (T.81 B.1.1.2): skipped as libjpeg does, not taken for
    the end of the scan."""
    v = SyntheticVideo(320, 240, 12)
    frames = [encode(v.frame(0), quality=80, restart_marker_blocks=3), encode(v.frame(1), quality=90, restart_marker_rows=1),
              encode(image(240, 320, "noise", seed=4), quality=75, restart_marker_blocks=1), encode(v.frame(2), quality=70)]
    filled = [fill_before_markers(j, n) for j in frames]
    dec = MJpegDecoder(320, 240, max_frames=len(frames))
    got = dec.decode(filled)
    for i, f in enumerate(frames):
        assert np.array_equal(got[i], reference_decode(f)), i
    dec.close()


def test_submit_jpeg_refuses_a_mismatched_decoder():
    """A decoder created for another frame size, or for fewer frames than a batch holds, is refused before
    anything is enqueued (its output would not fit the batch's input buffer)."""
    W, H, S, T = 64, 48, 2, 3
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    jp = [encode(image(H, W, "smooth", seed=s), quality=80) for s in range(T * S)]
    for dec in (MJpegDecoder(W * 2, H, max_frames=T * S), MJpegDecoder(W, H, max_frames=T * S - 1)):
        with pytest.raises(FMError):
            eng.submit_jpeg(dec, jp)
        dec.close()
    dec = MJpegDecoder(W, H, max_frames=T * S)
    eng._inflight.clear()
    eng.submit_jpeg(dec, jp)  # the context is still usable
    eng.wait()
    assert eng.counts().shape == (T, S)
    eng.close()
