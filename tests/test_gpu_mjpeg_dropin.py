"""The drop-in on MJPEG input (SURVEY.md §8(f)-3 wired into §8(b)): an MJPEG AVI read by
videoio.MjpegAviCapture is decoded on the GPU in front of the hot path (BatchFeeder JPEG mode ->
fm_submit_jpeg).  Decisions must equal the oracle's on the libjpeg-turbo-decoded frames
(cv2.VideoCapture's frames, fm.py:497-506), raw frames fetched lazily (fm_read_frame, or the
one-frame decoder once the batch is gone) must equal those decoded frames, and an MJPG output
must hold the source's JPEG bytes of exactly the written frames."""
import numpy as np
import pytest

import oracle
from find_motion_amd import MotionEngine, motion, videoio
from find_motion_amd.synthetic import SyntheticVideo
from jpeg_cases import encode, reference_decode
from oracle.decision import written_indices

pytestmark = pytest.mark.gpu


def _mjpeg_avi(path, W, H, n, seed, **kw):
    vid = SyntheticVideo(W, H, seed)
    jp = [encode(vid.frame(i), **kw) for i in range(n)]
    w = videoio.MjpegAviWriter(str(path), 30, (W, H))
    for j in jp:
        w.write_jpeg(j)
    w.release()
    return jp


def _oracle_written(jp, W, H, box, ksize=5, threshold=12):
    st = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=box, ksize=ksize, thresh=threshold))
    counts = [st.step(reference_decode(j))["count"] for j in jp]
    return written_indices(counts, min_time=0.1, cache_time=0.3)


def _read_all(cap):
    out = []
    while True:
        ok, f = cap.read_jpeg() if hasattr(cap, "read_jpeg") else cap.read()
        if not ok:
            return out
        out.append(f)


@pytest.mark.parametrize("batch", [1, 8])
def test_video_motion_on_mjpeg_avi(tmp_path, batch):
    W, H, n = 480, 270, 48
    src = tmp_path / "v.avi"
    jp = _mjpeg_avi(src, W, H, n, 0, quality=85)
    vm = motion.VideoMotion(filename=str(src), box_size=100, threshold=12, cache_time=0.3, min_time=0.1,
                            batch=batch, outdir=str(tmp_path))
    assert isinstance(vm.cap, videoio.MjpegAviCapture)
    vm.find_motion()
    want = _oracle_written(jp, W, H, 100)
    assert want and vm.written_indices == want
    got = _read_all(videoio.MjpegAviCapture(vm.outfile_name))
    assert got == [jp[i] for i in want]  # MJPG out: the source's bytes, no re-encode


def test_lazy_raw_frames_written_uncompressed(tmp_path):
    """Codec 'DIB ': every written frame is decoded -- from the engine's input slot while its batch is
    current, by the one-frame decoder for cached frames of batches already overwritten."""
    W, H, n = 320, 240, 40
    src = tmp_path / "v.avi"
    jp = _mjpeg_avi(src, W, H, n, 1, quality=90, restart_marker_rows=2)
    vm = motion.VideoMotion(filename=str(src), box_size=100, threshold=12, cache_time=0.3, min_time=0.1,
                            batch=8, outdir=str(tmp_path), codec="DIB ")
    vm.find_motion()
    want = _oracle_written(jp, W, H, 100)
    assert want and vm.written_indices == want
    got = _read_all(videoio.RawAviCapture(vm.outfile_name))
    assert len(got) == len(want)
    for g, i in zip(got, want):
        assert np.array_equal(g, reference_decode(jp[i])), i


def test_unsupported_frames_mid_stream_decode_on_the_host(tmp_path):
    """A stream whose first frame the GPU decoder takes but whose later frames it refuses (progressive
    JPEGs at frames 10-29, then 4:4:4 instead of the first frame's 4:2:0 sampling at frames 30-35): the
    batches holding them are decoded on the host and submitted as frames (feeder), cached frames of
    overwritten batches too (one-frame decoder) -- decisions and every written raw frame equal the
    oracle's on the libjpeg-turbo-decoded frames, nothing raises."""
    W, H, n = 320, 240, 40
    vid = SyntheticVideo(W, H, 3)
    jp = [encode(vid.frame(i), quality=85, progressive=10 <= i < 30, subsampling=0 if 30 <= i < 36 else 2)
          for i in range(n)]
    src = tmp_path / "v.avi"
    w = videoio.MjpegAviWriter(str(src), 30, (W, H))
    for j in jp:
        w.write_jpeg(j)
    w.release()
    vm = motion.VideoMotion(filename=str(src), box_size=100, threshold=12, cache_time=0.3, min_time=0.1,
                            batch=8, outdir=str(tmp_path), codec="DIB ", gpu_decode=True)
    assert isinstance(vm.cap, videoio.MjpegAviCapture) and vm.cap.gpu_decode
    vm.find_motion()
    want = _oracle_written(jp, W, H, 100)
    assert want and vm.written_indices == want
    assert any(10 <= i < 30 for i in want)
    got = _read_all(videoio.RawAviCapture(vm.outfile_name))
    assert len(got) == len(want)
    for g, i in zip(got, want):
        assert np.array_equal(g, reference_decode(jp[i])), i
    cap = videoio.JpegListCapture(jp[8:12] + jp[28:32])
    for k in range(8):  # the one-frame GPU decoder: baseline frames on the GPU, progressive / 4:4:4 ones on the host
        ok, f = cap.read()
        assert ok and np.array_equal(f, reference_decode((jp[8:12] + jp[28:32])[k])), k
    cap.release()


def test_stream_group_on_mjpeg(tmp_path):
    W, H, n, S = 320, 180, 24, 3
    srcs = [tmp_path / f"s{s}.avi" for s in range(S)]
    jps = [_mjpeg_avi(p, W, H, n, s, quality=80, subsampling=1) for s, p in enumerate(srcs)]
    grp = motion.StreamGroup([str(p) for p in srcs], batch=6, box_size=320, blur_scale=64, threshold=12,
                             cache_time=0.3, min_time=0.1, outdir=str(tmp_path))
    grp.find_motion()
    for s, v in enumerate(grp.videos):
        assert v.written_indices == _oracle_written(jps[s], W, H, 320), s


def test_read_frame_after_submit_and_submit_jpeg():
    W, H, S, T = 160, 96, 2, 3
    vids = [SyntheticVideo(W, H, s) for s in range(S)]
    kw = dict(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    eng = MotionEngine(**kw)
    frames = np.stack([np.stack([vids[s].frame(t) for s in range(S)]) for t in range(T)])
    eng.submit(frames)
    eng.wait()
    for t in range(T):
        for s in range(S):
            assert np.array_equal(eng.read_frame(t, s), frames[t, s])
    from find_motion_amd import MJpegDecoder
    dec = MJpegDecoder(W, H, max_frames=T * S)
    jp = [encode(vids[s].frame(T + t), quality=70) for t in range(T) for s in range(S)]
    eng.submit_jpeg(dec, jp)
    eng.wait()
    for t in range(T):
        for s in range(S):
            assert np.array_equal(eng.read_frame(t, s), reference_decode(jp[t * S + s]))
    dec.close()
    eng.close()


@pytest.mark.parametrize("codec", ["MJPG", "MP42"])
def test_cli_on_mjpeg_file(tmp_path, codec):
    """The reference CLI (python -m find_motion_amd FILE -o DIR, fm.py:1448-1489 flags and defaults:
    -B 100 -b 20 -t 12 -M 0.5 -C 1.0) on an MJPEG AVI: written frames = the oracle's on the decoded
    frames; an MJPG output holds the source's JPEG bytes, the default MP42 falls back to uncompressed
    AVI here (no cv2) with the decoded frames."""
    from find_motion_amd import cli
    W, H, n = 480, 270, 90
    src = tmp_path / "cam.avi"
    jp = _mjpeg_avi(src, W, H, n, 2, quality=80)
    out = tmp_path / "out"
    cli.main([str(src), "-o", str(out), "-I", "-k", codec, "--batch", "16"])
    st = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=100, ksize=5, thresh=12))
    want = written_indices([st.step(reference_decode(j))["count"] for j in jp], min_time=0.5, cache_time=1.0)
    assert want
    res = out / "cam.avi_1_motion.avi"
    if codec == "MJPG":
        assert _read_all(videoio.MjpegAviCapture(str(res))) == [jp[i] for i in want]
    else:
        got = _read_all(videoio.RawAviCapture(str(res)))
        assert len(got) == len(want)
        for g, i in zip(got, want):
            assert np.array_equal(g, reference_decode(jp[i])), i


def test_stream_group_mixed_chroma_sampling(tmp_path):
    """Same-size MJPEG streams with different chroma sampling (4:2:0 and 4:2:2) cannot share one GPU
    decode call: the feeder leaves JPEG mode and the captures decode frame by frame (on the GPU);
    decisions still equal the oracle's."""
    W, H, n = 320, 180, 24
    srcs = [tmp_path / "a.avi", tmp_path / "b.avi"]
    jps = [_mjpeg_avi(srcs[0], W, H, n, 0, quality=80), _mjpeg_avi(srcs[1], W, H, n, 1, quality=80, subsampling=1)]
    grp = motion.StreamGroup([str(p) for p in srcs], batch=6, box_size=320, blur_scale=64, threshold=12,
                             cache_time=0.3, min_time=0.1, outdir=str(tmp_path))
    grp.find_motion()
    for s, v in enumerate(grp.videos):
        assert v.written_indices == _oracle_written(jps[s], W, H, 320), s


def test_find_objects_reads_gpu_decoded_frames_in_place(tmp_path):
    """find_objects (fm.py:703-731) on an MJPEG frame whose batch is current: the cascade reads the
    decoded frame in the engine's input slot (fm_frame_device), raw is never fetched to the host,
    and the detections equal the oracle's on the libjpeg-turbo-decoded frame."""
    from find_motion_amd.cascade import to_xml
    from haar_cases import make_cascade
    from oracle import haar

    W, H, n = 640, 360, 16
    src = tmp_path / "v.avi"
    jp = _mjpeg_avi(src, W, H, n, 2, quality=90)
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    (tmp_path / "haarcascade_frontalface_default.xml").write_text(to_xml(cs))
    vm = motion.VideoMotion(filename=str(src), box_size=100, threshold=12, batch=8, outdir=str(tmp_path),
                            cascades=["frontalface_default"], cascade_dir=str(tmp_path))
    title = next(iter(vm.cascades))
    for i in range(15):
        assert vm.read()
        seen = vm.find_objects(minNeighbours=2)
    fr = vm.current_frame
    assert fr.index == 14 and fr._raw is None  # the 15th frame: detected in place, not fetched
    ref = haar.detect_multiscale(cs, oracle.resize_area_bgr(reference_decode(jp[14]), 300), 1.1, 2)
    assert seen == ({title} if ref else set())
    assert vm.last_objects.get(title, []) == [((x, y), (x + w, y + h)) for x, y, w, h in ref]
