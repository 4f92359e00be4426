"""GPU parity of the object-ROI stage (fm_haar_*) against
oracle/haar.py: the ungrouped candidate rects of detectMultiScaleNoGrouping and
the grouped detections must be identical (integer rects, same order).
Cascades and images are synthetic (tests/haar_cases.py); the reference's
cascade files are not on the GPU box.  Parity vs OpenCV itself: unpinned.
"""
import glob
import os

import numpy as np
import pytest

from find_motion_amd import CascadeClassifier
from haar_cases import make_cascade, make_image
import oracle
from oracle import haar

pytestmark = pytest.mark.gpu

CASES = [
    (1, 0.41, dict(depth=2)),                 # stumps + depth-2 trees, ~120 candidates
    (1, 0.38, dict(depth=2, tilted=True)),    # tilted features, ~2k candidates
    (3, 0.44, dict()),                        # stumps, ~9k candidates
    (3, 0.41, dict(tilted=True)),             # tilted stumps, ~12k candidates
    (1, 0.38, dict(stages=6, trees=6)),       # deeper cascade
    (1, 0.50, dict()),                        # rejects everything
]


@pytest.mark.parametrize("seed,tight,kw", CASES)
def test_candidates_and_groups_match_oracle(seed, tight, kw):
    cs = make_cascade(seed, tight=tight, **kw)
    img = make_image(2)
    det = CascadeClassifier(cs)
    got = det.detectMultiScale(img, scaleFactor=1.1, minNeighbors=5)
    cand = det.candidates()
    ref_c = haar.detect_candidates(cs, img, 1.1)
    assert [tuple(r) for r in cand.tolist()] == ref_c
    ref = haar.group_rectangles(ref_c, 5)
    assert [tuple(r) for r in np.asarray(got).reshape(-1, 4).tolist()] == ref
    det.close()


def test_batch_of_images_and_gray_input():
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    imgs = np.stack([make_image(s) for s in range(5)])
    det = CascadeClassifier(cs)
    got = det.detect_batch(imgs, 1.1, 3)
    for i in range(len(imgs)):
        ref = haar.detect_multiscale(cs, imgs[i], 1.1, 3)
        assert [tuple(r) for r in got[i].tolist()] == ref, i
    g = haar.bgr2gray(imgs[0])
    got1 = det.detect_batch(g[None], 1.1, 3)[0]
    assert [tuple(r) for r in got1.tolist()] == haar.detect_multiscale(cs, g, 1.1, 3)
    det.close()


@pytest.mark.parametrize("size,sf,mn,mins,maxs", [
    ((300, 169), 1.2, 2, (30, 30), (0, 0)),
    ((300, 169), 1.05, 5, (0, 0), (90, 90)),
    ((173, 97), 1.1, 0, (0, 0), (0, 0)),      # minNeighbors 0: raw candidates
    ((21, 20), 1.1, 1, (0, 0), (0, 0)),       # one window position
    ((19, 40), 1.1, 1, (0, 0), (0, 0)),       # narrower than the window: nothing
])
def test_sizes_scale_factors_and_limits(size, sf, mn, mins, maxs):
    cs = make_cascade(1, tight=0.41, depth=2)
    w, h = size
    img = make_image(7, w=max(w, 40), h=max(h, 40))[:h, :w]
    det = CascadeClassifier(cs)
    got = det.detectMultiScale(np.ascontiguousarray(img), scaleFactor=sf, minNeighbors=mn, minSize=mins, maxSize=maxs)
    ref = haar.detect_multiscale(cs, img, sf, mn, mins, maxs)
    assert [tuple(r) for r in np.asarray(got).reshape(-1, 4).tolist()] == ref
    det.close()


def _raw_frame(seed, W, H):
    small = make_image(seed, w=300, h=169)
    ys = (np.arange(H) * 169) // H
    xs = (np.arange(W) * 300) // W
    return np.ascontiguousarray(small[ys][:, xs])


@pytest.mark.parametrize("W,H", [(640, 360), (600, 338), (300, 169)])  # general INTER_AREA, exact 2x, identity
def test_detect_frames_resizes_on_device(W, H):
    # find_objects on raw frames: imutils.resize(raw, width=300) (INTER_AREA) on the device, then detection
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    raws = np.stack([_raw_frame(s, W, H) for s in range(3)])
    det = CascadeClassifier(cs)
    got = det.detect_frames(raws, 300, 1.1, 3)
    for i in range(len(raws)):
        roi = oracle.resize_area_bgr(raws[i], 300) if W != 300 else raws[i]
        assert roi.shape[:2] == (int(H * (300 / W)), 300)
        assert [tuple(r) for r in got[i].tolist()] == haar.detect_multiscale(cs, roi, 1.1, 3), i
    with pytest.raises(Exception):
        det.detect_frames(raws[:, :, :200], 300)  # narrower than the ROI: INTER_AREA upscaling unsupported
    det.close()


@pytest.mark.parametrize("W,H,roi_w", [(640, 360, 300),    # 6-tap INTER_AREA: read in place
                                        (1920, 1080, 300),  # 8 taps (find_objects on 1080p)
                                        (600, 338, 300),    # exact 2x: gathered, resizeAreaFast
                                        (300, 169, 300),    # identity: gathered
                                        (3840, 1280, 90)])  # 44 taps: gathered, the LDS-staged resize
def test_detect_frame_list_reads_frames_in_place(W, H, roi_w):
    """fm_haar_detect_frame_list: ROI frames at separate device addresses (out of order, in one big
    buffer with gaps, as find_objects collects them over streams and batches) give the detections of
    the contiguous call and of the restatement, on every resize path."""
    import torch
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    raws = np.stack([_raw_frame(s, W, H) for s in range(4)])
    det = CascadeClassifier(cs)
    ring = torch.zeros((9, H, W, 3), dtype=torch.uint8, device="cuda:0")
    slots = [7, 2, 5, 0]  # frame i lives in ring slot slots[i]
    for i, k in enumerate(slots):
        ring[k].copy_(torch.from_numpy(raws[i]))
    torch.cuda.synchronize()
    got = det.detect_frame_list([ring[k].data_ptr() for k in slots], H, W, roi_w, 1.1, 3)
    cont = det.detect_frames(raws, roi_w, 1.1, 3)
    for i in range(len(raws)):
        roi = oracle.resize_area_bgr(raws[i], roi_w) if W != roi_w else raws[i]
        ref = haar.detect_multiscale(cs, roi, 1.1, 3)
        assert [tuple(r) for r in got[i].tolist()] == ref, i
        assert [tuple(r) for r in cont[i].tolist()] == ref, i
    det.close()


def test_detect_frame_list_async_collect():
    """fm_haar_detect_frame_list_async + fm_haar_collect (the configs[4] bench's overlapped Haar stage):
    the same detections as the synchronous call and the restatement; a second queue before collecting is
    refused (FM_ESTATE); collect can be repeated with a larger cap; the synchronous call after an
    uncollected queue still returns its own results."""
    import torch

    from find_motion_amd import FMError
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    W, H = 1920, 1080
    raws = np.stack([_raw_frame(s, W, H) for s in range(4)])
    det = CascadeClassifier(cs)
    ring = torch.from_numpy(raws).to("cuda:0")
    torch.cuda.synchronize()
    ptrs = [ring[k].data_ptr() for k in (3, 1, 0, 2)]
    sync = det.detect_frame_list(ptrs, H, W, 300, 1.1, 3)
    assert det.detect_frame_list_async(ptrs, H, W, 300, 1.1, 3) == 4
    with pytest.raises(FMError):
        det.detect_frame_list_async(ptrs, H, W, 300, 1.1, 3)
    got = det.collect(4, cap=1)  # grows the cap and collects again
    again = det.collect(4)
    for i, k in enumerate((3, 1, 0, 2)):
        ref = haar.detect_multiscale(cs, oracle.resize_area_bgr(raws[k], 300), 1.1, 3)
        assert [tuple(r) for r in got[i].tolist()] == ref, i
        assert [tuple(r) for r in again[i].tolist()] == ref, i
        assert [tuple(r) for r in sync[i].tolist()] == ref, i
    det.detect_frame_list_async(ptrs[:2], H, W, 300, 1.1, 3)
    later = det.detect_frame_list(ptrs[2:], H, W, 300, 1.1, 3)  # finishes the queued call first
    for i, k in enumerate((0, 2)):
        assert [tuple(r) for r in later[i].tolist()] == haar.detect_multiscale(
            cs, oracle.resize_area_bgr(raws[k], 300), 1.1, 3), i
    det.close()


def test_detect_frames_device_input():
    # frames already resident in HBM (on_device = 1: no H2D copy) give the host path's and the
    # restatement's detections
    import torch
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    raws = np.stack([_raw_frame(s, 640, 360) for s in range(3)])
    det = CascadeClassifier(cs)
    dev = torch.from_numpy(raws).to("cuda:0")
    got = det.detect_frames(dev, 300, 1.1, 3)
    host = det.detect_frames(raws, 300, 1.1, 3)
    for i in range(len(raws)):
        ref = haar.detect_multiscale(cs, oracle.resize_area_bgr(raws[i], 300), 1.1, 3)
        assert [tuple(r) for r in got[i].tolist()] == ref, i
        assert [tuple(r) for r in host[i].tolist()] == ref, i
    with pytest.raises(ValueError):
        det.detect_frames(dev[:, :, ::2], 300)  # not contiguous
    det.close()

def test_video_motion_find_objects(tmp_path):
    # the drop-in loads haarcascade_<name>.xml from cascade_dir and runs find_objects every 15th frame
    from types import SimpleNamespace

    from find_motion_amd import motion, videoio
    from find_motion_amd.cascade import to_xml

    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    (tmp_path / "haarcascade_frontalface_default.xml").write_text(to_xml(cs))
    vm = motion.VideoMotion(filename=str(tmp_path / "v"), capture=videoio.SyntheticCapture(640, 360, 4, 0),
                            box_size=100, cascades=["frontalface_default", "fullbody"], cascade_dir=str(tmp_path),
                            outdir=str(tmp_path))
    assert list(vm.cascades) == ["Face 4"]  # fullbody has no file there: skipped with a warning
    fr = SimpleNamespace(raw=_raw_frame(0, 640, 360))
    for _ in range(14):
        assert vm.find_objects(fr) == set()
    seen = vm.find_objects(fr)
    roi = oracle.resize_area_bgr(fr.raw, 300)
    ref = haar.detect_multiscale(cs, roi, 1.1, 5)
    assert seen == ({"Face 4"} if ref else set())
    assert vm.last_objects.get("Face 4", []) == [((x, y), (x + w, y + h)) for x, y, w, h in ref]


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "haar_*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures_through_the_c_abi(path):
    from find_motion_amd.cascade import parse
    z = np.load(path)
    det = CascadeClassifier(parse(str(z["xml"])))
    got = det.detect_batch(z["image"][None], float(z["scale_factor"]), int(z["min_neighbors"]))[0]
    assert np.array_equal(det.candidates(), z["candidates"])
    assert np.array_equal(got, z["detections"])
    det.close()


def test_device_resident_images():
    # on_device = 1: images already in HBM (a decoder's buffer in production; hipMalloc here)
    import ctypes as C

    from find_motion_amd import _native
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    imgs = np.ascontiguousarray(np.stack([make_image(s) for s in range(3)]))
    det = CascadeClassifier(cs)
    hip = C.CDLL("libamdhip64.so")
    ptr = C.c_void_p()
    assert hip.hipMalloc(C.byref(ptr), C.c_size_t(imgs.nbytes)) == 0
    try:
        assert hip.hipMemcpy(ptr, C.c_void_p(imgs.ctypes.data), C.c_size_t(imgs.nbytes), 1) == 0  # H2D
        n, H, W = imgs.shape[:3]
        rects = np.zeros((n, 64, 4), np.int32)
        counts = np.zeros(n, np.int32)
        L = _native.load()
        rc = L.fm_haar_detect(det._h, ptr.value, n, H, W, 3, 1, 1.1, 3, 0, 0, 0, 0, rects.ctypes.data, 64,
                              counts.ctypes.data)
        assert rc == 0, L.fm_haar_last_error(det._h)
        for i in range(n):
            assert [tuple(r) for r in rects[i, :counts[i]].tolist()] == haar.detect_multiscale(cs, imgs[i], 1.1, 3)
    finally:
        hip.hipFree(ptr)
        det.close()


# --- the reference's own cascade (haarcascade_frontalface_default.xml, config 5) ----------------

def test_frontalface_roi_candidates_and_detections():
    from golden_cases import load_frontalface

    cs, z = load_frontalface()
    det = CascadeClassifier(cs)
    got = det.detectMultiScale(z["roi_image"], scaleFactor=1.1, minNeighbors=5)
    assert [tuple(r) for r in det.candidates().tolist()] == [tuple(int(v) for v in r) for r in z["roi_candidates"]]
    assert [tuple(r) for r in np.asarray(got).reshape(-1, 4).tolist()] == [tuple(int(v) for v in r)
                                                                          for r in z["roi_detections"]]
    det.close()


def test_frontalface_on_4k_frames_resized_on_device():
    """find_objects on config 5's 3840x2160 frames: INTER_AREA to width 300 on the device, then
    detectMultiScale(1.1, 5) with the real cascade, four frames per call."""
    from golden_cases import load_frontalface
    from haar_cases import FACE_FRAMES_4K, face_frame_4k

    cs, z = load_frontalface()
    frames = np.stack([face_frame_4k(i) for i in range(len(FACE_FRAMES_4K))])
    det = CascadeClassifier(cs)
    got = det.detect_frames(frames, 300, 1.1, 5)
    want = z["frames_detections_list"]
    assert [[tuple(int(v) for v in r) for r in np.asarray(g).reshape(-1, 4)] for g in got] == want
    assert sum(len(w) for w in want) == 6
    det.close()


def test_old_format_licence_plate_cascade():
    """The reference's one haartraining-format cascade (64x16 window, read as
    CascadeClassifier::convert rewrites it): candidates and detections equal the fixture's."""
    from golden_cases import load_licence_plate_old
    from haar_cases import plate_image

    cs, cases = load_licence_plate_old()
    det = CascadeClassifier(cs)
    for seed, cand, dets in cases:
        got = det.detectMultiScale(plate_image(seed), scaleFactor=1.1, minNeighbors=5)
        assert [tuple(r) for r in det.candidates().tolist()] == cand, seed
        assert [tuple(r) for r in np.asarray(got).reshape(-1, 4).tolist()] == dets, seed
    det.close()


def test_config5_workload_streams_masks_and_faces(tmp_path):
    """configs[4] as one workload: 4 streams of 3840x2160 through StreamGroup with -B 3840 -b 183 (k 21),
    the MASK_SCHEMA polygons and the frontalface_default cascade on every 15th written frame
    (find_motion.py:549-589, 703-731).  Written frames equal the decision restatement on oracle counts;
    the objects seen equal the fixture's detections of the 15th written frame of each stream."""
    from find_motion_amd import motion, videoio
    from find_motion_amd.cascade import to_xml
    from golden_cases import load_frontalface
    from haar_cases import FACE_FRAMES_4K, face_frame_4k
    from oracle.decision import written_indices

    cs, z = load_frontalface()
    (tmp_path / "haarcascade_frontalface_default.xml").write_text(to_xml(cs))
    uniq = [face_frame_4k(i) for i in range(len(FACE_FRAMES_4K))]
    S, n = 4, 20
    order = [[(s + t) % len(uniq) for t in range(n)] for s in range(S)]  # stream s cycles the frames from s
    masks = [((0, 0), (639, 359)), ((3839, 2159), (3200, 2159), (3839, 1600))]
    caps = [videoio.ArrayCapture([uniq[i] for i in order[s]]) for s in range(S)]
    grp = motion.StreamGroup([str(tmp_path / f"s{s}") for s in range(S)], batch=4, captures=caps, box_size=3840,
                             blur_scale=183, threshold=12, cache_time=0.3, min_time=0.1, mask_areas=masks,
                             cascades=["frontalface_default"], cascade_dir=str(tmp_path), outdir=str(tmp_path))
    res = grp.find_motion()
    cfg = oracle.OracleConfig(H=2160, W=3840, box=3840, ksize=21)
    keep = motion.rasterize_masks(2160, 3840, 1.0, masks)
    for s, v in enumerate(grp.videos):
        r = oracle.OracleStream(cfg, keep).run(np.stack([uniq[i] for i in order[s]]), nthreads=8)
        want = written_indices(list(r.counts), min_time=0.1, cache_time=0.3)
        assert v.written_indices == want, s
        # find_objects runs on every frame written as the current one (not on flushed cache frames)
        # and detects on its 15th call
        cur = written_indices(list(r.counts), min_time=0.1, cache_time=0.3, current_only=True)
        fifteenth = order[s][cur[14]] if len(cur) >= 15 else None
        seen = {"Face 4"} if fifteenth is not None and z["frames_detections_list"][fifteenth] else set()
        assert set(res[s][3]) == seen, (s, fifteenth)


def test_cascade_on_engine_frames_left_in_hbm():
    # find_objects on an MJPEG frame the engine decoded on the GPU (fm_frame_device): the cascade
    # reads the engine's input slot directly and finds what the host round trip and the oracle find
    from find_motion_amd import MJpegDecoder, MotionEngine
    from jpeg_cases import encode

    W, H, T, S = 640, 360, 3, 2
    cs = make_cascade(1, tight=0.38, depth=2, tilted=True)
    det = CascadeClassifier(cs)
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    dec = MJpegDecoder(W, H, max_frames=T * S)
    jp = [encode(_raw_frame(7 * t + s, W, H), quality=90) for t in range(T) for s in range(S)]
    eng.submit_jpeg(dec, jp)
    eng.wait()
    for t in range(T):
        for s in range(S):
            got = det.detect_frames((eng.frame_device_ptr(t, s), 1, H, W), 300, 1.1, 3)[0]
            raw = eng.read_frame(t, s)
            host = det.detect_frames(raw[None], 300, 1.1, 3)[0]
            ref = haar.detect_multiscale(cs, oracle.resize_area_bgr(raw, 300), 1.1, 3)
            assert [tuple(r) for r in got.tolist()] == ref, (t, s)
            assert [tuple(r) for r in host.tolist()] == ref, (t, s)
    with pytest.raises(Exception):
        eng.frame_device_ptr(T, 0)  # past the batch
    eng.close()
    det.close()
