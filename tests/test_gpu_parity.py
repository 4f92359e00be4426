"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): threshold/dilate masks bit-exact, background
within 1e-4 (it is in fact compared exactly here), contour count exact and
bounding boxes exact (the bar allows +-1 px).  Frames are the seeded
synthetic streams of find_motion_amd.synthetic; sizes are chosen so the
oracle finishes in seconds.
"""
import numpy as np
import pytest

import oracle
from find_motion_amd import MotionEngine, make_gaussian, rasterize_masks
from find_motion_amd._native import PLANE_BLUR, PLANE_DELTA, PLANE_GRAY
from find_motion_amd.synthetic import batch

pytestmark = pytest.mark.gpu


def _eq(got, ref, msg):
    if not np.array_equal(got, ref):
        bad = np.argwhere(got != ref)
        raise AssertionError(f"{msg}: {len(bad)} mismatches, first {bad[:16].tolist()} "
                             f"got {got[tuple(bad[:8].T)].tolist()} ref {ref[tuple(bad[:8].T)].tolist()}")


def run_pair(W, H, box, blur_scale=20, ksize=None, S=1, T=3, n_batches=2, thresh=12, alpha=0.1,
             masks=None, keep_planes=True, start=0, frames=None):
    k = ksize if ksize is not None else make_gaussian(box, blur_scale)
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=k, threshold=thresh, avg=alpha,
                       max_batch=T, keep_planes=keep_planes)
    h, w = eng.work_shape
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k, thresh=thresh, alpha=alpha)
    assert (cfg.h, cfg.w) == (h, w)
    keeps = [None] * S
    if masks:
        for s in range(S):
            keeps[s] = rasterize_masks(h, w, box / W, masks)
            eng.set_mask(s, keeps[s])
    orc = [oracle.OracleStream(cfg, keeps[s]) for s in range(S)]
    for b in range(n_batches):
        fr = frames[b] if frames is not None else batch(W, H, S, start + b * T, T)
        eng.submit(fr)
        eng.wait()
        counts = eng.counts()
        for t in range(fr.shape[0]):
            for s in range(S):
                ref = orc[s].step(fr[t, s])
                tag = f"batch {b} frame {t} stream {s}"
                if keep_planes:
                    _eq(eng.plane(PLANE_GRAY, t, s), ref["gray"], "gray " + tag)
                    _eq(eng.plane(PLANE_BLUR, t, s), ref["blur"], "blur " + tag)
                    _eq(eng.plane(PLANE_DELTA, t, s), ref["delta"], "delta " + tag)
                np.testing.assert_array_equal(eng.mask(t, s), ref["mask"], err_msg="mask " + tag)
                assert counts[t, s] == ref["count"], tag
                got = [c.bbox for c in eng.contours(t, s)]
                assert got == ref["boxes"], tag
                assert [c.origin for c in eng.contours(t, s)] == ref["origins"], tag
        for s in range(S):
            bg = eng.background(s)
            if not np.allclose(bg, orc[s].bg, rtol=0, atol=1e-4):
                bad = np.argwhere(np.abs(bg - orc[s].bg) > 1e-4)
                raise AssertionError(f"background batch {b} stream {s}: {len(bad)} bad, first {bad[:8].tolist()} "
                                     f"got {bg[tuple(bad[:8].T)].tolist()} ref {orc[s].bg[tuple(bad[:8].T)].tolist()}")
            assert np.array_equal(bg, orc[s].bg), "background not bit-identical"
    eng.close()


def test_mode_f_small():
    run_pair(160, 120, 160, blur_scale=32)  # k=5


def test_mode_d_640x480_config1():
    run_pair(640, 480, 100)  # 75x100, k=5: configs[0] geometry


def test_mode_d_1080p():
    run_pair(1920, 1080, 100, T=4, n_batches=2)


MASKS_1080 = [((0, 0), (639, 359)), ((1919, 1079), (1500, 1079), (1919, 700))]


@pytest.mark.parametrize("W,H,box,bs,S,T,nb,masks", [
    (1920, 1080, 100, 20, 1, 5, 3, None),        # mode D, the reference CLI default (-B 100 -b 20): k 5
    (1920, 1080, 100, 20, 1, 1, 4, None),        # one frame per batch (a first-frame launch, then singles)
    (640, 480, 100, 20, 2, 4, 3, None),          # configs[0] geometry 100 x 75: accumulateWeighted's tail
    (642, 481, 100, 20, 1, 3, 2, None),          # 100 x 74, 3*W % 4 == 2
    (1920, 1080, 100, 9, 1, 3, 2, None),         # k 11
    (1920, 1080, 100, 5, 1, 3, 2, None),         # k 21
    (1920, 1080, 100, 3, 1, 3, 2, None),         # k 33 (REFLECT_101 past the 56-row image's edge rows)
    (1920, 1080, 100, 20, 3, 3, 2, MASKS_1080),  # three streams with mask polygons
    (3840, 2160, 100, 20, 1, 2, 2, None),        # 4K -> 100 x 56 (the 40-tap LDS-staged resize)
    (1920, 1080, 128, 25, 1, 3, 2, None),        # 128 x 72: two tile rows and columns
    (337, 203, 100, 20, 2, 3, 2, None),          # odd source size, 100 x 60
])
def test_small_image_path_vs_oracle(W, H, box, bs, S, T, nb, masks):
    """The small-image path (fm_small.hip: every frame's gray / blur / keep-mask in parallel, then one wave
    per column scanning the frames with the f64 background in a register; the contour tile's column words
    by ballot) -- the product path for mode D -- against the oracle on every frame: masks, counts, boxes,
    origins and the background bit for bit."""
    run_pair(W, H, box, blur_scale=bs, S=S, T=T, n_batches=nb, masks=masks, keep_planes=False)


def test_mode_d_resize_paths():
    # staged INTER_AREA (3*W % 16 == 0) with a ragged last tap, the plain kernel (3*W % 16 != 0),
    # two streams through the resize stream
    run_pair(336, 200, 100, T=3, n_batches=2)
    run_pair(642, 481, 100, T=2, n_batches=2)
    run_pair(640, 480, 100, S=2, T=2, n_batches=2)


@pytest.mark.parametrize("W,H,box,S,T", [
    (1920, 1080, 100, 1, 5),   # mode D, the reference CLI default (-B 100): 22-tap register kernel
    (1920, 1080, 300, 2, 3),   # find_objects' ROI width (fm.py:706): 8 taps
    (3840, 2160, 300, 1, 2),   # config 5's ROI resize: 14 taps
    (3840, 2160, 100, 1, 2),   # 40 taps: past the register kernel, the LDS-staged one
    (640, 480, 100, 2, 3),     # configs[0] geometry: 8 taps
    (642, 481, 100, 1, 3),     # 3*W % 4 == 2: rows start at every byte alignment
    (337, 203, 100, 3, 2),     # odd width, ragged taps, three streams
    (101, 40, 100, 1, 4),      # scale just above 1: 2 taps, most of them partial
    (2000, 300, 7, 1, 2),      # one destination row, 287 taps a pixel
])
def test_resize_area_bytes_vs_oracle(W, H, box, S, T):
    """The INTER_AREA output itself (`small`, fm.py:490), every byte of every frame of every stream, against
    the oracle's restatement of cv2.resize(INTER_AREA): the tap order of each float chain is OpenCV's, so the
    bytes must be identical.  The last frame of the batch ends the input buffer, so the last columns' windows
    run past it (their out-of-range dwords carry zero weights)."""
    if int(H * (box / float(W))) < 1:
        pytest.skip("work height 0")
    from find_motion_amd._native import PLANE_SMALL
    k = make_gaussian(box, 20)
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=T)
    for b in range(2):
        fr = batch(W, H, S, 7 + b * T, T)
        eng.submit(fr)
        eng.wait()
        for t in range(T):
            for s in range(S):
                _eq(eng.plane(PLANE_SMALL, t, s), oracle.resize_area_bgr(fr[t, s], box), f"small b{b} t{t} s{s}")
    eng.close()


def test_resize_area_bytes_from_device_ring_end():
    """Device-resident input whose last frame ends exactly at the end of its allocation (the caller's ring,
    fm_submit on_device = 1): the windows of the last row's last columns reach past the allocation."""
    import torch

    from find_motion_amd._native import PLANE_SMALL
    W, H, box, T = 1920, 1080, 100, 4
    fr = batch(W, H, 1, 3, T)
    dev = torch.from_numpy(fr).to("cuda")
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=5, threshold=12, avg=0.1, max_batch=T)
    eng.submit_device(dev.data_ptr(), T)
    eng.wait()
    for t in range(T):
        _eq(eng.plane(PLANE_SMALL, t, 0), oracle.resize_area_bgr(fr[t, 0], box), f"small t{t}")
    eng.close()


def test_mode_f_1080p_k5():
    run_pair(1920, 1080, 1920, blur_scale=384, T=2, n_batches=2)


def test_fast_area_2x_and_4x():
    run_pair(160, 120, 80, blur_scale=20)   # 2x2 integer path, k=5
    run_pair(160, 120, 40, blur_scale=10)   # 4x4 integer path, k=5


def test_odd_sizes_and_large_k():
    run_pair(37, 23, 37, ksize=21)          # k larger than the image: REFLECT_101 repeats
    run_pair(101, 67, 101, ksize=9)
    run_pair(7, 5, 7, ksize=3)              # < 16 pixels: scalar convertScaleAbs / accumulate tails


def test_multi_stream_masks():
    masks = [((0, 0), (60, 40)), ((150, 110), (110, 119), (159, 80))]
    run_pair(160, 120, 160, blur_scale=32, S=3, T=2, masks=masks)


def test_4k_k21_masks_config5_geometry():
    masks = [((0, 0), (639, 359)), ((3839, 2159), (3200, 2159), (3839, 1600))]
    run_pair(3840, 2160, 3840, blur_scale=183, T=1, n_batches=2, masks=masks, keep_planes=False)


def test_k21_tall_bands_odd_tile_rows():
    """k = 21 on k_pixw's 128-row bands (a grid of >= 2048 tile-streams: 16 x 15 tiles x 9 streams): 15 tile
    rows, so the last band's second 64-row tile lies past the grid and its waves store nothing; masks on
    every stream, REFLECT_101 at the band edges."""
    masks = [((0, 0), (200, 150)), ((1023, 899), (700, 899), (1023, 600))]
    run_pair(1024, 900, 1024, ksize=21, S=9, T=2, n_batches=2, masks=masks, keep_planes=False, start=40)


@pytest.mark.parametrize("W,H,masks", [(256, 256, False), (252, 250, True)])
def test_k5_four_wave_tiles(W, H, masks):
    """k = 5 on k_pix5's 4-wave, 16-row tiles (a grid of >= 1,024 tile-streams: 64 streams x 16 tiles): without
    masks, and with masks on every stream plus accumulateWeighted's scalar tail (252 x 250: h*w % 16 = 8), a right
    tile 60 px wide and a bottom tile 58 rows tall (round 6)."""
    m = [((0, 0), (W // 5, H // 4)), ((W - 1, H - 1), (W // 2, H - 1), (W - 1, H // 2))] if masks else None
    run_pair(W, H, W, ksize=5, S=64, T=3, n_batches=2, masks=m, keep_planes=False, start=30)


def test_k21_bands_scalar_tail_and_masks():
    """k = 21 on 128-row bands (4 streams x 16 x 8 bands = 512) with accumulateWeighted's scalar tail
    (1000 x 901: h*w % 16 = 8), 15 tile rows (the last band's lower waves store nothing), masks (round 6)."""
    masks = [((0, 0), (200, 150)), ((999, 900), (700, 900), (999, 600))]
    run_pair(1000, 901, 1000, ksize=21, S=4, T=3, n_batches=2, masks=masks, keep_planes=False, start=60)


@pytest.mark.parametrize("W,H,S", [(200, 131, 2), (40, 30, 1), (1000, 70, 1), (320, 240, 3), (203, 90, 1)])
def test_k21_wide_kernel_geometries(W, H, S):
    """k = 21 steady state (k_pixw, no planes): a right tile 8 px wide, both REFLECT_101 edges in one tile
    (w = 40), accumulateWeighted's scalar tail (h*w % 16 != 0), several streams with masks; w = 203 (not a
    multiple of 4) takes k_pix<21>."""
    masks = [((0, 0), (W // 5, H // 4)), ((W - 1, H - 1), (W // 2, H - 1), (W - 1, H // 2))]
    run_pair(W, H, W, ksize=21, S=S, T=4, n_batches=2, masks=masks if S > 1 else None, keep_planes=False, start=90)


def test_thresholds_and_alpha():
    run_pair(160, 120, 160, blur_scale=32, thresh=0, alpha=0.5)
    run_pair(160, 120, 160, blur_scale=32, thresh=-1, alpha=0.02)
    run_pair(160, 120, 160, blur_scale=32, thresh=255, alpha=1.0)


def test_random_masks_contours():
    """Random binary-ish content with holes and nesting: stresses the CCL external test."""
    rng = np.random.default_rng(5)
    H, W = 96, 128
    fr = []
    for b in range(3):
        f = np.zeros((2, 1, H, W, 3), np.uint8)
        for t in range(2):
            img = (rng.random((H, W)) < 0.35).astype(np.uint8) * 255
            f[t, 0] = img[..., None]
        fr.append(f)
    run_pair(W, H, W, ksize=1, T=2, n_batches=3, thresh=20, alpha=0.5, frames=fr)


def _pattern_frames(patterns):
    """Frames whose dilated threshold mask is dilate(pattern): frame 0 is black
    (background init), every later frame is the pattern (ksize 1: no blur)."""
    H, W = patterns[0].shape
    fr = np.zeros((len(patterns) + 1, 1, H, W, 3), np.uint8)
    for i, p in enumerate(patterns):
        fr[i + 1, 0] = (p.astype(np.uint8) * 255)[..., None]
    return fr


def test_heavy_tiles_stripes_and_rings():
    """Tiles with > 256 runs (heavy CCL pass) and nested rings (external test)."""
    H, W = 150, 200
    stripes = np.zeros((H, W), bool)
    stripes[:, ::6] = True                      # dilates to 5-px bars with 1-px gaps: ~22 runs per row
    rings = np.zeros((H, W), bool)
    for k, (cy, cx) in enumerate([(40, 40), (75, 130), (120, 60)]):
        for rad in (30, 18, 8):
            yy, xx = np.ogrid[:H, :W]
            d = np.abs(np.hypot(yy - cy, xx - cx) - rad)
            rings |= d < 0.6
        rings[cy, cx] = True                    # a dot inside the innermost ring
    checker = np.zeros((H, W), bool)
    checker[::7, ::7] = True
    frames = _pattern_frames([stripes, rings, checker])
    run_pair(W, H, W, ksize=1, T=frames.shape[0], n_batches=1, thresh=100, alpha=0.5, frames=[frames])


def _convex_blobs(H, W, rng, n):
    """n random convex shapes (ellipses, rectangles, parallelograms, dots), some past the image edges: after the
    5x5 dilation most tiles they touch hold at most one foreground run per row (the contour pass's simple tiles),
    others two shapes side by side or stacked (the general run labelling)."""
    yy, xx = np.mgrid[:H, :W]
    p = np.zeros((H, W), bool)
    for _ in range(n):
        kind = rng.integers(4)
        cy, cx = rng.integers(-20, H + 20), rng.integers(-20, W + 20)
        if kind == 0:
            ry, rx = rng.integers(2, 70), rng.integers(2, 70)
            p |= ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1
        elif kind == 1:
            hy, hx = rng.integers(1, 60), rng.integers(1, 90)
            p |= (np.abs(yy - cy) <= hy) & (np.abs(xx - cx) <= hx)
        elif kind == 2:  # parallelogram: a slanted band of limited height
            slope, half, hy = rng.uniform(-3, 3), rng.integers(1, 12), rng.integers(5, 80)
            p |= (np.abs(xx - cx - slope * (yy - cy)) <= half) & (np.abs(yy - cy) <= hy)
        else:
            p[np.clip(cy, 0, H - 1), np.clip(cx, 0, W - 1)] = True
    return p


@pytest.mark.parametrize("W,H,seed", [(200, 150, 1), (200, 150, 2), (330, 260, 3), (330, 260, 4), (128, 64, 5)])
def test_simple_tiles_vs_oracle(W, H, seed):
    """Convex blobs whose tiles mostly hold one foreground run per row -- the contour pass's simple-tile path
    (one component, background chains left and right of it, top and bottom regions, tiles cut by the image's
    right / bottom edge) -- and mixes with two shapes per tile (the general labelling), on both contour pass
    layouts (12 / 2 tiles: one workgroup per frame; 30 tiles: the kernel chain), against the oracle."""
    rng = np.random.default_rng(seed)
    pats = [_convex_blobs(H, W, rng, n) for n in (1, 2, 3, 5, 8)]
    frames = _pattern_frames(pats)
    run_pair(W, H, W, ksize=1, T=frames.shape[0], n_batches=1, thresh=100, alpha=0.5, frames=[frames])


def _streak_rows(H, W, rng, maxruns, maxlen=23):
    """Streaks of identical rows (1..maxlen rows each, 0..maxruns random runs per row, some past the image edges):
    after the dilation most tiles hold several runs per row, holes and separate components, but few distinct
    rows -- the contour pass's compact tiles (one lane per run of the distinct rows); the busiest exceed 64
    such runs and take the row-per-lane labelling."""
    p = np.zeros((H, W), bool)
    y = 0
    while y < H:
        n = int(rng.integers(1, maxlen + 1))
        row = np.zeros(W, bool)
        for _ in range(int(rng.integers(0, maxruns + 1))):
            x, ln = int(rng.integers(-10, W)), int(rng.integers(1, 80))
            row[max(x, 0):max(x + ln, 0)] = True
        p[y:y + n] = row
        y += n
    return p


@pytest.mark.parametrize("W,H,seed", [(200, 150, 11), (330, 260, 12), (330, 260, 13), (128, 64, 14), (700, 300, 15)])
def test_compact_tiles_vs_oracle(W, H, seed):
    """Tiles with few distinct rows (streaks of repeated rows with several runs each: holes, nested and side-by-side
    components, background regions split by them, rows cut by the image's right / bottom edge), on both contour
    pass layouts, against the oracle; the denser patterns exceed 64 runs and cover the fallback labelling too."""
    rng = np.random.default_rng(seed)
    pats = [_streak_rows(H, W, rng, r) for r in (1, 2, 3, 4, 6, 8)] + [_streak_rows(H, W, rng, 6, maxlen=2)]
    frames = _pattern_frames(pats)
    run_pair(W, H, W, ksize=1, T=frames.shape[0], n_batches=1, thresh=100, alpha=0.5, frames=[frames])


@pytest.mark.parametrize("k", [1, 5])
@pytest.mark.parametrize("W,H", [(320, 256), (300, 204)])
def test_full_tiles(W, H, k):
    """Tiles whose dilated mask is all set take the contour pass's closed-form record: full tiles on
    the left image edge (outer reference) and inside the image (edge reference), next to holes,
    diagonal neighbours, a whole-frame foreground (edge tiles cut by the image never count as full)."""
    pats = []
    p = np.zeros((H, W), bool)
    p[10:H - 6, 0:W - 20] = True
    p[100:120, 150:170] = False                 # a hole inside the block ...
    p[110, 160] = True                          # ... with a dot in it
    pats.append(p)
    pats.append(np.ones((H, W), bool))
    p = np.zeros((H, W), bool)
    p[2:62, 2:62] = True                        # dilates to exactly tile (0, 0)
    p[66:126, 66:126] = True                    # and tile (1, 1): corner-to-corner neighbours
    p[130:190, 200:W - 1] = True
    pats.append(p)
    p = np.zeros((H, W), bool)
    p[64:192, 64:256] = True                    # full tiles away from the image edge
    p[5, 5] = True
    pats.append(p)
    frames = _pattern_frames(pats)
    run_pair(W, H, W, ksize=k, T=frames.shape[0], n_batches=1, thresh=100, alpha=0.5, frames=[frames])


# --- committed golden fixtures through the C ABI -------------------------------

from golden_cases import boxes_of, chain_files, contour_cases, load_chain, origins_of  # noqa: E402


@pytest.mark.parametrize("path", chain_files(), ids=lambda p: p.rsplit("/", 1)[-1])
@pytest.mark.parametrize("batch", [1, 0])  # 1 frame per submit, or the whole sequence in one launch
def test_golden_chain_fixture(path, batch):
    c = load_chain(path)
    T = c["T"] if batch == 0 else batch
    eng = MotionEngine(n_streams=1, src_w=c["W"], src_h=c["H"], box_size=c["box"], ksize=c["ksize"],
                       threshold=c["thresh"], avg=c["alpha"], max_batch=T, keep_planes=True)
    if c["has_keep"]:
        eng.set_mask(0, c["keep"])
    for t0 in range(0, c["T"], T):
        fr = c["frames"][t0:t0 + T]
        eng.submit(fr[:, None])
        eng.wait()
        counts = eng.counts()
        for i in range(fr.shape[0]):
            t = t0 + i
            for plane, name in ((PLANE_GRAY, "gray"), (PLANE_BLUR, "blur"), (PLANE_DELTA, "delta")):
                np.testing.assert_array_equal(eng.plane(plane, i, 0), c[name][t], err_msg=f"{name} frame {t}")
            np.testing.assert_array_equal(eng.mask(i, 0), c["mask"][t], err_msg=f"mask frame {t}")
            assert counts[i, 0] == c["count"][t]
            assert [x.bbox for x in eng.contours(i, 0)] == boxes_of(c, t)
            assert [x.origin for x in eng.contours(i, 0)] == origins_of(c, t)
    np.testing.assert_array_equal(eng.background(0), c["bg"])
    eng.close()


@pytest.mark.parametrize("name", sorted(contour_cases()))
def test_golden_contour_fixture(name):
    """The fixture pattern enters as frame 1 after a black frame 0 (ksize 1, threshold 0), so the
    threshold mask is the pattern and the kernel dilates it; the GPU's contours of the dilated pattern
    are compared with the oracle's."""
    case = contour_cases()[name]
    m = case["mask"]
    H, W = m.shape
    fr = np.zeros((2, 1, H, W, 3), np.uint8)
    fr[1, 0] = m[..., None]
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.5, max_batch=2)
    eng.submit(fr)
    eng.wait()
    d = oracle.dilate5(m)
    np.testing.assert_array_equal(eng.mask(1, 0), d)
    want = oracle.find_contours_ext(d)
    assert eng.counts()[1, 0] == len(want)
    assert [c.bbox for c in eng.contours(1, 0)] == [c["bbox"] for c in want]
    eng.close()


# --- the drop-in VideoMotion on the real engine ---------------------------------

@pytest.mark.parametrize("batch", [1, 8])
def test_video_motion_dropin_decisions(tmp_path, batch):
    from find_motion_amd import motion, videoio
    from oracle.decision import written_indices

    W, H, n = 480, 270, 48
    vm = motion.VideoMotion(filename=str(tmp_path / "v"), capture=videoio.SyntheticCapture(W, H, n, 0),
                            box_size=100, threshold=12, cache_time=0.3, min_time=0.1, batch=batch,
                            outdir=str(tmp_path))
    vm.find_motion()
    cfg = oracle.OracleConfig(H=H, W=W, box=100, ksize=5)
    st = oracle.OracleStream(cfg)
    vid = videoio.SyntheticCapture(W, H, n, 0).video
    counts = [st.step(vid.frame(i))["count"] for i in range(n)]
    assert vm.written_indices == written_indices(counts, min_time=0.1, cache_time=0.3)
    assert vm.written_indices


def test_stream_group_on_gpu(tmp_path):
    from find_motion_amd import motion, videoio
    from oracle.decision import written_indices

    W, H, n, S = 320, 180, 24, 4
    caps = [videoio.SyntheticCapture(W, H, n, s) for s in range(S)]
    grp = motion.StreamGroup([str(tmp_path / f"s{s}") for s in range(S)], batch=6, captures=caps, box_size=320,
                             blur_scale=64, threshold=12, cache_time=0.3, min_time=0.1, outdir=str(tmp_path))
    grp.find_motion()
    cfg = oracle.OracleConfig(H=H, W=W, box=320, ksize=5)
    for s, v in enumerate(grp.videos):
        st = oracle.OracleStream(cfg)
        vid = videoio.SyntheticCapture(W, H, n, s).video
        counts = [st.step(vid.frame(i))["count"] for i in range(n)]
        assert v.written_indices == written_indices(counts, min_time=0.1, cache_time=0.3), s


@pytest.mark.parametrize("k", [3, 5, 7, 21])
def test_convert_scale_abs_ties_and_saturation(k):
    """Background values on exact .5 ties, just off them, negative and > 255 (convertScaleAbs, fm.py:250):
    the GPU's f64 -> f32 -> rne -> saturate chain and the accumulate must match the oracle bit for bit."""
    W, H = 96, 40
    rng = np.random.default_rng(k)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=k, threshold=1, avg=0.25, max_batch=1,
                       keep_planes=True)
    base = np.floor(rng.random((H, W)) * 300 - 20)
    frac = rng.choice([0.5, -0.5, 0.4999999999, 0.5000000001, 0.25, 0.0, 1.5, 2.5], size=(H, W))
    bg = base + frac
    bg[0, :8] = [-0.5, -1.5, 255.5, 256.5, 254.5, 0.5, 1e9, -1e9]
    eng.set_background(0, bg)
    fr = np.repeat(rng.integers(0, 256, (1, 1, H, W, 1), dtype=np.uint8), 3, axis=-1)
    eng.submit(fr)
    eng.wait()
    blur = oracle.gauss_blur(oracle.bgr2gray(fr[0, 0]), k)
    np.testing.assert_array_equal(eng.plane(PLANE_BLUR, 0, 0), blur)
    delta, th = oracle.diff_thresh(blur, bg, 1)
    np.testing.assert_array_equal(eng.plane(PLANE_DELTA, 0, 0), delta)
    np.testing.assert_array_equal(eng.mask(0, 0), oracle.dilate5(th))
    ref = bg.copy()
    oracle.accumulate(blur, ref, 0.25)
    np.testing.assert_array_equal(eng.background(0), ref)
    eng.close()


@pytest.mark.parametrize("W,H", [(1920, 1080), (100, 56), (203, 131), (64, 64), (65, 1)])
def test_batch_split_and_tail_geometries(W, H):
    """Odd sizes exercise the partial tiles, the unaligned-row gray path, reflected borders and
    accumulateWeighted's scalar tail (h*w % 16 != 0); batch of 5 includes the init frame launch."""
    run_pair(W, H, W, ksize=5, T=5, n_batches=2, keep_planes=False)


def test_batches_in_flight_match_sequential():
    """fm_submit of later batches before fm_wait of batch i (the pipelined mode): each wait completes the
    oldest batch, results and background match the oracle run frame by frame; one submit beyond
    fm_max_inflight is refused."""
    W, H, S, T = 320, 180, 2, 3
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T,
                       keep_planes=True)
    cfg = oracle.OracleConfig(H=H, W=W, box=W, ksize=5)
    orc = [oracle.OracleStream(cfg) for _ in range(S)]
    depth = eng.max_inflight
    assert depth >= 2
    NB = depth + 2  # the last two batches reuse slots
    batches = [batch(W, H, S, 90 + T * b, T) for b in range(NB)]
    for b in range(depth):
        eng.submit(batches[b])
    with pytest.raises(Exception):
        eng.submit(batches[0])  # all slots in flight
    for b in range(NB):
        eng.wait()
        counts = eng.counts()
        for t in range(T):
            for s in range(S):
                ref = orc[s].step(batches[b][t, s])
                assert counts[t, s] == ref["count"]
                assert [c.bbox for c in eng.contours(t, s)] == ref["boxes"]
                np.testing.assert_array_equal(eng.mask(t, s), ref["mask"])
                np.testing.assert_array_equal(eng.plane(PLANE_BLUR, t, s), ref["blur"])
        if b + depth < NB:  # reuses batch b's slot: its device-side results are gone after this
            eng.submit(batches[b + depth])
    for s in range(S):
        np.testing.assert_array_equal(eng.background(s), orc[s].bg)
    eng.close()


def test_pinned_host_buffers_match_pageable():
    # page-locked batches (fm_host_alloc, DMA on the input stream) give the same results
    # as pageable numpy batches, with batches in flight
    W, H = 320, 240
    fr = batch(W, H, 2, 0, 6)
    results = []
    for pinned in (False, True):
        eng = MotionEngine(n_streams=2, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=3)
        bufs = []
        for b in range(2):
            if pinned:
                pb = eng.host_buffer(3)
                pb[:] = fr[3 * b:3 * b + 3]
                bufs.append(pb)
            else:
                bufs.append(np.ascontiguousarray(fr[3 * b:3 * b + 3]))
        out = []
        for b in range(2):
            eng.submit(bufs[b])
        for b in range(2):
            eng.wait()
            out.append((eng.counts().copy(), [eng.mask(t, s).copy() for t in range(3) for s in range(2)]))
        results.append(out)
        eng.close()
    for (ca, ma), (cb, mb) in zip(results[0], results[1]):
        assert np.array_equal(ca, cb)
        assert all(np.array_equal(x, y) for x, y in zip(ma, mb))


def test_batch128_matches_oracle():
    # the bench default batch: 128 frames per pixel-kernel launch, two batches, against the oracle
    run_pair(320, 180, 320, ksize=5, S=2, T=128, n_batches=2, keep_planes=False)


def test_batch_size_invariance_1080p():
    # full-size size-independent property: one 128-frame launch == two 64-frame launches
    # (counts, contours, masks of sampled frames, background bit-identical)
    W, H, N = 1920, 1080, 128
    fr = batch(W, H, 1, 0, N)
    out = []
    for T in (128, 64):
        eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
        counts, boxes, masks = [], [], []
        for b in range(N // T):
            eng.submit(fr[b * T:(b + 1) * T])
            eng.wait()
            c = eng.counts()
            for t in range(T):
                counts.append(int(c[t, 0]))
                boxes.append([x.bbox for x in eng.contours(t, 0)])
                if (b * T + t) % 17 == 0:
                    masks.append(eng.mask(t, 0).copy())
        out.append((counts, boxes, masks, eng.background(0).copy()))
        eng.close()
    (ca, ba, ma, ga), (cb, bb, mb, gb) = out
    assert ca == cb and ba == bb
    assert all(np.array_equal(x, y) for x, y in zip(ma, mb))
    assert np.array_equal(ga, gb)
    assert sum(ca) > 0


def test_bench_shape_in_flight_matches_oracle():
    """bench.py's exact shape (configs[1], mode F): 1080p, k 5, 256-frame launches of the production
    k_pix5 (no planes), two batches in flight before the first wait, every frame's count, boxes and
    origins against the oracle, sampled masks, and the final background bit for bit."""
    W, H, T, NB = 1920, 1080, 256, 2
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    assert eng.max_inflight >= NB
    frs = [batch(W, H, 1, b * T, T) for b in range(NB)]
    for fr in frs:
        eng.submit(fr)
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=5, thresh=12, alpha=0.1))
    total = 0
    for b in range(NB):
        eng.wait()
        counts = eng.counts()
        for t in range(T):
            ref = orc.step(frs[b][t, 0])
            tag = f"batch {b} frame {t}"
            assert counts[t, 0] == ref["count"], tag
            assert [c.bbox for c in eng.contours(t, 0)] == ref["boxes"], tag
            assert [c.origin for c in eng.contours(t, 0)] == ref["origins"], tag
            if t % 32 == 0:
                np.testing.assert_array_equal(eng.mask(t, 0), ref["mask"], err_msg="mask " + tag)
            total += ref["count"]
    assert np.array_equal(eng.background(0), orc.bg), "background not bit-identical"
    assert total > 0
    eng.close()
