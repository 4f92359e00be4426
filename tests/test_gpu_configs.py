"""GPU parity at the BASELINE configurations and on the product paths the small
cases do not reach, against the CPU oracle (oracle.OracleStream.run: the same
arithmetic as step(), frames scheduled in parallel where find_diff's data flow
allows, so full-size sequences finish in seconds).

* the bench workload itself: 1080p, mode F, T = 256 frames per launch from a
  256-frame device-resident ring cycling 64 synthetic frames, the production
  k_pix5 (no planes kept), fm_max_inflight (10) batches submitted before the
  first wait, 12 batches so that slots are reused;
* configs[2]: 8 x 1080p streams on one GPU, batches in flight -- also at the
  perf shape quoted for it (T = 128 per launch, 4 in flight, 7 batches, device ring) and every slot reused
  at 32 frames per launch;
* configs[4] geometry: 4 x 3840x2160 streams, -B 3840 -b 183 (k 21), the two
  MASK_SCHEMA polygons (find_motion.py:86-100) -- also at its perf shape
  (T = 64, 2 in flight);
* more contours than max_contours (a dot lattice: every contour counted and
  kept, in raster order, fm.py:674-694), heavy tiles, and the pixel-level
  fallback once a batch exhausts its node pool;
* k = 97 (-B 1920 -b 20, fm.py:478-484: the per-frame k_pixel path) and k_fused
  at k 11, 33, 49.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle
from find_motion_amd import MotionEngine, make_gaussian, rasterize_masks
from find_motion_amd.synthetic import batch

pytestmark = pytest.mark.gpu

CONFIG5_MASKS = [((0, 0), (639, 359)), ((3839, 2159), (3200, 2159), (3839, 1600))]


def _check_frame(eng, res, t, s, f, tag, mask=True):
    """Engine results (batch frame t, stream s) against oracle result res (sequence frame f)."""
    got = eng.contours(t, s)
    assert eng.counts()[t, s] == res.counts[f], f"count {tag}"
    assert len(got) == res.counts[f], f"len(contours) {tag}"
    assert [c.bbox for c in got] == res.boxes(f), f"boxes {tag}"
    assert [c.origin for c in got] == res.origins(f), f"origins {tag}"
    if mask and f in res.masks:
        np.testing.assert_array_equal(eng.mask(t, s), res.masks[f], err_msg=f"mask {tag}")


def test_bench_shape_inflight_ring_wrap():
    """bench.py's exact workload (its defaults: --batch 256 --ring 256 --ring-period 64, max_contours 1 << 14,
    fm_max_inflight batches submitted before the first wait) through the production kernel, against the
    oracle on every frame: 256-frame launches from a 256-frame device ring cycling 64 synthetic frames, ten
    batches in flight, twelve batches so that two slots are reused, node pools sized for 256 frames."""
    torch = pytest.importorskip("torch")
    W, H, T, PERIOD = 1920, 1080, 256, 64
    uniq = batch(W, H, 1, 0, PERIOD)                   # bench: ring slot t holds synthetic frame t % 64
    ring_h = np.concatenate([uniq] * (T // PERIOD))    # [256][1][H][W][3]
    ring = torch.from_numpy(ring_h).to("cuda:0")
    torch.cuda.synchronize()
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T,
                       max_contours=1 << 14)
    assert not eng.keep_planes
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=5))
    depth = eng.max_inflight
    assert depth == 10
    NB = depth + 2                                     # two batches onto reused slots
    for b in range(depth):
        eng.submit_device(ring.data_ptr(), T)
    total = 0
    for b in range(NB):
        res = orc.run(ring_h[:, 0], mask_frames=range(b % 7, T, 23))
        eng.wait()
        for t in range(T):
            _check_frame(eng, res, t, 0, t, f"batch {b} frame {t}")
        total += int(res.counts.sum())
        if b + depth < NB:                             # slot of batch b reused: the ring wrap
            eng.submit_device(ring.data_ptr(), T)
    np.testing.assert_array_equal(eng.background(0), orc.bg)
    assert total > 0
    eng.close()


def test_mode_d_bench_shape_inflight_ring_wrap():
    """bench.py's mode D side leg (`--mode D`: -B 100 -b 20, the reference CLI's default; 256-frame launches
    from the same device ring, fm_max_inflight batches in flight, two slots reused) through the product path
    for small work images -- the INTER_AREA resize, k_small_blur + k_small_scan, k_frame_contours -- against
    the oracle on every frame, and the final background."""
    torch = pytest.importorskip("torch")
    W, H, T, PERIOD = 1920, 1080, 256, 64
    uniq = batch(W, H, 1, 0, PERIOD)
    ring_h = np.concatenate([uniq] * (T // PERIOD))
    ring = torch.from_numpy(ring_h).to("cuda:0")
    torch.cuda.synchronize()
    k = make_gaussian(100, 20)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=100, ksize=k, threshold=12, avg=0.1, max_batch=T,
                       max_contours=1 << 14, profile="pix")
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=100, ksize=k))
    depth = eng.max_inflight
    NB = depth + 2
    for b in range(depth):
        eng.submit_device(ring.data_ptr(), T)
    total = 0
    for b in range(NB):
        res = orc.run(ring_h[:, 0], mask_frames=range(b % 5, T, 17))
        eng.wait()
        for t in range(T):
            _check_frame(eng, res, t, 0, t, f"batch {b} frame {t}")
        total += int(res.counts.sum())
        if b + depth < NB:
            eng.submit_device(ring.data_ptr(), T)
    np.testing.assert_array_equal(eng.background(0), orc.bg)
    assert total > 0
    assert "small_scan" in {n for n, (ms, c) in eng.kernel_times().items() if c > 0}
    eng.close()


def _run_streams(W, H, box, k, S, T, NB, masks=None, start=0, mask_every=7, threads=4):
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=T)
    h, w = eng.work_shape
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k)
    keeps = [None] * S
    if masks:
        for s in range(S):
            keeps[s] = rasterize_masks(h, w, box / W, masks)
            eng.set_mask(s, keeps[s])
    orc = [oracle.OracleStream(cfg, keeps[s]) for s in range(S)]
    batches = [batch(W, H, S, start + b * T, T) for b in range(NB)]
    depth = min(eng.max_inflight, NB)
    for b in range(depth):
        eng.submit(batches[b])
    pool = ThreadPoolExecutor(S)
    for b in range(NB):
        fr = batches[b]
        res = list(pool.map(lambda s: orc[s].run(fr[:, s], mask_frames=range(s % mask_every, T, mask_every),
                                                 nthreads=threads), range(S)))
        eng.wait()
        for s in range(S):
            for t in range(T):
                _check_frame(eng, res[s], t, s, t, f"batch {b} frame {t} stream {s}")
        if b + depth < NB:
            eng.submit(batches[b + depth])
    for s in range(S):
        np.testing.assert_array_equal(eng.background(s), orc[s].bg, err_msg=f"background stream {s}")
    pool.shutdown()
    eng.close()


def test_config3_eight_1080p_streams_inflight():
    """configs[2]: 8 x 1080p streams batched on one GPU, per-stream background, 7 batches of 8 frames
    (6 in flight, one slot reused)."""
    _run_streams(1920, 1080, 1920, 5, S=8, T=8, NB=7, start=40, threads=2)


def test_config5_four_4k_streams_k21_masks():
    """configs[4] geometry: 4 x 3840x2160, -B 3840 -b 183 -> k 21, MASK_SCHEMA rect + triangle."""
    k = make_gaussian(3840, 183)
    assert k == 21
    _run_streams(3840, 2160, 3840, k, S=4, T=3, NB=2, masks=CONFIG5_MASKS, start=10, mask_every=2)


def _run_ring(W, H, box, k, S, T, NB, depth, period, masks=None, mask_every=23, threads=2):
    """bench.py's loop at a BASELINE config's quoted perf shape: a [T][S] device-resident ring cycling `period`
    synthetic frames per stream, `depth` batches submitted before the first wait, NB batches (slots reused),
    every frame of every stream against the oracle (counts, boxes, start pixels; sampled masks), then the
    final backgrounds."""
    torch = pytest.importorskip("torch")
    uniq = batch(W, H, S, 0, period)
    ring_h = np.concatenate([uniq] * (T // period)) if T > period else uniq[:T]
    assert ring_h.shape[0] == T
    ring = torch.from_numpy(ring_h).to("cuda:0")
    torch.cuda.synchronize()
    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=T,
                       max_contours=1 << 14)
    assert not eng.keep_planes and depth <= eng.max_inflight
    h, w = eng.work_shape
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k)
    keeps = [None] * S
    if masks:
        for s in range(S):
            keeps[s] = rasterize_masks(h, w, box / W, masks)
            eng.set_mask(s, keeps[s])
    orc = [oracle.OracleStream(cfg, keeps[s]) for s in range(S)]
    for _ in range(depth):
        eng.submit_device(ring.data_ptr(), T)
    pool = ThreadPoolExecutor(S)
    total = 0
    for b in range(NB):
        res = list(pool.map(lambda s: orc[s].run(ring_h[:, s], cap=1 << 14,
                                                 mask_frames=range((b + 3 * s) % mask_every, T, mask_every),
                                                 nthreads=threads), range(S)))
        eng.wait()
        for s in range(S):
            for t in range(T):
                _check_frame(eng, res[s], t, s, t, f"batch {b} frame {t} stream {s}")
            total += int(res[s].counts.sum())
        if b + depth < NB:
            eng.submit_device(ring.data_ptr(), T)
    for s in range(S):
        np.testing.assert_array_equal(eng.background(s), orc[s].bg, err_msg=f"background stream {s}")
    assert total > 0
    pool.shutdown()
    eng.close()


@pytest.mark.timeout(400)
def test_config3_perf_shape_eight_streams_t128():
    """configs[2] at the shape its throughput is quoted on (bench.py --streams 8 --batch 128): 8 x 1080p
    streams, 128 frames per stream per launch, 4 batches in flight, 7 batches."""
    _run_ring(1920, 1080, 1920, 5, S=8, T=128, NB=7, depth=4, period=64)


@pytest.mark.timeout(400)
def test_eight_streams_slot_reuse():
    """8 x 1080p streams through every batch slot and round again (fm_max_inflight + 2 batches of 32 frames per
    stream, 4 in flight): the slots' node pools, records and counters re-armed between batches."""
    eng = MotionEngine(n_streams=1, src_w=64, src_h=64, box_size=64, ksize=5, threshold=12, avg=0.1, max_batch=1)
    nb = eng.max_inflight + 2
    eng.close()
    _run_ring(1920, 1080, 1920, 5, S=8, T=32, NB=nb, depth=4, period=32)


@pytest.mark.timeout(400)
def test_config5_perf_shape_four_4k_streams_t64():
    """configs[4] geometry at its quoted perf shape (bench.py --width 3840 --height 2160 --blur-scale 183
    --streams 4 --batch 64): k 21, the MASK_SCHEMA polygons, 64 frames per stream per launch, 2 batches in
    flight, 3 batches."""
    k = make_gaussian(3840, 183)
    _run_ring(3840, 2160, 3840, k, S=4, T=64, NB=3, depth=2, period=16, masks=CONFIG5_MASKS, threads=4)


def _lattice_frames(H, W, pitch, n, offset=0):
    """Frame 0 black (background init), then n frames of single-pixel dots on a pitch grid:
    dilated 5x5 with 1-px gaps at pitch 6, one contour per dot (ksize 1, threshold 0)."""
    fr = np.zeros((n + 1, 1, H, W, 3), np.uint8)
    for i in range(n):
        o = (offset + i) % pitch
        fr[i + 1, 0, o::pitch, o::pitch] = 255
    return fr


@pytest.mark.parametrize("cap", [4096, 100])
def test_contours_past_max_contours(cap):
    """A 1080p dot lattice (~57,600 contours per frame, every tile heavy): the count and every record
    are exact whatever max_contours is, records in raster order of their start pixels."""
    H, W = 1080, 1920
    fr = _lattice_frames(H, W, 6, 2)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.5,
                       max_batch=fr.shape[0], max_contours=cap)
    eng.submit(fr)
    eng.wait()
    assert eng.fallbacks() == 0
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=1, thresh=0, alpha=0.5))
    res = orc.run(fr[:, 0], cap=1 << 17, mask_frames=[1, 2])
    assert res.counts[1] > 50000
    for t in range(fr.shape[0]):
        _check_frame(eng, res, t, 0, t, f"frame {t}")
    eng.close()


def test_node_pool_exhaustion_falls_back_to_pixel_ccl():
    """32 dense-lattice frames in one batch (~107 components per tile-frame) need more union-find nodes
    than the slot's pool holds (64 per tile-frame on average): the frames that fail to get nodes are
    relabelled by the pixel-level CCL in fm_wait (fm_kernels.hip) -- every frame still equals the oracle."""
    H, W = 540, 960
    fr = _lattice_frames(H, W, 6, 32, offset=1)
    # avg 0: the background stays black, so every frame's threshold mask is its own lattice
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.0,
                       max_batch=fr.shape[0], max_contours=512)
    eng.submit(fr)
    eng.wait()
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=1, thresh=0, alpha=0.0))
    res = orc.run(fr[:, 0], cap=1 << 16, mask_frames=range(fr.shape[0]))
    assert res.counts[1:].min() > 10000
    assert eng.fallbacks() > 0  # all frames allocate concurrently, so typically every one of them
    for t in range(fr.shape[0]):
        _check_frame(eng, res, t, 0, t, f"frame {t}")
    eng.close()


@pytest.mark.parametrize("depth", [1, 4])
def test_frame_contour_pass_pool_heavy_tiles_and_slot_reuse(depth):
    """Work images of at most 16 tiles run the whole contour pass of a frame in one workgroup
    (k_frame_contours, fm_ccl.hip).  A 200 x 150 dot lattice (12 tiles, ~825 contours per frame, every
    tile heavy: ~1,100 runs) overflows each frame's node quota into the slot's shared pool, and the heavy
    tiles run in the workgroup's own LDS; 14 batches of 16 frames reuse the 10 slots, so a pool word not
    re-armed after a batch would exhaust the pool (fallbacks); depth 4 keeps batches in flight."""
    H, W, T, NB = 150, 200, 16, 14
    seq = _lattice_frames(H, W, 6, T * NB - 1, offset=1)  # frame 0 black; avg 0 keeps the background black
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.0,
                       max_batch=T, max_contours=1024)
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=1, thresh=0, alpha=0.0))
    res = orc.run(seq[:, 0], cap=1 << 14, mask_frames=range(0, T * NB, 7))
    assert res.counts[1:].min() > 700
    submitted = 0
    for b in range(NB):
        while submitted < NB and submitted < b + depth:
            eng.submit(seq[submitted * T:(submitted + 1) * T])
            submitted += 1
        eng.wait()
        st = eng.ccl_stats()
        assert eng.fallbacks() == 0, f"batch {b}: the shared pool ran out"
        assert st["shared_nodes"] > 0 and st["heavy_tiles"] >= T, (b, st)
        for t in range(T):
            _check_frame(eng, res, t, 0, b * T + t, f"batch {b} frame {t}")
    eng.close()


def test_frame_contour_pass_varying_batch_sizes():
    """k_frame_contours keeps its slot-wide words (shared pool, heavy tally, frames done) at indices set by the
    batch's frame count and re-arms them for the next batch of the same size; a stream's last, partial batch --
    or any change of size -- lands on a slot whose words sit elsewhere.  Batches of 16, 5, 16, 3, 9, ... frames
    of the dot lattice (the shared pool in use) over the 10 slots, 3 in flight: every frame against the oracle,
    no frame falling back."""
    H, W = 150, 200
    sizes = [16, 5, 16, 3, 9, 16, 1, 12, 16, 4, 16, 7, 2, 16, 11, 16, 6, 13, 16, 5]
    seq = _lattice_frames(H, W, 6, sum(sizes) - 1, offset=3)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.0,
                       max_batch=16, max_contours=1024)
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=1, thresh=0, alpha=0.0))
    res = orc.run(seq[:, 0], cap=1 << 14, mask_frames=range(0, sum(sizes), 11))
    starts = np.concatenate([[0], np.cumsum(sizes)])
    depth, submitted = 3, 0
    for b, n in enumerate(sizes):
        while submitted < len(sizes) and submitted < b + depth:
            eng.submit(seq[starts[submitted]:starts[submitted + 1]])
            submitted += 1
        eng.wait()
        assert eng.fallbacks() == 0, f"batch {b} ({n} frames)"
        for t in range(n):
            _check_frame(eng, res, t, 0, int(starts[b]) + t, f"batch {b} ({n} frames) frame {t}")
    eng.close()


def test_frame_contour_pass_pool_exhaustion_falls_back():
    """The same lattice, 64 frames in one batch: the frames' overflow nodes exceed the slot's shared pool
    (12 tiles x 1,600), so some frames are flagged and relabelled by the host's pixel-level CCL -- every
    frame still equals the oracle, and the next batch (pool re-armed) needs no fallback."""
    H, W, T = 150, 200, 64
    seq = _lattice_frames(H, W, 6, 2 * T - 1, offset=2)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=1, threshold=0, avg=0.0,
                       max_batch=T, max_contours=1024)
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=1, thresh=0, alpha=0.0))
    res = orc.run(seq[:, 0], cap=1 << 14, mask_frames=range(0, 2 * T, 9))
    eng.submit(seq[:T])
    eng.wait()
    assert eng.fallbacks() > 0
    for t in range(T):
        _check_frame(eng, res, t, 0, t, f"frame {t}")
    eng.submit(seq[T:T + 8])
    eng.wait()
    assert eng.fallbacks() == 0
    for t in range(8):
        _check_frame(eng, res, t, 0, T + t, f"second batch frame {t}")
    eng.close()


def test_k97_per_frame_path():
    """-B 1920 -b 20 (the CLI's default blur scale at full width): k = 97 > 49 takes the per-frame k_pixel
    kernel and the pixel-level CCL (fm_kernels.hip)."""
    k = make_gaussian(1920, 20)
    assert k == 97
    _run_streams(1920, 120, 1920, k, S=2, T=3, NB=2, mask_every=1)


def test_per_frame_path_more_contours_than_cap_over_batches():
    """k > 49 (the per-frame k_pixel + pixel-level CCL path): frames with more contours than max_contours,
    batches of several frames, several batches.  A frame past the cap is relabelled whole at fm_wait; that
    must not shrink the batch-wide record buffer the next submit writes (advisor, round 2)."""
    H, W, k, T, NB, cap = 540, 960, 51, 3, 3, 50
    fr = np.zeros((T * NB, 1, H, W, 3), np.uint8)
    for i in range(T * NB):
        o = 8 * (i % 2)
        for y in range(12 + o, H - 8, 64):
            for x in range(12 + o, W - 8, 64):
                fr[i, 0, y:y + 6, x:x + 6] = 255
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=k, threshold=0, avg=0.5, max_batch=T,
                       max_contours=cap)
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=k, thresh=0, alpha=0.5))
    res = orc.run(fr[:, 0], cap=1 << 14, mask_frames=range(0, T * NB, 2))
    assert res.counts[1:].min() > cap
    for b in range(NB):
        eng.submit(fr[b * T:(b + 1) * T])
        eng.wait()
        for t in range(T):
            _check_frame(eng, res, t, 0, b * T + t, f"batch {b} frame {t}")
    np.testing.assert_array_equal(eng.background(0), orc.bg)
    eng.close()


@pytest.mark.parametrize("S", [2, 8])
def test_submit_streams_1080p_large_pitch(S):
    """fm_submit_streams at 1080p: each stream's copy is one 2-D copy whose row is a whole 6.2 MB frame and
    whose pitch is S frames (50 MB at S = 8) -- the batch's input slot must hold exactly the frames, from
    host and from device buffers, and the results equal fm_submit's."""
    torch = pytest.importorskip("torch")
    W, H, T = 1920, 1080, 3
    kw = dict(n_streams=S, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    a, b, c = (MotionEngine(**kw) for _ in range(3))
    f = batch(W, H, S, 5, T)
    per = [np.ascontiguousarray(f[:, s]) for s in range(S)]
    dev = [torch.from_numpy(p).to("cuda:0") for p in per]
    torch.cuda.synchronize()
    a.submit(f)
    b.submit_streams(per)
    c.submit_streams([t.data_ptr() for t in dev], on_device=True, n_frames=T)
    for x in (a, b, c):
        x.wait()
    for t in range(T):
        for s in range(S):
            for x in (b, c):
                assert np.array_equal(x.read_frame(t, s), f[t, s]), (t, s)
    for x in (b, c):
        assert np.array_equal(a.counts(), x.counts())
        for s in range(S):
            assert np.array_equal(a.background(s), x.background(s))
    for x in (a, b, c):
        x.close()


def test_submit_streams_equals_submit():
    """fm_submit_streams (one frame buffer per stream) == fm_submit of the same frames gathered
    into [t][s] order: host buffers, device buffers, and one stream's device buffer read in place."""
    torch = pytest.importorskip("torch")
    W, H, S, T = 320, 240, 3, 4
    kw = dict(src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T)
    a, b, c = (MotionEngine(n_streams=S, **kw) for _ in range(3))
    d, e = MotionEngine(n_streams=1, **kw), MotionEngine(n_streams=1, **kw)
    for bi in range(3):
        f = batch(W, H, S, bi * T, T)
        per = [np.ascontiguousarray(f[:, s]) for s in range(S)]
        dev = [torch.from_numpy(p).to("cuda:0") for p in per]
        torch.cuda.synchronize()
        a.submit(f)
        b.submit_streams(per)
        c.submit_streams([t.data_ptr() for t in dev], on_device=True, n_frames=T)
        d.submit(f[:, :1])
        e.submit_streams([dev[0].data_ptr()], on_device=True, n_frames=T)
        for x in (a, b, c, d, e):
            x.wait()
        for x in (b, c):
            assert np.array_equal(a.counts(), x.counts())
        assert np.array_equal(d.counts(), e.counts()) and np.array_equal(d.counts()[:, 0], a.counts()[:, 0])
        for t in range(T):
            for s in range(S):
                want = [q.bbox for q in a.contours(t, s)]
                assert [q.bbox for q in b.contours(t, s)] == want and [q.bbox for q in c.contours(t, s)] == want
                assert np.array_equal(a.mask(t, s), b.mask(t, s)) and np.array_equal(a.mask(t, s), c.mask(t, s))
            assert [q.bbox for q in e.contours(t, 0)] == [q.bbox for q in a.contours(t, 0)]
    for s in range(S):
        assert np.array_equal(a.background(s), b.background(s)) and np.array_equal(a.background(s), c.background(s))
    assert np.array_equal(e.background(0), a.background(0))
    for x in (a, b, c, d, e):
        x.close()


@pytest.mark.parametrize("k", [11, 33, 49])
def test_k_fused_generic_taps(k):
    """k outside k_pix's {3, 5, 7, 21} and <= 49: the generic temporally blocked k_fused kernel."""
    _run_streams(256, 200, 256, k, S=2, T=4, NB=2, mask_every=1)


# --- contourArea for the live area filter (fm.py:679-684) ------------------------

def _area_case(frames, **kw):
    H, W = frames.shape[2:4]
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, max_batch=frames.shape[0], contour_area=True, **kw)
    eng.submit(frames)
    eng.wait()
    orc = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=W, ksize=kw["ksize"], thresh=kw["threshold"],
                                                  alpha=kw["avg"]))
    res = orc.run(frames[:, 0], cap=1 << 17)
    for t in range(frames.shape[0]):
        got = eng.contours(t, 0)
        assert [c.bbox for c in got] == res.boxes(t), t
        np.testing.assert_array_equal(np.array([c.area for c in got]), res.areas(t), err_msg=f"areas frame {t}")
    eng.close()
    return res


def test_contour_area_fixtures_and_random_masks():
    from golden_cases import contour_cases

    for name, case in sorted(contour_cases().items()):
        m = case["mask"]
        fr = np.zeros((2, 1) + m.shape + (3,), np.uint8)
        fr[1, 0] = m[..., None]
        _area_case(fr, ksize=1, threshold=0, avg=0.5)
    rng = np.random.default_rng(11)
    fr = np.zeros((4, 1, 150, 230, 3), np.uint8)
    for t in range(1, 4):
        fr[t, 0] = ((rng.random((150, 230)) < 0.003 * t) * 255).astype(np.uint8)[..., None]
    res = _area_case(fr, ksize=1, threshold=0, avg=0.0)
    assert res.counts[1:].min() > 10


def test_contour_area_synthetic_video_and_lattice():
    _area_case(batch(640, 360, 1, 90, 12), ksize=5, threshold=12, avg=0.1)   # includes a flash frame (97)
    _area_case(_lattice_frames(270, 480, 6, 2), ksize=1, threshold=0, avg=0.0)


def test_video_motion_live_area_filter_on_gpu(tmp_path):
    """-m 1: max_area 5400 < min_area 10000 (192x108, box 100): contours with contourArea in
    (5400, 10000) are skipped (fm.py:684), on the engine's GPU-traced areas."""
    from find_motion_amd import motion, videoio
    from oracle.decision import written_indices

    W, H, n = 192, 108, 110
    vm = motion.VideoMotion(filename=str(tmp_path / "v"), capture=videoio.SyntheticCapture(W, H, n, 0), box_size=100,
                            min_box_scale=1, threshold=12, cache_time=0.3, min_time=0.1, batch=8, outdir=str(tmp_path))
    assert vm.area_filter
    vm.find_motion()
    st = oracle.OracleStream(oracle.OracleConfig(H=H, W=W, box=100, ksize=5))
    vid = videoio.SyntheticCapture(W, H, n, 0).video
    counts, skipped = [], 0
    for i in range(n):
        a = st.step(vid.frame(i))["areas"]
        keep = [x for x in a if not (5400 < x < 10000)]
        skipped += len(a) - len(keep)
        counts.append(len(keep))
    assert skipped > 0
    assert vm.written_indices == written_indices(counts, min_time=0.1, cache_time=0.3)


@pytest.mark.parametrize("W,H,box,bs,want", [
    (1920, 1080, 1920, 384, {"pix"}),                   # configs[1] mode F, k 5: the pixel kernel (not k_fused)
    (3840, 2160, 3840, 183, {"pix"}),                   # configs[4] geometry, k 21
    (1920, 1080, 100, 20, {"small_scan"}),              # mode D, k 5: the small-image path (fm_small.hip)
    (1920, 1080, 100, 9, {"small_scan"}),               # mode D at k 11: the small-image path takes any k
    (640, 480, 640, 58, {"fused"}),                     # k 11 on a large image: k_fused
])
def test_product_kernel_selection(W, H, box, bs, want):
    """Which kernel the product runs for each configuration, read from the engine's own launch timing (the
    round-5 bench ran k_fused at 1080p k = 5 for one build because the pixel-kernel test saw an unset
    work-plane size: every parity test stayed green on the slower generic path)."""
    k = make_gaussian(box, bs)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=4,
                       profile="pix")
    fr = batch(W, H, 1, 0, 4)
    for _ in range(2):  # the second batch has no first-frame launch
        eng.submit(fr)
        eng.wait()
    names = {n for n, (ms, cnt) in eng.kernel_times().items() if cnt > 0}
    eng.close()
    assert names & want, (names, want)
    if "fused" not in want:
        assert "fused" not in names, names
