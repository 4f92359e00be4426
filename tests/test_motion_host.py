"""Host side of the drop-in (find_motion_amd.motion / cli / videoio) on CPU.

The per-frame results come from tests/fake_engine.OracleEngine (the CPU
oracle behind MotionEngine's interface), so these tests exercise the
reference's unchanged state machine -- find_movement (fm.py:665-700),
decide_output (fm.py:549-589), the writer (fm.py:447-546) -- and check it
against the independent restatement in oracle/decision.py: the list of
written frame indices must be identical.
"""
import functools
import json
import logging
import os
import time
from argparse import ArgumentParser

import numpy as np
import pytest

import oracle
from fake_engine import OracleEngine
from find_motion_amd import cli, motion, videoio
from oracle.decision import written_indices


def oracle_counts(W, H, n, box, k, thresh=12, alpha=0.1, stream=0, keep=None):
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k, thresh=thresh, alpha=alpha)
    st = oracle.OracleStream(cfg, keep)
    cap = videoio.SyntheticCapture(W, H, n, stream)
    out = []
    while True:
        ok, fr = cap.read()
        if not ok:
            return out
        out.append(st.step(fr)["count"])


def make_vm(tmp_path, W=192, H=108, n=40, box=100, batch=1, stream=0, **kw):
    cap = videoio.SyntheticCapture(W, H, n, stream)
    k = motion.make_gaussian_size(box, kw.get("blur_scale", 20))
    eng = OracleEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=k, threshold=kw.get("threshold", 12),
                       avg=kw.get("avg", 0.1), max_batch=batch, keep_planes=kw.pop("keep_planes", False))
    kw.setdefault("threshold", 12)
    vm = motion.VideoMotion(filename=str(tmp_path / f"vid{stream}"), capture=cap, engine=eng, batch=batch,
                            box_size=box, cache_time=kw.pop("cache_time", 0.3), min_time=kw.pop("min_time", 0.1),
                            fps=kw.pop("fps", 30), outdir=str(tmp_path), **kw)
    return vm, eng


# --- decision restatement ----------------------------------------------------

def test_decision_known_answers():
    # fps 10: cache 3 frames, min 2 contours
    c = [0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0]
    # frame 4: counter 1 < 2 -> cached; frame 5: counter 2 -> flush cache (2,3,4) + 5; decay 3 -> 6,7 written
    # (decay 2, 1 at frames 6, 7; frame 8: decay 0 -> cached)
    assert written_indices(c, fps=10, min_time=0.2, cache_time=0.3) == [2, 3, 4, 5, 6, 7]
    assert written_indices([3] * 5, fps=10, min_time=0.2, cache_time=0.3) == [0, 1, 2, 3, 4]
    assert written_indices([0] * 9, fps=10, min_time=0.2, cache_time=0.3) == []
    # min_time 0: every frame is written (0 >= 0)
    assert written_indices([0, 0, 1], fps=10, min_time=0.0, cache_time=0.3) == [0, 1, 2]
    # zero-length cache
    assert written_indices([0, 2, 0, 0], fps=10, min_time=0.2, cache_time=0.0) == [1]


# --- VideoMotion driven by the oracle engine ----------------------------------

@pytest.mark.parametrize("batch", [1, 4, 7])
def test_written_frames_match_decision_restatement(tmp_path, batch):
    vm, eng = make_vm(tmp_path, batch=batch)
    wrote, err, seen = vm.find_motion()
    counts = oracle_counts(192, 108, 40, 100, 5)
    want = written_indices(counts, fps=30, min_time=0.1, cache_time=0.3)
    assert sum(counts) > 0 and want, "synthetic stream has motion"
    assert vm.written_indices == want
    assert wrote is True and err == "" and seen == ()
    assert eng.submits == -(-40 // batch) and eng.closed is False  # injected engines are not closed


def test_output_avi_holds_the_written_source_frames(tmp_path):
    vm, _ = make_vm(tmp_path, n=30)
    vm.find_motion()
    assert os.path.basename(vm.outfile_name) == "vid0_1_motion.avi"
    cap = videoio.RawAviCapture(vm.outfile_name)
    src = videoio.SyntheticCapture(192, 108, 30, 0).video
    got = []
    while True:
        ok, fr = cap.read()
        if not ok:
            break
        got.append(fr)
    assert len(got) == len(vm.written_indices)
    for fr, i in zip(got, vm.written_indices):
        np.testing.assert_array_equal(fr, src.frame(i))


def test_frame_attributes_bound_from_engine(tmp_path):
    vm, eng = make_vm(tmp_path, n=6, keep_planes=True, pipeline_depth=1)  # ref_frame after every frame
    cfg = eng.cfg
    st = oracle.OracleStream(cfg)
    seen = 0
    while vm.read():
        vm.blur_frame()
        vm.mask_off_areas()
        vm.find_diff()
        f = vm.current_frame
        ref = st.step(f.raw)
        np.testing.assert_array_equal(f.thresh, ref["mask"])
        np.testing.assert_array_equal(f.gray, ref["gray"])
        np.testing.assert_array_equal(f.blur, ref["blur"])
        np.testing.assert_array_equal(f.frame_delta, ref["delta"])
        assert [c.bbox for c in f.contours] == ref["boxes"]
        np.testing.assert_array_equal(vm.ref_frame, st.bg)
        vm.step()
        seen += 1
    assert seen == 6


def test_planes_absent_without_show_and_stale_results_raise(tmp_path):
    vm, _ = make_vm(tmp_path, n=4, batch=2)
    assert vm.ref_frame is None
    assert vm.read()
    f0 = vm.current_frame
    assert f0.gray is None and f0.blur is None and f0.thresh is not None
    f1_bound = motion._Bound(vm.engine, vm.engine.generation, 1, 0)
    vm.read()
    vm.read()  # the next batch replaces the device results of frames 0-1
    with pytest.raises(RuntimeError):
        f1_bound.fetch("thresh")


def test_masks_rasterised_once_and_applied(tmp_path):
    masks = [((0, 0), (96, 54)), ((191, 107), (150, 107), (191, 60))]
    vm, eng = make_vm(tmp_path, n=3, keep_planes=True, mask_areas=masks)
    keep = eng.streams[0].keep
    assert keep is not None and keep[:28, :50].max() == 0 and keep[30:45, 55:70].min() == 1
    vm.read()
    assert (vm.current_frame.blur[keep == 0] == 0).all()


def test_find_diff_without_processing_raises_reference_message(tmp_path):
    vm, _ = make_vm(tmp_path, n=2)
    with pytest.raises(Exception, match="Blur frame is None"):
        vm.find_diff(motion.VideoFrame(np.zeros((108, 192, 3), np.uint8)))


def test_external_frame_through_blur_frame(tmp_path):
    vm, eng = make_vm(tmp_path, n=2)
    fr = motion.VideoFrame(videoio.SyntheticCapture(192, 108, 1).video.frame(0))
    vm.blur_frame(fr)
    vm.find_diff(fr)
    assert fr.processed and fr.contours == [] and eng.initialized(0)


def test_live_area_filter_skips_by_contour_area(tmp_path):
    """-m 1 at 192x108, box 100: max_area 5400 < min_area 10000, so the filter of fm.py:684 is live and
    contours whose contourArea lies in (5400, 10000) do not count (the flash frames' full-frame blobs)."""
    W, H, n, box = 192, 108, 110, 100
    cap = videoio.SyntheticCapture(W, H, n, 0)
    k = motion.make_gaussian_size(box, 20)
    eng = OracleEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=4,
                       contour_area=True)
    vm = motion.VideoMotion(filename=str(tmp_path / "v"), capture=cap, engine=eng, batch=4, box_size=box,
                            min_box_scale=1, cache_time=0.3, min_time=0.1, outdir=str(tmp_path))
    assert vm.area_filter and (vm.max_area, vm.min_area) == (5400, 10000)
    vm.find_motion()
    cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k)
    st = oracle.OracleStream(cfg)
    vid = videoio.SyntheticCapture(W, H, n, 0).video
    counts, skipped = [], 0
    for i in range(n):
        r = st.step(vid.frame(i))
        keep = [a for a in r["areas"] if not (5400 < a < 10000)]
        skipped += len(r["areas"]) - len(keep)
        counts.append(len(keep))
    assert skipped > 0  # the flash frames (every 97th) make full-frame contours of area ~5300-5600
    assert vm.written_indices == written_indices(counts, min_time=0.1, cache_time=0.3)


def test_run_vid_error_tuple():
    wrote, name, err, seen = motion.run_vid("/nonexistent/video.avi", engine=None)
    assert wrote is None and name == "/nonexistent/video.avi" and err and seen is None


def test_stream_group_matches_per_video_runs(tmp_path):
    S, n = 3, 24
    caps = [videoio.SyntheticCapture(192, 108, n - 5 * s, s) for s in range(S)]  # ragged lengths
    names = [str(tmp_path / f"g{s}") for s in range(S)]
    grp = motion.StreamGroup(names, batch=5, captures=caps, engine=OracleEngine, box_size=100, threshold=12,
                             cache_time=0.3, min_time=0.1, outdir=str(tmp_path))
    res = grp.find_motion()
    assert [r[1] for r in res] == names
    for s, v in enumerate(grp.videos):
        counts = oracle_counts(192, 108, n - 5 * s, 100, 5, stream=s)
        assert v.written_indices == written_indices(counts, min_time=0.1, cache_time=0.3), s


# --- videoio -------------------------------------------------------------------

@pytest.mark.parametrize("W,H", [(64, 48), (37, 5), (640, 480)])
def test_raw_avi_round_trip(tmp_path, W, H):
    rng = np.random.default_rng(W)
    frames = rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8)
    p = str(tmp_path / "x.avi")
    w = videoio.RawAviWriter(p, 25, (W, H))
    for f in frames:
        w.write(f)
    w.release()
    cap = videoio.open_capture(p) if videoio.cv2 is None else videoio.RawAviCapture(p)
    assert cap.get(videoio.CAP_PROP_FRAME_COUNT) == 3
    assert (cap.get(videoio.CAP_PROP_FRAME_WIDTH), cap.get(videoio.CAP_PROP_FRAME_HEIGHT)) == (W, H)
    for f in frames:
        ok, g = cap.read()
        assert ok
        np.testing.assert_array_equal(g, f)
    assert cap.read()[0] is False


def test_open_capture_sources():
    c = videoio.open_capture("synthetic:64x48:5:2")
    assert c.get(videoio.CAP_PROP_FRAME_COUNT) == 5 and c.read()[1].shape == (48, 64, 3)
    a = videoio.open_capture(np.zeros((2, 4, 6, 3), np.uint8))
    assert a.get(videoio.CAP_PROP_FRAME_WIDTH) == 6
    bad = videoio.RawAviCapture("/nonexistent.avi")
    assert not bad.isOpened()


# --- CLI -----------------------------------------------------------------------

def parse(argv):
    p = ArgumentParser()
    cli.get_args(p)
    return p.parse_args(argv)


def test_cli_flags_and_defaults_match_reference():
    a = parse([])
    assert (a.box_size, a.blur_scale, a.threshold, a.avg, a.mintime, a.cachetime, a.fps, a.codec, a.min_box_scale,
            a.processes) == (100, 20, 12, 0.1, 0.5, 1.0, 30, "MP42", 50, 1)
    a = parse(["x.avi", "-B", "1920", "-b", "384", "-t", "7", "-a", "0.2", "-M", "1", "-C", "2", "-m", "((0,0),(5,5))",
               "-O", "fullbody", "-J", "4", "-s", "-cu", "-d", "-T", "-k", "MJPG", "-f", "25", "--gpus", "8"])
    assert a.files == ["x.avi"] and a.box_size == 1920 and a.blur_scale == 384 and a.masks == [((0, 0), (5, 5))]
    assert a.cascade_object == ["fullbody"] and a.gpus == 8 and a.show and a.cleanup and a.test


def test_ini_overrides_cli(tmp_path):
    ini = tmp_path / "c.ini"
    ini.write_text("[settings]\nbox-size = 1920\navg = 0.5\nshow = True\nmasks = [((0, 0), (3, 3))]\n")
    a = cli.process_config(str(ini), parse(["-B", "100"]))
    assert a.box_size == 1920 and a.avg == 0.5 and a.show is True and a.masks == [((0, 0), (3, 3))]
    ini.write_text("[settings]\nshow = yes\n")
    with pytest.raises(ValueError):
        cli.process_config(str(ini), parse([]))


def test_read_masks_schema(tmp_path):
    f = tmp_path / "m.json"
    f.write_text(json.dumps([[[0, 0], [639, 359]], [[3839, 2159], [3200, 2159], [3839, 1600]]]))
    assert cli.read_masks(str(f)) == [((0, 0), (639, 359)), ((3839, 2159), (3200, 2159), (3839, 1600))]
    for bad in ([[[0, 0]]], [[[0, 0], [1.5, 2]]], [[[0, 0, 1], [1, 2]]], {"a": 1}):
        f.write_text(json.dumps(bad))
        assert cli.read_masks(str(f)) == []


def test_file_ordering_priority_and_progress(tmp_path):
    files = []
    for i, hhmm in enumerate(["10:00", "02:30", "23:10", "02:45"]):
        p = tmp_path / f"v{i}.avi"
        p.write_bytes(b"x")
        t = time.mktime(time.strptime(f"2026-01-0{i + 1} {hhmm}", "%Y-%m-%d %H:%M")) - time.timezone
        os.utime(p, (t, t))
        files.append(str(p))
    order = [os.path.basename(f) for f, _ in cli.sort_files_by_time(files, cli.process_times(["02:00-03:00", "bad"]))]
    assert order == ["v1.avi", "v3.avi", "v0.avi", "v2.avi"]
    log = tmp_path / "progress.log"
    log.write_text(f"{files[0]} // ()\n")
    left = cli.process_progress(cli.sort_files_by_time(files, []), str(log))
    assert files[0] not in [f for f, _ in left] and len(left) == 3
    assert sorted(cli.find_files(str(tmp_path))) == sorted(files)  # progress.log itself is skipped


def test_shard_contiguous_blocks():
    assert cli.shard(list(range(64)), 8) == [list(range(8 * g, 8 * g + 8)) for g in range(8)]
    assert cli.shard([1, 2, 3], 2) == [[1, 2], [3]]
    assert cli.shard([], 4) == [[], [], [], []]


def test_cli_run_end_to_end_on_avi(tmp_path, monkeypatch):
    """Config 1 plumbing: a 640x480 AVI through the CLI, per-video engine injected (no GPU here)."""
    src = tmp_path / "in"
    src.mkdir()
    W, H, n = 640, 480, 24
    w = videoio.RawAviWriter(str(src / "cam.avi"), 30, (W, H))
    vid = videoio.SyntheticCapture(W, H, n, 0).video
    for i in range(n):
        w.write(vid.frame(i))
    w.release()
    monkeypatch.setattr(motion, "MotionEngine", OracleEngine)
    out = tmp_path / "out"
    res = cli.run(parse(["-i", str(src), "-o", str(out), "-M", "0.1", "-C", "0.3", "--batch", "4"]))
    assert len(res) == 1 and res[0][2] == "", res
    counts = oracle_counts(W, H, n, 100, 5)
    want = written_indices(counts, min_time=0.1, cache_time=0.3)
    got = videoio.RawAviCapture(str(out / "cam.avi_1_motion.avi")) if want else None
    if want:
        assert got.get(videoio.CAP_PROP_FRAME_COUNT) == len(want)
    assert "cam.avi // ()" in (out / "progress.log").read_text()
