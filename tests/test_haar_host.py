"""Object-ROI stage on the CPU: the cascade reader, the
detectMultiScale restatement (oracle/haar.py) against brute force and known
answers, and the C ABI's cascade validation (no device calls).

Parity unpinned: OpenCV is absent and the reference holds no detection
fixtures; the restatement is pinned by the known-answer and brute-force checks
here, the GPU path by tests/test_gpu_haar.py against it.
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from find_motion_amd import _native
from find_motion_amd.cascade import CASCADE_LOOKUP, THRESHOLD_EPS, parse, to_xml
from haar_cases import make_cascade, make_image
from oracle import haar

REF_CASCADES = "/root/reference/find_motion/haarcascades"


@pytest.mark.skipif(not os.path.isdir(REF_CASCADES), reason="reference cascades not present")
def test_reference_cascades_parse():
    # every cascade the reference can load (CASCADE_LOOKUP, find_motion.py:104-122) reads into
    # consistent arrays
    for name in CASCADE_LOOKUP:
        cs = parse(os.path.join(REF_CASCADES, f"haarcascade_{name}.xml"))
        assert cs.n_stages > 0 and cs.stage_ntrees.sum() == len(cs.tree_nodes)
        assert cs.tree_nodes.sum() == len(cs.node_left) == len(cs.node_threshold)
        assert len(cs.leaves) == len(cs.tree_nodes) + len(cs.node_left)
        assert cs.node_feature.max() < len(cs.feat_tilted)
        assert cs.has_tilted == (name in ("frontalcatface_extended", "fullbody", "lowerbody")), name
    d = parse(os.path.join(REF_CASCADES, "haarcascade_frontalface_default.xml"))
    assert (d.win_w, d.win_h, d.n_stages) == (24, 24, 25)
    assert d.stage_threshold[0] == np.float32(np.float32(-5.0425500869750977) - THRESHOLD_EPS)


@pytest.mark.skipif(not os.path.isdir(REF_CASCADES), reason="reference cascades not present")
def test_reference_old_format_cascade():
    # haarcascade_licence_plate_rus_16stages.xml (haartraining's format, commented out of
    # CASCADE_LOOKUP): 64x16 window, 16 stages of stumps, values as CascadeClassifier::convert
    # writes them; its first stage and first tree as the file states them
    cs = parse(os.path.join(REF_CASCADES, "haarcascade_licence_plate_rus_16stages.xml"))
    assert (cs.win_w, cs.win_h, cs.n_stages, len(cs.tree_nodes)) == (64, 16, 16, 91)
    assert (cs.tree_nodes == 1).all() and len(cs.leaves) == 2 * 91 and not cs.has_tilted
    assert (cs.node_left == 0).all() and (cs.node_right == -1).all()
    assert list(cs.feat_rects[0, :2].ravel()) == [32, 2, 8, 6, 32, 4, 8, 2]
    assert list(cs.feat_weights[0]) == [-1, 3, 0]
    assert cs.node_threshold[0] == np.float32(1.6915600746870041e-002)
    assert list(cs.leaves[:2]) == [np.float32(-9.5547717809677124e-001), np.float32(8.9129137992858887e-001)]
    assert cs.stage_ntrees[0] == 4
    assert cs.stage_threshold[-1] == np.float32(np.float32(-9.1314977407455444e-001) - THRESHOLD_EPS)
    rc, msg = _create(cs)
    assert rc in (_native.FM_OK, _native.FM_EHIP), msg


@pytest.mark.skipif(not os.path.isdir(REF_CASCADES), reason="reference cascades not present")
def test_reference_cascades_pass_the_abi_validation():
    # fm_haar_create validates before touching the device: on this CPU-only host a valid
    # description fails only at the first HIP call (FM_EHIP), never with FM_EINVAL
    for name in CASCADE_LOOKUP:
        cs = parse(os.path.join(REF_CASCADES, f"haarcascade_{name}.xml"))
        rc, msg = _create(cs)
        assert rc in (_native.FM_OK, _native.FM_EHIP), (name, msg)


def _create(cs):
    L = _native.load()
    keep = [np.ascontiguousarray(a) for a in (cs.stage_ntrees, cs.stage_threshold, cs.tree_nodes, cs.node_left,
                                              cs.node_right, cs.node_feature, cs.node_threshold, cs.leaves,
                                              cs.feat_rects, cs.feat_weights, cs.feat_tilted)]
    d = _native.FMHaarDesc(cs.win_w, cs.win_h, len(cs.stage_ntrees), len(cs.tree_nodes), len(cs.node_left),
                           len(cs.leaves), len(cs.feat_tilted), *[a.ctypes.data for a in keep])
    h = C.c_void_p()
    rc = L.fm_haar_create(0, C.byref(d), C.byref(h))
    msg = L.fm_haar_last_error(h).decode()
    L.fm_haar_destroy(h)
    return rc, msg


def test_abi_rejects_inconsistent_cascades():
    base = make_cascade(0, tilted=True)
    assert _create(base)[0] in (_native.FM_OK, _native.FM_EHIP)
    bad = []
    c = make_cascade(0)
    c.node_feature = c.node_feature.copy()
    c.node_feature[0] = len(c.feat_tilted)
    bad.append(c)
    c = make_cascade(0)
    c.feat_rects = c.feat_rects.copy()
    c.feat_rects[0, 0, 2] = c.win_w + 1
    bad.append(c)
    c = make_cascade(0)
    c.leaves = c.leaves[:-1]
    bad.append(c)
    c = make_cascade(0, depth=2)
    c.node_left = c.node_left.copy()
    c.node_left[1] = 5  # link out of the tree
    bad.append(c)
    c = make_cascade(0)
    c.feat_tilted = c.feat_tilted.copy()
    c.feat_tilted[0] = 1  # the full-window rect cannot be a tilted rect
    bad.append(c)
    for c in bad:
        rc, msg = _create(c)
        assert rc == _native.FM_EINVAL and msg


@pytest.mark.parametrize("kw", [dict(), dict(depth=2), dict(tilted=True, depth=2)])
def test_xml_round_trip(kw):
    cs = make_cascade(5, **kw)
    cs2 = parse(to_xml(cs))
    for f in cs.__dataclass_fields__:
        assert np.array_equal(getattr(cs, f), getattr(cs2, f)), f


def test_old_format_fixture():
    # the committed arrays are the reference file's (when it is here) and the restatement's
    # candidates on the plate images are the fixture's
    from golden_cases import load_licence_plate_old
    from haar_cases import plate_image

    cs, cases = load_licence_plate_old()
    path = os.path.join(REF_CASCADES, "haarcascade_licence_plate_rus_16stages.xml")
    if os.path.isfile(path):
        ref = parse(path)
        for f in cs.__dataclass_fields__:
            assert np.array_equal(getattr(cs, f), getattr(ref, f)), f
    for seed, cand, dets in cases[:2]:
        got = haar.detect_candidates(cs, plate_image(seed), 1.1)
        assert [tuple(r) for r in got] == cand and haar.group_rectangles(got, 5) == dets


def _old_xml(cs):
    """The same cascade in haartraining's format (nodes in tree order, leaves by value)."""
    f9 = lambda x: format(float(x), ".9e")  # noqa: E731
    out = ["<?xml version=\"1.0\"?>", "<opencv_storage>", "<c type_id=\"opencv-haar-classifier\">",
           f"<size>{cs.win_w} {cs.win_h}</size>", "<stages>"]
    ti = ni = li = 0
    for s in range(cs.n_stages):
        out.append("<_><trees>")
        for _ in range(cs.stage_ntrees[s]):
            nn = int(cs.tree_nodes[ti])
            out.append("<_>")
            for k in range(nn):
                fi = cs.node_feature[ni + k]
                rs = "".join(f"<_>{' '.join(str(int(v)) for v in cs.feat_rects[fi, j])} {f9(cs.feat_weights[fi, j])}</_>"
                             for j in range(3) if cs.feat_weights[fi, j] != 0 or j == 0)
                kids = ""
                for side, v in (("left", cs.node_left[ni + k]), ("right", cs.node_right[ni + k])):
                    kids += f"<{side}_node>{v}</{side}_node>" if v > 0 else f"<{side}_val>{f9(cs.leaves[li - v])}</{side}_val>"
                out.append(f"<_><feature><rects>{rs}</rects><tilted>{int(cs.feat_tilted[fi])}</tilted></feature>"
                           f"<threshold>{f9(cs.node_threshold[ni + k])}</threshold>{kids}</_>")
            out.append("</_>")
            ti += 1
            ni += nn
            li += nn + 1
        from find_motion_amd.cascade import _unshift
        out.append(f"</trees><stage_threshold>{f9(_unshift(cs.stage_threshold[s]))}</stage_threshold>"
                   f"<parent>{s - 1}</parent><next>-1</next></_>")
    out += ["</stages>", "</c>", "</opencv_storage>"]
    return "\n".join(out)


@pytest.mark.parametrize("kw", [dict(), dict(depth=2), dict(tilted=True, depth=2)])
def test_old_format_reads_as_the_same_cascade(kw):
    # one feature per node and leaves renumbered in node order, so compare what the cascade does:
    # the same detections on the same image, and the same stage structure and thresholds
    cs = make_cascade(7, **kw)
    old = parse(_old_xml(cs))
    for f in ("win_w", "win_h", "stage_ntrees", "stage_threshold", "tree_nodes", "node_threshold"):
        assert np.array_equal(getattr(cs, f), getattr(old, f)), f
    assert len(old.feat_tilted) == len(old.node_left) and len(old.leaves) == len(cs.leaves)
    img = make_image(3)
    assert haar.detect_candidates(cs, img) == haar.detect_candidates(old, img)
    assert len(haar.detect_candidates(cs, img)) > 0


def test_old_format_refuses_stage_trees():
    xml = _old_xml(make_cascade(1)).replace("<parent>1</parent>", "<parent>0</parent>")
    with pytest.raises(ValueError):
        parse(xml)


def test_linear_exact_known_answers():
    # identity, exact 2x (= INTER_AREA fast path (a+b+c+d+2)>>2), 1-row 2 -> 4 upscale
    rng = np.random.default_rng(0)
    g = rng.integers(0, 256, (17, 23), dtype=np.uint8)
    assert np.array_equal(haar.resize_linear_exact(g, 23, 17), g)
    g = rng.integers(0, 256, (16, 24), dtype=np.uint8)
    a = g.astype(np.int32)
    ref = (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
    assert np.array_equal(haar.resize_linear_exact(g, 12, 8), ref)
    assert haar.resize_linear_exact(np.array([[0, 255]], np.uint8), 4, 1).tolist() == [[0, 64, 191, 255]]


def test_integrals_brute_force():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (9, 13), dtype=np.uint8)
    S, Q, T = haar.integrals(img, True)
    h, w = img.shape
    v = img.astype(np.int64)
    for Y in range(h + 1):
        for X in range(w + 1):
            assert S[Y, X] == v[:Y, :X].sum()
            assert Q[Y, X] == (v[:Y, :X] ** 2).sum()
            t = sum(int(v[y, x]) for y in range(Y) for x in range(w) if abs(x - X + 1) <= Y - y - 1)
            assert T[Y, X] == t


def _eval_one(cs, S, Q, T, x, y):
    """One window, scalar, straight from HaarEvaluator::setWindow + predictOrdered."""
    W, H = cs.win_w, cs.win_h

    def rs(I, r, tl):
        rx, ry, rw, rh = (int(v) for v in r)
        if not tl:
            v = int(I[y + ry, x + rx]) - int(I[y + ry, x + rx + rw]) - int(I[y + ry + rh, x + rx]) + \
                int(I[y + ry + rh, x + rx + rw])
        else:
            v = int(I[y + ry, x + rx]) - int(I[y + ry + rh, x + rx - rh]) - int(I[y + ry + rw, x + rx + rw]) + \
                int(I[y + ry + rw + rh, x + rx + rw - rh])
        return (v + (1 << 31)) % (1 << 32) - (1 << 31)

    area = float((W - 2) * (H - 2))
    vs = rs(S, (1, 1, W - 2, H - 2), False)
    vq = rs(Q, (1, 1, W - 2, H - 2), False) & 0xFFFFFFFF
    nf = area * vq - float(vs) * vs
    if not nf > 0:
        return -1
    vnf = np.float32(1.0 / np.sqrt(nf))
    if not area * float(vnf) < 0.1:
        return -1
    ti = ni = li = 0
    for si in range(cs.n_stages):
        tot = 0.0
        for _ in range(int(cs.stage_ntrees[si])):
            idx = 0
            while True:
                nd = ni + idx
                f = int(cs.node_feature[nd])
                I = T if cs.feat_tilted[f] else S
                val = np.float32(cs.feat_weights[f, 0] * np.float32(rs(I, cs.feat_rects[f, 0], cs.feat_tilted[f])))
                val = np.float32(val + np.float32(cs.feat_weights[f, 1] *
                                                  np.float32(rs(I, cs.feat_rects[f, 1], cs.feat_tilted[f]))))
                if cs.feat_weights[f, 2] != 0:
                    val = np.float32(val + np.float32(cs.feat_weights[f, 2] *
                                                      np.float32(rs(I, cs.feat_rects[f, 2], cs.feat_tilted[f]))))
                val = np.float32(val * vnf)
                idx = int(cs.node_left[nd] if float(val) < float(cs.node_threshold[nd]) else cs.node_right[nd])
                if idx <= 0:
                    break
            tot += float(cs.leaves[li - idx])
            ni += int(cs.tree_nodes[ti])
            li += int(cs.tree_nodes[ti]) + 1
            ti += 1
        if tot < float(cs.stage_threshold[si]):
            return -si
    return 1


@pytest.mark.parametrize("seed,tight,kw", [(1, 0.41, dict(depth=2)), (1, 0.38, dict(depth=2, tilted=True)),
                                           (3, 0.44, dict())])
def test_eval_windows_matches_scalar(seed, tight, kw):
    cs = make_cascade(seed, tight=tight, **kw)
    img = haar.bgr2gray(make_image(2))[30:140, 130:250]
    S, Q, T = haar.integrals(img, cs.has_tilted)
    gy, gx = np.meshgrid(np.arange(0, img.shape[0] + 1 - cs.win_h, 2), np.arange(0, img.shape[1] + 1 - cs.win_w, 2),
                         indexing="ij")
    res = haar.eval_windows(cs, S, Q, T, gx.ravel(), gy.ravel())
    ref = np.array([_eval_one(cs, S, Q, T, int(x), int(y)) for x, y in zip(gx.ravel(), gy.ravel())])
    assert np.array_equal(res, ref)
    assert (ref == 0).any() and (ref != 0).any()


def test_scale_list_roi_frame():
    # the reference's ROI frame: width 300 from a 16:9 source -> 300 x 168; 24x24 window
    sc = haar.scale_list(300, 168, 24, 24, 1.1)
    assert sc[0] == np.float32(1.0) and len(sc) == 21  # 1.1^20 * 24 = 161 <= 168 < 178
    assert all(round(24 * float(s)) <= 168 for s in sc)
    assert haar.scale_list(300, 168, 24, 24, 1.1, min_size=(40, 40))[0] > np.float32(1.6)
    assert haar.scale_list(20, 20, 24, 24) == []


def _partition_scalar(rects, eps):
    n = len(rects)
    parent, rank = [-1] * n, [0] * n

    def root(i):
        while parent[i] >= 0:
            i = parent[i]
        return i

    for i in range(n):
        r = root(i)
        for j in range(n):
            if i == j or not haar._similar(rects[i], rects[j], eps):
                continue
            r2 = root(j)
            if r2 != r:
                if rank[r] > rank[r2]:
                    parent[r2] = r
                else:
                    parent[r] = r2
                    rank[r2] += rank[r] == rank[r2]
                    r = r2
                for k0 in (j, i):
                    k = k0
                    while parent[k] >= 0:
                        p = parent[k]
                        parent[k] = r
                        k = p
    lab, out = {}, []
    for i in range(n):
        out.append(lab.setdefault(root(i), len(lab)))
    return out, len(lab)


def test_partition_vectorised_matches_scalar():
    rng = np.random.default_rng(4)
    for _ in range(5):
        rects = [(int(x), int(y), int(s), int(s)) for x, y, s in
                 zip(rng.integers(0, 60, 120), rng.integers(0, 60, 120), rng.integers(20, 30, 120))]
        assert haar.partition(rects, 0.2) == _partition_scalar(rects, 0.2)


def test_group_rectangles_known_answers():
    # 6 similar rects -> one class (6 > 5 neighbours) with the rounded mean; a class of 2 is dropped
    cl = [(100, 100, 40, 40), (101, 100, 40, 40), (100, 102, 41, 41), (99, 100, 40, 40), (100, 99, 40, 40),
          (102, 101, 40, 40)]
    far = [(10, 10, 30, 30), (11, 10, 30, 30)]
    got = haar.group_rectangles(cl + far, 5)
    assert got == [(100, 100, 40, 40)]  # means 100.33, 100.33, 40.17, 40.17
    # a weaker class inside a stronger one is dropped; equal-strength nested classes both stay unless n2 > max(3, n1)
    big = [(50, 50, 100, 100)] * 9
    small = [(70, 70, 30, 30)] * 6
    assert haar.group_rectangles(big + small, 5) == [(50, 50, 100, 100)]
    assert sorted(haar.group_rectangles([(50, 50, 100, 100)] * 6 + small, 5)) == [(50, 50, 100, 100), (70, 70, 30, 30)]
    # minNeighbors 0: the candidates unchanged
    assert haar.group_rectangles(cl, 0) == cl


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "haar_*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_matches_golden_fixtures(path):
    z = np.load(path)  # allow_pickle=False (default): plain arrays and the XML text
    cs = parse(str(z["xml"]))
    cand = haar.detect_candidates(cs, z["image"], float(z["scale_factor"]))
    assert np.array_equal(np.asarray(cand, np.int32).reshape(-1, 4), z["candidates"])
    det = haar.group_rectangles(cand, int(z["min_neighbors"]))
    assert np.array_equal(np.asarray(det, np.int32).reshape(-1, 4), z["detections"])


def test_golden_fixtures_present():
    assert len(GOLDEN) == 3


# --- the reference's own cascade (tests/golden/cascade_frontalface_default.npz) --------------

REF_XML = "/root/reference/find_motion/haarcascades/haarcascade_frontalface_default.xml"


@pytest.mark.skipif(not os.path.exists(REF_XML), reason="reference tree not mounted (GPU box)")
def test_frontalface_fixture_is_the_reference_cascade():
    """The fixture's arrays are find_motion_amd.cascade.parse of the reference's XML (config 5's cascade)."""
    from golden_cases import load_frontalface

    cs, _ = load_frontalface()
    ref = parse(REF_XML)
    assert (cs.win_w, cs.win_h) == (ref.win_w, ref.win_h) == (24, 24) and cs.n_stages == 25
    for f in ("stage_ntrees", "stage_threshold", "tree_nodes", "node_left", "node_right", "node_feature",
              "node_threshold", "leaves", "feat_rects", "feat_weights", "feat_tilted"):
        np.testing.assert_array_equal(getattr(cs, f), getattr(ref, f), err_msg=f)


def test_frontalface_fixture_detections_from_oracle():
    """oracle/haar.py on the fixture's ROI image reproduces its stored candidates and detections
    (the two cartoon faces are found by the real cascade)."""
    from golden_cases import load_frontalface

    cs, z = load_frontalface()
    cand = haar.detect_candidates(cs, z["roi_image"], 1.1)
    assert cand == [tuple(int(v) for v in r) for r in z["roi_candidates"]]
    assert haar.group_rectangles(cand, 5) == [tuple(int(v) for v in r) for r in z["roi_detections"]]
    assert len(z["roi_detections"]) == 2
