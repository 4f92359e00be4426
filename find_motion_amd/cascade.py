"""Haar cascade files -> flat arrays (the object-ROI stage).

The reference loads `haarcascades/haarcascade_<name>.xml` with
`cv2.CascadeClassifier` (find_motion.py:383-399) and runs
`detectMultiScale(frame.resized, scaleFactor=1.1, minNeighbors=5)` on every
15th frame resized to width 300 (find_motion.py:703-731).  This module reads
the files OpenCV >= 2.4 writes (`<cascade>` with `<stageNum>`, HAAR features,
stump or tree weak classifiers) into the arrays `fm_haar_create` takes, with
the value conversions of OpenCV's CascadeClassifierImpl::Data::read /
HaarEvaluator::Feature::read (cascadedetect.cpp, 4.x):

* stage thresholds: `(float)value - 1e-5f` (THRESHOLD_EPS), in float32;
* node thresholds, leaf values and rect weights: float32 of the decimal text;
* node (left, right): > 0 internal node of the same tree, <= 0 leaf -idx;
  every tree has nodeCount + 1 leaves.

The old `opencv-haar-classifier` format (haartraining's `<stages>` of `<trees>`;
one file in the reference, `licence_plate_rus_16stages`, commented out of
CASCADE_LOOKUP) is read the way OpenCV's CascadeClassifier::convert rewrites it
into the format above (cascadedetect_convert.cpp): one feature per tree node in
node order, `left_node`/`right_node` kept as internal-node indices of the tree,
`left_val`/`right_val` numbered as that tree's leaves 0, 1, ... in node order,
`stage_threshold` then shifted by THRESHOLD_EPS as for a new file.  Only the plain
stage chain (stage s has parent s - 1 and next -1) is a cascade of that format;
stage trees are refused.  Detection then runs as for any converted cascade.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from dataclasses import dataclass

import numpy as np

THRESHOLD_EPS = np.float32(1e-5)

# find_motion.py:104-122 (entries commented out there are left out here too)
CASCADE_LOOKUP = {
    "frontalcatface": "Cat 1",
    "frontalcatface_extended": "Cat 2",
    "frontalface_alt": "Face 1",
    "frontalface_alt2": "Face 2",
    "frontalface_alt_tree": "Face 3",
    "frontalface_default": "Face 4",
    "fullbody": "Person",
    "lowerbody": "Legs",
    "profileface": "Face 5",
}


@dataclass
class Cascade:
    win_w: int
    win_h: int
    stage_ntrees: np.ndarray     # int32 [n_stages]
    stage_threshold: np.ndarray  # float32 [n_stages], THRESHOLD_EPS already subtracted
    tree_nodes: np.ndarray       # int32 [n_trees], internal nodes per tree
    node_left: np.ndarray        # int32 [n_nodes]
    node_right: np.ndarray       # int32 [n_nodes]
    node_feature: np.ndarray     # int32 [n_nodes]
    node_threshold: np.ndarray   # float32 [n_nodes]
    leaves: np.ndarray           # float32 [n_trees + n_nodes]
    feat_rects: np.ndarray       # int32 [n_features, 3, 4] (x, y, w, h); unused rects are zero
    feat_weights: np.ndarray     # float32 [n_features, 3]; unused rects weigh 0
    feat_tilted: np.ndarray      # uint8 [n_features]

    @property
    def has_tilted(self) -> bool:
        return bool(self.feat_tilted.any())

    @property
    def n_stages(self) -> int:
        return len(self.stage_ntrees)


def _nums(text: str) -> list[str]:
    return text.split()


def parse(path_or_text: str) -> Cascade:
    """Parse a cascade file (path) or its XML text."""
    if path_or_text.lstrip().startswith("<"):
        root = ET.fromstring(path_or_text)
    else:
        root = ET.parse(path_or_text).getroot()
    c = root.find("cascade") if root.tag != "cascade" else root
    if c is None:
        old = next((e for e in ([root] + list(root)) if e.get("type_id") == "opencv-haar-classifier"), None)
        if old is not None:
            return _parse_old(old)
    if c is None or c.find("stageNum") is None:
        raise ValueError("not a new-format OpenCV cascade (<cascade> with <stageNum>)")
    ftype = (c.findtext("featureType") or "").strip()
    if ftype != "HAAR":
        raise ValueError(f"feature type {ftype!r}: only HAAR cascades are supported")
    if int((c.findtext("featureParams/maxCatCount") or "0").strip()) != 0:
        raise ValueError("categorical (subset) splits are not HAAR")
    win_w, win_h = int(c.findtext("width")), int(c.findtext("height"))

    ntrees, sthr, tnodes = [], [], []
    left, right, feat, nthr, leaves = [], [], [], [], []
    for st in c.find("stages").findall("_"):
        sthr.append(np.float32(np.float32(float(st.findtext("stageThreshold"))) - THRESHOLD_EPS))
        weak = st.find("weakClassifiers").findall("_")
        ntrees.append(len(weak))
        for wc in weak:
            v = _nums(wc.findtext("internalNodes"))
            if len(v) % 4:
                raise ValueError("internalNodes is not a multiple of 4 values")
            nn = len(v) // 4
            tnodes.append(nn)
            for i in range(nn):
                left.append(int(v[4 * i]))
                right.append(int(v[4 * i + 1]))
                feat.append(int(v[4 * i + 2]))
                nthr.append(np.float32(float(v[4 * i + 3])))
            lv = _nums(wc.findtext("leafValues"))
            if len(lv) != nn + 1:
                raise ValueError("a tree needs nodeCount + 1 leaf values")
            leaves.extend(np.float32(float(x)) for x in lv)

    fl = c.find("features").findall("_")
    rects = np.zeros((len(fl), 3, 4), np.int32)
    wts = np.zeros((len(fl), 3), np.float32)
    tilt = np.zeros(len(fl), np.uint8)
    for i, f in enumerate(fl):
        rs = f.find("rects").findall("_")
        if not 1 <= len(rs) <= 3:
            raise ValueError("a HAAR feature has 1..3 rects")
        for j, r in enumerate(rs):
            v = _nums(r.text)
            rects[i, j] = [int(x) for x in v[:4]]
            wts[i, j] = np.float32(float(v[4]))
        tilt[i] = 1 if int((f.findtext("tilted") or "0").strip()) != 0 else 0

    nf = len(fl)
    if feat and (min(feat) < 0 or max(feat) >= nf):
        raise ValueError("node feature index out of range")
    return Cascade(win_w, win_h,
                   np.asarray(ntrees, np.int32), np.asarray(sthr, np.float32), np.asarray(tnodes, np.int32),
                   np.asarray(left, np.int32), np.asarray(right, np.int32), np.asarray(feat, np.int32),
                   np.asarray(nthr, np.float32), np.asarray(leaves, np.float32), rects, wts, tilt)


def _parse_old(c) -> Cascade:
    """haartraining's format: <size>W H</size>, <stages> of {<trees> of trees (lists of nodes with
    <feature>, <threshold>, <left_val>|<left_node>, <right_val>|<right_node>), <stage_threshold>,
    <parent>, <next>}."""
    size = _nums(c.findtext("size") or "")
    if len(size) != 2:
        raise ValueError("old-format cascade without <size>W H</size>")
    win_w, win_h = int(size[0]), int(size[1])
    ntrees, sthr, tnodes = [], [], []
    left, right, feat, nthr, leaves = [], [], [], [], []
    frects, fw, ftilt = [], [], []
    stages = c.find("stages")
    if stages is None:
        raise ValueError("old-format cascade without <stages>")
    for s, st in enumerate(stages.findall("_")):
        if int(st.findtext("parent", str(s - 1))) != s - 1 or int(st.findtext("next", "-1")) != -1:
            raise ValueError("stage trees (parent/next other than a chain) are not supported")
        sthr.append(np.float32(np.float32(float(st.findtext("stage_threshold"))) - THRESHOLD_EPS))
        trees = st.find("trees").findall("_")
        ntrees.append(len(trees))
        for tr in trees:
            nodes = tr.findall("_")
            nn = len(nodes)
            if nn == 0:
                raise ValueError("empty tree")
            tnodes.append(nn)
            nleaf = 0
            for nd in nodes:
                rs = nd.find("feature/rects").findall("_")
                if not 1 <= len(rs) <= 3:
                    raise ValueError("a HAAR feature has 1..3 rects")
                r4 = np.zeros((3, 4), np.int32)
                w3 = np.zeros(3, np.float32)
                for j, r in enumerate(rs):
                    v = _nums(r.text)
                    r4[j] = [int(x) for x in v[:4]]
                    w3[j] = np.float32(float(v[4]))
                feat.append(len(frects))
                frects.append(r4)
                fw.append(w3)
                ftilt.append(1 if int((nd.findtext("feature/tilted") or "0").strip()) != 0 else 0)
                nthr.append(np.float32(float(nd.findtext("threshold"))))
                for side, out in (("left", left), ("right", right)):
                    child = nd.findtext(f"{side}_node")
                    if child is not None:
                        k = int(child)
                        if not 0 < k < nn:
                            raise ValueError(f"{side}_node {k} outside its tree")
                        out.append(k)
                    else:
                        out.append(-nleaf)
                        leaves.append(np.float32(float(nd.findtext(f"{side}_val"))))
                        nleaf += 1
            if nleaf != nn + 1:
                raise ValueError("a tree needs nodeCount + 1 leaf values")
    if not ntrees:
        raise ValueError("cascade without stages")
    return Cascade(win_w, win_h,
                   np.asarray(ntrees, np.int32), np.asarray(sthr, np.float32), np.asarray(tnodes, np.int32),
                   np.asarray(left, np.int32), np.asarray(right, np.int32), np.asarray(feat, np.int32),
                   np.asarray(nthr, np.float32), np.asarray(leaves, np.float32),
                   np.asarray(frects, np.int32).reshape(-1, 3, 4), np.asarray(fw, np.float32).reshape(-1, 3),
                   np.asarray(ftilt, np.uint8))


def to_xml(cs: Cascade) -> str:
    """Write a cascade in the same format (stage thresholds written back without the
    epsilon).  Used to make synthetic test cascades; float32 values print with 9
    significant digits, so parse(to_xml(c)) == c."""
    def f9(x):
        return format(float(x), ".9e")

    out = ["<?xml version=\"1.0\"?>", "<opencv_storage>", "<cascade type_id=\"opencv-cascade-classifier\">",
           "  <stageType>BOOST</stageType>", "  <featureType>HAAR</featureType>",
           f"  <height>{cs.win_h}</height>", f"  <width>{cs.win_w}</width>",
           "  <featureParams><maxCatCount>0</maxCatCount></featureParams>",
           f"  <stageNum>{cs.n_stages}</stageNum>", "  <stages>"]
    ti = ni = li = 0
    for s in range(cs.n_stages):
        # the stored value v satisfies float32(float32(v) - eps) == stage_threshold; search for it
        out.append(f"    <_><maxWeakCount>{cs.stage_ntrees[s]}</maxWeakCount>"
                   f"<stageThreshold>{f9(_unshift(cs.stage_threshold[s]))}</stageThreshold><weakClassifiers>")
        for _ in range(cs.stage_ntrees[s]):
            nn = int(cs.tree_nodes[ti])
            nodes = " ".join(f"{cs.node_left[ni + k]} {cs.node_right[ni + k]} {cs.node_feature[ni + k]} "
                             f"{f9(cs.node_threshold[ni + k])}" for k in range(nn))
            lv = " ".join(f9(cs.leaves[li + k]) for k in range(nn + 1))
            out.append(f"      <_><internalNodes>{nodes}</internalNodes><leafValues>{lv}</leafValues></_>")
            ti += 1
            ni += nn
            li += nn + 1
        out.append("    </weakClassifiers></_>")
    out.append("  </stages>")
    out.append("  <features>")
    for i in range(len(cs.feat_tilted)):
        rs = "".join(f"<_>{' '.join(str(int(v)) for v in cs.feat_rects[i, j])} {f9(cs.feat_weights[i, j])}</_>"
                     for j in range(3) if cs.feat_weights[i, j] != 0 or j == 0)
        out.append(f"    <_><rects>{rs}</rects><tilted>{int(cs.feat_tilted[i])}</tilted></_>")
    out += ["  </features>", "</cascade>", "</opencv_storage>"]
    return "\n".join(out)


def _unshift(t: np.float32) -> float:
    # a decimal v with float32(float32(v) - 1e-5f) == t: start from t + eps and step by ulps
    v = np.float32(t + THRESHOLD_EPS)
    for _ in range(64):
        r = np.float32(v - THRESHOLD_EPS)
        if r == t:
            return float(v)
        v = np.nextafter(v, np.float32(np.inf) if r < t else np.float32(-np.inf), dtype=np.float32)
    raise ValueError("stage threshold not representable")
