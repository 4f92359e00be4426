"""Loader for the committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def chain_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "chain_*.npz")))


def load_chain(path):
    d = np.load(path, allow_pickle=False)
    W, H, box, k, T, thresh = (int(v) for v in d["params"])
    case = {k_: d[k_] for k_ in d.files}
    case.update(W=W, H=H, box=box, ksize=k, T=T, thresh=thresh, alpha=float(d["alpha"]),
                has_keep=bool(int(d["has_keep"])), name=os.path.basename(path)[6:-4])
    return case


def boxes_of(case, t):
    b = case["boxes"]
    return [tuple(int(v) for v in r[1:]) for r in b[b[:, 0] == t]] if len(b) else []


def origins_of(case, t):
    o = case["origins"]
    return [tuple(int(v) for v in r[1:]) for r in o[o[:, 0] == t]] if len(o) else []


def contour_cases():
    d = np.load(os.path.join(GOLDEN, "contours_external.npz"), allow_pickle=False)
    names = sorted({k.split("__")[0] for k in d.files})
    return {n: {"mask": d[n + "__mask"], "boxes": [tuple(int(v) for v in r) for r in d[n + "__boxes"]],
                "origins": [tuple(int(v) for v in r) for r in d[n + "__origins"]], "areas": d[n + "__areas"]}
            for n in names}


def load_frontalface():
    """(Cascade, fixture dict) of tests/golden/cascade_frontalface_default.npz (make_golden_cascade.py)."""
    from find_motion_amd.cascade import Cascade

    z = dict(np.load(os.path.join(GOLDEN, "cascade_frontalface_default.npz"), allow_pickle=False))
    fields = ("stage_ntrees", "stage_threshold", "tree_nodes", "node_left", "node_right", "node_feature",
              "node_threshold", "leaves", "feat_rects", "feat_weights", "feat_tilted")
    cs = Cascade(int(z["win"][0]), int(z["win"][1]), *[z[f] for f in fields])
    dets, k = [], 0
    for n in z["frames_counts"]:
        dets.append([tuple(int(v) for v in r) for r in z["frames_detections"][k:k + n]])
        k += n
    z["frames_detections_list"] = dets
    return cs, z


def load_licence_plate_old():
    """(Cascade, [(seed, candidates, detections)]) of tests/golden/cascade_licence_plate_old.npz
    (make_golden_cascade_old.py)."""
    from find_motion_amd.cascade import Cascade

    z = dict(np.load(os.path.join(GOLDEN, "cascade_licence_plate_old.npz"), allow_pickle=False))
    fields = ("stage_ntrees", "stage_threshold", "tree_nodes", "node_left", "node_right", "node_feature",
              "node_threshold", "leaves", "feat_rects", "feat_weights", "feat_tilted")
    cs = Cascade(int(z["win"][0]), int(z["win"][1]), *[z[f] for f in fields])
    cases, kc, kd = [], 0, 0
    for s, nc, nd in zip(z["seeds"], z["cand_counts"], z["det_counts"]):
        cases.append((int(s), [tuple(int(v) for v in r) for r in z["candidates"][kc:kc + nc]],
                      [tuple(int(v) for v in r) for r in z["detections"][kd:kd + nd]]))
        kc += nc
        kd += nd
    return cs, cases
