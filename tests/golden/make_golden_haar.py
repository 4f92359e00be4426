#!/usr/bin/env python3
"""Golden fixtures for the object-ROI stage (tests/golden/haar_*.npz) from oracle/haar.py.

No OpenCV here and no detection fixtures in the reference, so these pin the
restatement against regressions (tests/test_haar_host.py, CPU) and the GPU path
(tests/test_gpu_haar.py) on stored inputs.  Each case stores the cascade as
XML text (tests/haar_cases.py generators, find_motion_amd.cascade.to_xml), the
ROI image (BGR u8), the parameters, the ungrouped candidates and the grouped
detections.

Run from the repo root:  python tests/golden/make_golden_haar.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from find_motion_amd.cascade import to_xml  # noqa: E402
from haar_cases import make_cascade, make_image  # noqa: E402
from oracle import haar  # noqa: E402

CASES = {
    "haar_trees_roi300": dict(cascade=dict(seed=1, tight=0.41, depth=2), image=dict(seed=2), sf=1.1, mn=5),
    "haar_tilted_roi300": dict(cascade=dict(seed=1, tight=0.38, depth=2, tilted=True), image=dict(seed=4), sf=1.1, mn=3),
    "haar_stumps_odd_size": dict(cascade=dict(seed=3, tight=0.44), image=dict(seed=6, w=173, h=97), sf=1.2, mn=2),
}


def main():
    for name, c in CASES.items():
        cs = make_cascade(**c["cascade"])
        img = make_image(**c["image"])
        cand = haar.detect_candidates(cs, img, c["sf"])
        det = haar.group_rectangles(cand, c["mn"])
        np.savez_compressed(os.path.join(HERE, name + ".npz"), xml=np.array(to_xml(cs)), image=img,
                            scale_factor=c["sf"], min_neighbors=c["mn"],
                            candidates=np.asarray(cand, np.int32).reshape(-1, 4),
                            detections=np.asarray(det, np.int32).reshape(-1, 4))
        print(name, img.shape, len(cand), "candidates", len(det), "detections")


if __name__ == "__main__":
    main()
