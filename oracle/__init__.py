"""CPU oracle for the find_motion per-frame motion chain.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package
(find_motion_amd/).

Parity status: "parity unpinned" by the reference.  The reference
(/root/reference/find_motion/find_motion.py) has no tests or fixtures and its
arithmetic lives in opencv-python (unpinned, requirements.txt:4), which is not
installed anywhere in this image.  The oracle is a restatement of OpenCV 4.x
CPU semantics, pinned by analytic known-answer tests and cross-checked by two
independent implementations (C: fm_oracle.c, numpy/scipy: oracle_np.py).
"""
from .oracle import (  # noqa: F401
    OracleConfig,
    OracleStream,
    bgr2gray,
    build,
    dilate5,
    diff_thresh,
    accumulate,
    find_contours_ext,
    gauss_blur,
    gauss_coeffs,
    lib,
    make_gaussian,
    resize_area_bgr,
    run_streams,
    work_height,
)
