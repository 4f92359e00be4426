"""find_motion_amd — MI355X-native hot path of find_motion's per-frame motion chain.

The package mirrors the reference's surface (find_motion/find_motion.py):
VideoMotion / VideoFrame with the same constructor and methods, the same CLI
flags, and run_vid / run for embedding.  The per-frame cv2 chain
(blur_frame, mask_off_areas, find_diff) runs as HIP kernels for gfx950
through the C ABI in include/find_motion_amd.h; there is no CPU fallback.
"""
__version__ = "0.1.0"

import os as _os


def use_hw_queues(n: int = 8, force: bool = False) -> int:
    """Opt in to n hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default is 4).  With 4, the MJPEG
    decoder's two streams, the contour-pass streams and the input / aux streams share queues, and a shared
    queue runs its packets in order; with 8 each has its own (MJPEG-fed pipeline 72-73 k -> 79-81 k
    frames/s, the device-resident figure unchanged).  It changes the queue setup of every
    HIP user in the process (torch included) and takes effect only before the process's first HIP call, so
    it is never set on import: the CLI and bench.py call this first thing.  A value already in the
    environment wins unless `force` (the CLI forces only when FM_HW_QUEUES is set, cli.hw_queues_from_env; an
    exported GPU_MAX_HW_QUEUES is otherwise kept -- with HIP's 4 the input stream shares an in-order queue with a
    contour stream: mode D 498 k vs 591 k frames/s).
    Returns the value in effect."""
    if force:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))
    else:
        _os.environ.setdefault("GPU_MAX_HW_QUEUES", str(int(n)))
    return int(_os.environ["GPU_MAX_HW_QUEUES"])


from ._native import (  # noqa: F401
    CascadeClassifier,
    Contour,
    FMError,
    MJpegDecoder,
    MotionEngine,
    NativeLibraryMissing,
    rasterize_masks,
)
from .motion import StreamGroup, VideoError, VideoFrame, VideoMotion, run_vid  # noqa: F401,E402


def make_gaussian(box_size: int, blur_scale: int) -> int:
    """VideoMotion._make_gaussian (fm.py:478-484): odd kernel size from the box size."""
    k = int(box_size / blur_scale)
    return k + 1 if k % 2 == 0 else k


def work_height(src_h: int, src_w: int, box_size: int) -> int:
    """imutils.resize(width=box) height rule (fm.py:492)."""
    return int(src_h * (box_size / float(src_w)))
