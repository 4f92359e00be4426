"""find_motion_amd — MI355X-native hot path of find_motion's per-frame motion chain.

The package mirrors the reference's surface (find_motion/find_motion.py):
VideoMotion / VideoFrame with the same constructor and methods, the same CLI
flags, and run_vid / run for embedding.  The per-frame cv2 chain
(blur_frame, mask_off_areas, find_diff) runs as HIP kernels for gfx950
through the C ABI in include/find_motion_amd.h; there is no CPU fallback.
"""
__version__ = "0.1.0"

import os as _os

# Hardware queues per process: HIP's default of 4 puts the decoder's two streams, the contour
# streams and the input / aux streams on shared queues (a shared queue runs its packets in order);
# with 8 every stream the engine and the MJPEG decoder use has a queue of its own (MJPEG-fed
# pipeline 72-73 k -> 79-81 k frames/s, the device-resident figure unchanged).
# Only effective when this is imported before the process's first HIP call.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

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
