#!/usr/bin/env python3
"""Decoder-only driver for profiling: decode one batch of 1080p synthetic MJPEG frames `reps` times.
Usage: tools/jpeg_only.py [restart(0/1)] [reps] [n_frames] [quality]"""
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from PIL import Image  # noqa: E402

from find_motion_amd import MJpegDecoder  # noqa: E402
from find_motion_amd.synthetic import SyntheticVideo  # noqa: E402

rst = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
N = int(sys.argv[3]) if len(sys.argv) > 3 else 192
Q = int(sys.argv[4]) if len(sys.argv) > 4 else 75
W, H = 1920, 1080
v = SyntheticVideo(W, H, 0)
enc = []
for t in range(min(N, 64)):
    b = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(v.frame(t)[..., ::-1])).save(b, "JPEG", quality=Q,
                                                                         **({"restart_marker_rows": 1} if rst else {}))
    enc.append(b.getvalue())
jp = [enc[i % len(enc)] for i in range(N)]
dec = MJpegDecoder(W, H, max_frames=N)
dst = torch.empty((N, H, W, 3), dtype=torch.uint8, device="cuda")
ms = []
for _ in range(reps):
    dec.decode_device(jp, dst.data_ptr())
    ms.append(dec.last_ms())
print({"restart": rst, "ms": [round(m, 3) for m in ms]})
