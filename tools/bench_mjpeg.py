#!/usr/bin/env python3
"""Decode side (§8(f)-3): GPU MJPEG decode rate at 1080p, decoder alone and end to end through
fm_submit_jpeg (JPEG bytes in -> contours out), beside Pillow's libjpeg-turbo on one host core.
Frames: the synthetic video encoded by Pillow (4:2:0), without and with restart intervals.
Usage: tools/bench_mjpeg.py [n_frames] [quality]   (FM_JPEG_CB / FM_JPEG_OV: fm_mjpeg_tune values)"""
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (torch's HIP runtime first, as bench.py)
from PIL import Image  # noqa: E402

from find_motion_amd import MJpegDecoder, MotionEngine  # noqa: E402
from find_motion_amd.synthetic import SyntheticVideo  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 192
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 75
W, H = 1920, 1080
TUNE = {k: int(os.environ[e]) for k, e in (("chunk_bits", "FM_JPEG_CB"), ("spec_bits", "FM_JPEG_OV")) if e in os.environ}
v = SyntheticVideo(W, H, 0)
raw = [v.frame(t) for t in range(64)]
out = {"frames": N, "quality": Q}
for name, kw in [("no_restart", {}), ("restart_per_mcu_row", {"restart_marker_rows": 1})]:
    enc = []
    for f in raw:
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(f[..., ::-1])).save(b, "JPEG", quality=Q, **kw)
        enc.append(b.getvalue())
    jp = [enc[i % 64] for i in range(N)]
    r = {"bytes_per_frame": int(np.mean([len(j) for j in enc]))}
    t0 = time.perf_counter()
    for j in jp[:32]:
        np.asarray(Image.open(io.BytesIO(j)))
    r["pillow_1core_fps"] = round(32 / (time.perf_counter() - t0), 1)
    dec = MJpegDecoder(W, H, max_frames=N, **TUNE)
    dst = torch.empty((N, H, W, 3), dtype=torch.uint8, device="cuda")
    dec.decode_device(jp, dst.data_ptr())  # warm-up
    ms = []
    t0 = time.perf_counter()
    for _ in range(3):
        dec.decode_device(jp, dst.data_ptr())
        ms.append(dec.last_ms())
    wall = (time.perf_counter() - t0) / 3
    r["decoder_device_ms"] = round(float(np.median(ms)), 3)
    r["decoder_device_fps"] = round(N / (np.median(ms) / 1e3), 1)
    r["decoder_call_fps"] = round(N / wall, 1)
    # end to end: JPEG bytes -> contours, fm_max_inflight batches in flight
    T = min(N, 192)
    eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=W, ksize=5, threshold=12, avg=0.1, max_batch=T,
                       max_contours=1 << 14)
    dec2 = MJpegDecoder(W, H, max_frames=T, **TUNE)
    batches = [jp[(i * T) % N:(i * T) % N + T] for i in range(max(1, N // T))]
    nb = 8
    depth = eng.max_inflight
    eng.submit_jpeg(dec2, batches[0])  # warm-up batch
    eng.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(min(depth, nb)):
        eng.submit_jpeg(dec2, batches[i % len(batches)])
    for i in range(nb):
        eng.wait()
        if i + depth < nb:
            eng.submit_jpeg(dec2, batches[(i + depth) % len(batches)])
    torch.cuda.synchronize()
    r["end_to_end_fps"] = round(nb * T / (time.perf_counter() - t0), 1)
    eng.close()
    out[name] = r
print(json.dumps(out))
