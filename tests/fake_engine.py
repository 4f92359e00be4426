"""A MotionEngine stand-in backed by the CPU oracle, for host-logic tests on machines without a GPU.

TEST ONLY: it lets tests drive find_motion_amd.motion.VideoMotion's unchanged
state machine with exact per-frame results.  The product never uses it (the
product's engine is the HIP library; there is no CPU fallback).
"""
from collections import deque

import numpy as np

import oracle
from find_motion_amd._native import Contour


class OracleEngine:
    max_inflight = 4  # like the HIP engine: batches may be submitted before the oldest is waited

    def __init__(self, *, n_streams, src_w, src_h, box_size, ksize, threshold, avg, max_batch=1,
                 keep_planes=False, contour_area=False, **_):
        self.n_streams = n_streams
        self.cfg = oracle.OracleConfig(H=src_h, W=src_w, box=box_size, ksize=ksize, thresh=threshold, alpha=avg)
        self.work_shape = (self.cfg.h, self.cfg.w)
        self.max_batch = max_batch
        self.keep_planes = keep_planes
        self.streams = [oracle.OracleStream(self.cfg) for _ in range(n_streams)]
        self.generation = 0
        self.results = []
        self._queue = deque()
        self.src_shape = (src_h, src_w, 3)
        self.contour_area = contour_area
        self.submits = 0
        self.closed = False

    def set_mask(self, s, keep):
        self.streams[s].keep = None if keep is None else np.ascontiguousarray(keep, np.uint8)

    def reset(self, s):
        self.streams[s] = oracle.OracleStream(self.cfg, self.streams[s].keep)

    def initialized(self, s):
        return self.streams[s].initialized

    def background(self, s):
        return self.streams[s].bg.copy()

    def set_background(self, s, bg):
        self.streams[s].bg[...] = bg
        self.streams[s]._init.value = 1

    def submit(self, frames):
        frames = np.asarray(frames)
        if frames.ndim == 4:
            frames = frames[None]
        assert frames.shape[0] <= self.max_batch and frames.shape[1] == self.n_streams
        assert len(self._queue) < self.max_inflight
        self._queue.append([[st.step(frames[t, s]) for s, st in enumerate(self.streams)] for t in range(frames.shape[0])])
        self.submits += 1

    def host_buffer(self, n_frames):
        return np.empty((n_frames, self.n_streams) + self.src_shape, np.uint8)

    def wait(self):
        if self._queue:
            self.results = self._queue.popleft()
        self.generation += 1

    def counts(self):
        return np.array([[r["count"] for r in row] for row in self.results], np.int32)

    def contours(self, t, s):
        r = self.results[t][s]
        areas = r["areas"] if self.contour_area else [None] * len(r["boxes"])
        return [Contour(*b, o, None if a is None else float(a)) for b, o, a in zip(r["boxes"], r["origins"], areas)]

    def mask(self, t, s):
        return self.results[t][s]["mask"]

    def plane(self, which, t, s):
        return self.results[t][s][("gray", "blur", "delta")[which]]

    def close(self):
        self.closed = True
