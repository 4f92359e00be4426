"""Decode-ahead batch pipeline between the captures and the engine (the host side of
BASELINE.json north_star's "frame batches pinned and hipMemcpyAsync-overlapped with
compute").

The reference decodes and processes one frame at a time in one loop
(find_motion.py:852-904: read -> blur_frame -> find_diff -> find_movement ->
decide_output).  Here a decoder thread reads the next batches of every stream
into page-locked batch buffers (fm_host_alloc) while the engine works:

    decoder thread:  cap.read() x T x S  ->  pinned buffer  ->  `full` queue
    caller thread:   keep up to fm_max_inflight batches submitted (each
                     submit is an asynchronous DMA + kernels on the engine's
                     streams), wait for the oldest, hand its frames and
                     results to the per-stream state machines, recycle its
                     buffer.

So decode (host), H2D copies and the pixel kernel / contour pass of later
batches all overlap the state machines of the batch being consumed.  Frame
order per stream, and therefore every decision, is unchanged: batches are
waited in submission order and consumed frame by frame.

JPEG mode (every capture has read_jpeg(), i.e. MJPEG sources, SURVEY.md
§8(f)-3): the decoder thread only reads the compressed frames; the engine
decodes them on the GPU (fm_submit_jpeg) in front of the hot path, so only
compressed bytes cross PCIe.  Batch.frames then holds JPEG byte strings and
Batch.buf is None.
"""
from __future__ import annotations

import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from collections import deque
from dataclasses import dataclass

import numpy as np


@dataclass
class Batch:
    """One decoded batch: frames[s] = the raw frames of stream s (each a separate array, as cap.read()
    returns them, kept for the state machine and the writer); buf[:T] = the same frames in page-locked
    memory, the engine's input."""
    buf: np.ndarray
    frames: list
    T: int
    jpegs: list = None  # JPEG mode: the T x S compressed frames in [t][s] order, ended streams padded


class BatchFeeder:
    """Iterate over (Batch, engine) after the engine has processed the batch.

    caps: one capture per engine stream (same frame size).  A stream that ends
    early is padded with its last frame (results dropped by the caller, as
    StreamGroup always did); the iteration ends when every stream has ended.
    """

    def __init__(self, engine, caps: list, batch: int, depth: int | None = None, buffers: list | None = None,
                 jpeg: bool | None = None):
        self.engine = engine
        self.caps = list(caps)
        self.T = int(batch)
        self.depth = max(1, min(depth or engine.max_inflight, engine.max_inflight))
        # JPEG mode needs every capture to hand out compressed frames of one layout (size and chroma
        # sampling: one GPU decoder serves the whole batch); None: whenever they do, otherwise the
        # captures decode (cap.read())
        can = (bool(self.caps) and all(hasattr(c, "read_jpeg") and getattr(c, "gpu_decode", True) for c in self.caps)
               and self._one_layout())
        self.jpeg = can if jpeg is None else bool(jpeg)
        if self.jpeg and not can:
            raise ValueError("JPEG mode needs captures with read_jpeg() and one JPEG layout")
        self.decoder = None
        if self.jpeg:
            from ._native import MJpegDecoder
            sw, sh = engine.src_shape[1], engine.src_shape[0]
            self.decoder = MJpegDecoder(sw, sh, max_frames=self.T * len(self.caps), device=engine.device)
            buffers = []
        # depth batches in flight + one being decoded + one being consumed; page-locking is slow
        # (~0.3 s per GB), so callers that run several feeders pass the same buffers to each
        self.buffers = buffers if buffers is not None else self.make_buffers(engine, self.T, self.depth)
        self._free: queue.Queue = queue.Queue()
        for b in self.buffers:
            self._free.put(b)
        self._full: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._error = None
        # copies into page-locked memory run on a few threads (numpy releases the GIL for them): one
        # thread's memcpy (~7 GB/s) would otherwise cap a 1080p stream near 1.1 k frames/s
        self._copiers = ThreadPoolExecutor(max(1, min(8, len(os.sched_getaffinity(0)))), "fm-copy")
        self._thread = threading.Thread(target=self._decode, name="fm-decode", daemon=True)
        self._thread.start()

    def _one_layout(self) -> bool:
        from .videoio import jpeg_layout
        layouts = set()
        for c in self.caps:
            peek = getattr(c, "peek_jpeg", None)
            j = peek() if peek else None
            if j is None:
                continue  # an empty stream (or one that cannot be inspected) constrains nothing
            try:
                layouts.add(jpeg_layout(j))
            except ValueError:
                return False
        return len(layouts) <= 1

    @staticmethod
    def make_buffers(engine, batch: int, depth: int | None = None) -> list:
        d = max(1, min(depth or engine.max_inflight, engine.max_inflight))
        return [engine.host_buffer(int(batch)) for _ in range(d + 2)]

    # -- decoder thread -----------------------------------------------------------
    def _decode(self) -> None:
        S = len(self.caps)
        live = [True] * S
        last = [None] * S
        try:
            while any(live) and not self._stop.is_set():
                got = [[] for _ in range(S)]
                for s, cap in enumerate(self.caps):
                    while live[s] and len(got[s]) < self.T:
                        ok, fr = cap.read_jpeg() if self.jpeg else cap.read()
                        if not ok:
                            live[s] = False
                            break
                        got[s].append(fr)
                T = max(len(g) for g in got)
                if T == 0:
                    break
                if self.jpeg:
                    jp = []
                    # padding for a stream with no frame yet: any frame of this batch (same layout)
                    pad = next(g[0] for g in got if g)
                    for t in range(T):
                        for s in range(S):
                            if t < len(got[s]):
                                last[s] = got[s][t]
                            jp.append(last[s] if last[s] is not None else pad)
                    self._full.put(Batch(None, got, T, jp))
                    continue
                buf = self._free.get()
                if buf is None or self._stop.is_set():
                    break
                jobs = []
                for s in range(S):
                    for t in range(T):
                        if t < len(got[s]):
                            jobs.append((t, s, got[s][t]))
                            last[s] = got[s][t]
                        elif last[s] is not None:
                            jobs.append((t, s, last[s]))  # ended stream: padding

                def put(j, buf=buf):
                    np.copyto(buf[j[0], j[1]], j[2])

                list(self._copiers.map(put, jobs))
                self._full.put(Batch(buf, got, T))
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            self._error = e
        finally:
            self._full.put(None)

    def _submit_jpeg(self, b: Batch) -> None:
        """fm_submit_jpeg, or, when the GPU decoder refuses a frame of the batch (FM_ENOTSUP: a layout
        it does not take, e.g. separate component scans in a stream whose first frame it took), the
        batch decoded on the host and submitted as frames -- its results and VideoFrame.raw (read back
        from the engine's input slot) are the same."""
        from ._native import FM_ENOTSUP, FMError
        from .videoio import host_decode_jpeg
        try:
            self.engine.submit_jpeg(self.decoder, b.jpegs)
        except FMError as e:
            if e.code != FM_ENOTSUP:
                raise
            S = len(self.caps)
            fr = np.stack([host_decode_jpeg(j) for j in b.jpegs])
            self.engine.submit(fr.reshape((b.T, S) + fr.shape[1:]))

    # -- consumer -------------------------------------------------------------------
    def __iter__(self):
        eng = self.engine
        inflight: deque = deque()
        done = False
        try:
            while True:
                while not done and len(inflight) < self.depth:
                    b = self._full.get()
                    if b is None:
                        done = True
                        break
                    if b.jpegs is not None:
                        self._submit_jpeg(b)
                    else:
                        eng.submit(b.buf[:b.T])
                    inflight.append(b)
                if not inflight:
                    break
                b = inflight.popleft()
                eng.wait()
                yield b
                if b.buf is not None:
                    self._free.put(b.buf)
        finally:
            self._stop.set()
            while inflight:  # an abandoned iteration: finish what was submitted
                inflight.popleft()
                eng.wait()
            self._free.put(None)  # a decoder blocked on a free buffer wakes and stops
            self._thread.join(timeout=30)
            self._copiers.shutdown(wait=True)
            if self.decoder is not None:
                self.decoder.close()
                self.decoder = None
        if self._error is not None:
            raise self._error
