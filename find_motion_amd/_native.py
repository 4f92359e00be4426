"""ctypes binding of include/find_motion_amd.h (libfm_hip.so, built in-tree).

This is the only way the package reaches the hot path: there is no CPU
fallback.  If the HIP library is missing, importing the engine raises
NativeLibraryMissing with the build command.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libfm_hip.so")
# development override: an alternative build of the same library (A/B kernel variants)
LIB_PATH = os.environ.get("FM_HIP_LIB") or LIB_PATH  # unset or empty: the in-tree product library

FM_OK, FM_EINVAL, FM_EHIP, FM_ENOMEM, FM_ESTATE, FM_ENOTSUP = 0, -1, -2, -3, -4, -5
FM_FLAG_KEEP_PLANES, FM_FLAG_PROFILE, FM_FLAG_PROFILE_PIX, FM_FLAG_CONTOUR_AREA = 0x1, 0x2, 0x4, 0x8
PLANE_GRAY, PLANE_BLUR, PLANE_DELTA, PLANE_SMALL = 0, 1, 2, 3

EXPORTED = (
    "fm_abi_version", "fm_create", "fm_destroy", "fm_last_error", "fm_work_size", "fm_set_mask",
    "fm_reset_stream", "fm_submit", "fm_wait", "fm_get_counts", "fm_get_contours", "fm_read_mask",
    "fm_read_plane", "fm_read_background", "fm_write_background", "fm_set_hip_stream",
    "fm_kernel_times", "fm_kernel_time_spread", "fm_kernel_time_busy", "fm_kernel_time_stats", "fm_reset_kernel_times", "fm_rasterize_masks", "fm_max_inflight",
    "fm_host_alloc", "fm_host_free", "fm_last_fallbacks", "fm_last_ccl_stats",
    "fm_haar_create", "fm_haar_destroy", "fm_haar_last_error", "fm_haar_window", "fm_haar_detect",
    "fm_haar_candidates", "fm_haar_last_ms", "fm_haar_detect_frames",
    "fm_mjpeg_create", "fm_mjpeg_destroy", "fm_mjpeg_last_error", "fm_mjpeg_decode", "fm_mjpeg_last_ms",
    "fm_submit_jpeg", "fm_read_frame", "fm_mjpeg_tune", "fm_frame_device", "fm_mjpeg_geometry",
    "fm_submit_streams", "fm_footprint", "fm_haar_detect_frame_list", "fm_haar_detect_frame_list_async",
    "fm_haar_collect",
)


class NativeLibraryMissing(ImportError):
    pass


class FMError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"find_motion_amd error {code}: {msg}")
        self.code = code


class FMParams(C.Structure):
    _fields_ = [("device", C.c_int), ("n_streams", C.c_int), ("src_w", C.c_int), ("src_h", C.c_int),
                ("box_size", C.c_int), ("ksize", C.c_int), ("threshold", C.c_int), ("avg", C.c_double),
                ("max_batch", C.c_int), ("max_contours", C.c_int), ("flags", C.c_uint)]


class FMHaarDesc(C.Structure):
    _fields_ = [("win_w", C.c_int32), ("win_h", C.c_int32), ("n_stages", C.c_int32), ("n_trees", C.c_int32),
                ("n_nodes", C.c_int32), ("n_leaves", C.c_int32), ("n_features", C.c_int32),
                ("stage_ntrees", C.c_void_p), ("stage_threshold", C.c_void_p), ("tree_nodes", C.c_void_p),
                ("node_left", C.c_void_p), ("node_right", C.c_void_p), ("node_feature", C.c_void_p),
                ("node_threshold", C.c_void_p), ("leaves", C.c_void_p), ("feat_rects", C.c_void_p),
                ("feat_weights", C.c_void_p), ("feat_tilted", C.c_void_p)]


class FMContour(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("w", C.c_int32), ("h", C.c_int32),
                ("origin_x", C.c_int32), ("origin_y", C.c_int32), ("area2", C.c_int32),
                ("reserved1", C.c_int32)]


_lib = None


def load() -> C.CDLL:
    """Load libfm_hip.so (raises NativeLibraryMissing if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found: build the HIP extension with "
            f"`make -C {os.path.join(_PKG, 'csrc')}` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, i32, u8p = C.c_void_p, C.c_int, C.c_void_p
    L.fm_abi_version.restype = i32
    L.fm_create.argtypes = [C.POINTER(vp), C.POINTER(FMParams)]
    L.fm_destroy.argtypes = [vp]
    L.fm_destroy.restype = None
    L.fm_last_error.argtypes = [vp]
    L.fm_last_error.restype = C.c_char_p
    L.fm_work_size.argtypes = [vp, C.POINTER(i32), C.POINTER(i32)]
    L.fm_set_mask.argtypes = [vp, i32, u8p]
    L.fm_reset_stream.argtypes = [vp, i32]
    L.fm_submit.argtypes = [vp, vp, i32, i32]
    L.fm_wait.argtypes = [vp]
    L.fm_get_counts.argtypes = [vp, vp]
    L.fm_get_contours.argtypes = [vp, i32, i32, vp, i32]
    L.fm_read_mask.argtypes = [vp, i32, i32, vp]
    L.fm_read_plane.argtypes = [vp, i32, i32, i32, vp]
    L.fm_read_background.argtypes = [vp, i32, vp]
    L.fm_write_background.argtypes = [vp, i32, vp]
    L.fm_set_hip_stream.argtypes = [vp, vp]
    L.fm_kernel_times.argtypes = [vp, vp, vp, vp, i32]
    L.fm_host_alloc.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
    L.fm_host_free.argtypes = [vp, vp]
    L.fm_kernel_time_spread.argtypes = [vp, vp, i32]
    L.fm_kernel_time_busy.argtypes = [vp, vp, i32]
    L.fm_kernel_time_stats.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
    L.fm_reset_kernel_times.argtypes = [vp]
    L.fm_rasterize_masks.argtypes = [i32, i32, C.c_double, vp, vp, i32, vp]
    L.fm_max_inflight.argtypes = [vp]
    L.fm_last_fallbacks.argtypes = [vp]
    L.fm_last_ccl_stats.argtypes = [vp, C.POINTER(i32), C.POINTER(i32)]
    L.fm_footprint.argtypes = [vp, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    L.fm_haar_create.argtypes = [i32, C.POINTER(FMHaarDesc), C.POINTER(vp)]
    L.fm_haar_destroy.argtypes = [vp]
    L.fm_haar_destroy.restype = None
    L.fm_haar_last_error.argtypes = [vp]
    L.fm_haar_last_error.restype = C.c_char_p
    L.fm_haar_window.argtypes = [vp, C.POINTER(i32), C.POINTER(i32)]
    L.fm_haar_detect.argtypes = [vp, vp, i32, i32, i32, i32, i32, C.c_double, i32, i32, i32, i32, i32, vp, i32, vp]
    L.fm_haar_candidates.argtypes = [vp, vp, i32]
    L.fm_haar_detect_frames.argtypes = [vp, vp, i32, i32, i32, i32, i32, C.c_double, i32, vp, i32, vp, vp]
    L.fm_haar_detect_frame_list.argtypes = [vp, vp, i32, i32, i32, i32, C.c_double, i32, vp, i32, vp, vp]
    L.fm_haar_detect_frame_list_async.argtypes = [vp, vp, i32, i32, i32, i32, C.c_double, i32, vp]
    L.fm_haar_collect.argtypes = [vp, vp, i32, vp, i32]
    L.fm_haar_last_ms.argtypes = [vp]
    L.fm_haar_last_ms.restype = C.c_double
    L.fm_mjpeg_create.argtypes = [i32, i32, i32, i32, C.POINTER(vp)]
    L.fm_mjpeg_destroy.argtypes = [vp]
    L.fm_mjpeg_destroy.restype = None
    L.fm_mjpeg_last_error.argtypes = [vp]
    L.fm_mjpeg_last_error.restype = C.c_char_p
    L.fm_mjpeg_decode.argtypes = [vp, vp, vp, i32, vp, i32]
    L.fm_mjpeg_last_ms.argtypes = [vp]
    L.fm_mjpeg_last_ms.restype = C.c_double
    L.fm_submit_jpeg.argtypes = [vp, vp, vp, vp, i32]
    L.fm_read_frame.argtypes = [vp, i32, i32, vp]
    L.fm_frame_device.argtypes = [vp, i32, i32, C.POINTER(C.c_void_p)]
    L.fm_mjpeg_tune.argtypes = [vp, i32, i32]
    L.fm_mjpeg_geometry.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.fm_submit_streams.argtypes = [vp, vp, i32, i32]
    for name in EXPORTED:
        if name not in ("fm_destroy", "fm_last_error", "fm_abi_version", "fm_haar_destroy", "fm_haar_last_error",
                        "fm_haar_last_ms", "fm_mjpeg_destroy", "fm_mjpeg_last_error", "fm_mjpeg_last_ms"):
            getattr(L, name).restype = i32
    _lib = L
    return L


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def rasterize_masks(h: int, w: int, scale: float, polygons) -> np.ndarray:
    """mask_off_areas (fm.py:611-636) rasterised once: keep-mask (1 = keep, 0 = masked)."""
    L = load()
    polys = [list(p) for p in (polygons or [])]
    keep = np.empty((h, w), np.uint8)
    npts = np.array([len(p) for p in polys], np.int32)
    xy = np.array([c for p in polys for pt in p for c in pt], np.int32) if polys else np.zeros(2, np.int32)
    rc = L.fm_rasterize_masks(h, w, float(scale), _ptr(xy), _ptr(npts) if polys else None, len(polys), _ptr(keep))
    if rc != FM_OK:
        raise FMError(rc, "invalid mask polygons (each needs >= 2 points)")
    return keep


@dataclass
class Contour:
    """One external contour of VideoFrame.contours (fm.py:269-276).

    bbox is cv2.boundingRect's (x, y, w, h) (fm.py:792); origin is the border
    start (the component's raster-first pixel); area is cv2.contourArea of the
    CHAIN_APPROX_SIMPLE contour (fm.py:679), None unless the engine traces it."""
    x: int
    y: int
    w: int
    h: int
    origin: tuple
    area: float | None = None

    @property
    def bbox(self):
        return (self.x, self.y, self.w, self.h)


class MotionEngine:
    """One fm_ctx: n_streams background models on one HIP device."""

    def __init__(self, *, n_streams: int, src_w: int, src_h: int, box_size: int, ksize: int,
                 threshold: int, avg: float, max_batch: int = 1, max_contours: int = 4096,
                 keep_planes: bool = False, profile: bool | str = False, device: int = 0,
                 contour_area: bool = False):
        # profile: True = every kernel timed with HIP events, "pix" = pixel-stream kernels only
        self._L = load()
        p = FMParams(device, n_streams, src_w, src_h, box_size, ksize, int(threshold), float(avg),
                     max_batch, max_contours,
                     (FM_FLAG_KEEP_PLANES if keep_planes else 0) | (FM_FLAG_CONTOUR_AREA if contour_area else 0) |
                     (FM_FLAG_PROFILE_PIX if profile == "pix" else FM_FLAG_PROFILE if profile else 0))
        h = C.c_void_p()
        rc = self._L.fm_create(C.byref(h), C.byref(p))
        if rc != FM_OK:
            raise FMError(rc, self._L.fm_last_error(None).decode())
        self._h = h
        self.params = p
        hh, ww = C.c_int(), C.c_int()
        self._check(self._L.fm_work_size(h, C.byref(hh), C.byref(ww)))
        self.work_shape = (hh.value, ww.value)
        self.max_inflight = self._L.fm_max_inflight(h)
        self.n_streams = n_streams
        self.src_shape = (src_h, src_w, 3)
        self.device = int(device)
        self.max_batch = max_batch
        self.max_contours = max_contours
        self.last_batch = 0
        self.keep_planes = bool(keep_planes)
        self.generation = 0    # bumped at every wait(): results of older batches are gone
        self._init = [False] * n_streams
        self._inflight = []    # (n_frames, host frames kept alive) per submitted, not yet waited batch

    # -- plumbing ------------------------------------------------------------
    def _check(self, rc: int) -> int:
        if rc < 0:
            raise FMError(rc, self._L.fm_last_error(self._h).decode())
        return rc

    def close(self) -> None:
        if getattr(self, "_h", None):
            for buf in getattr(self, "_host_bufs", []):
                self._L.fm_host_free(self._h, buf)
            self._host_bufs = []
            self._L.fm_destroy(self._h)
            self._h = None

    def host_buffer(self, n_frames: int) -> np.ndarray:
        """Page-locked uint8 [n_frames][n_streams][H][W][3] array for frame batches: submit()
        of it is an asynchronous DMA on the engine's input stream, overlapped with the
        previous batches' kernels.  Freed by close(); keep it unchanged until wait() returns
        for a batch submitted from it."""
        shape = (n_frames, self.n_streams) + self.src_shape
        nbytes = int(np.prod(shape))
        p = C.c_void_p()
        self._check(self._L.fm_host_alloc(self._h, nbytes, C.byref(p)))
        if not hasattr(self, "_host_bufs"):
            self._host_bufs = []
        self._host_bufs.append(p)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(nbytes,)).reshape(shape)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- state ---------------------------------------------------------------
    def set_mask(self, stream: int, keep: np.ndarray | None) -> None:
        if keep is None:
            self._check(self._L.fm_set_mask(self._h, stream, None))
            return
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        if keep.shape != self.work_shape:
            raise ValueError(f"keep-mask shape {keep.shape} != work shape {self.work_shape}")
        self._check(self._L.fm_set_mask(self._h, stream, _ptr(keep)))

    def reset(self, stream: int) -> None:
        self._check(self._L.fm_reset_stream(self._h, stream))
        self._init[stream] = False

    def initialized(self, stream: int) -> bool:
        """True once the stream's background exists (after its first frame, fm.py:651-652)."""
        return self._init[stream]

    def background(self, stream: int) -> np.ndarray:
        out = np.empty(self.work_shape, np.float64)
        self._check(self._L.fm_read_background(self._h, stream, _ptr(out)))
        return out

    def set_background(self, stream: int, bg: np.ndarray) -> None:
        bg = np.ascontiguousarray(bg, dtype=np.float64)
        if bg.shape != self.work_shape:
            raise ValueError(f"background shape {bg.shape} != work shape {self.work_shape}")
        self._check(self._L.fm_write_background(self._h, stream, _ptr(bg)))
        self._init[stream] = True

    def set_hip_stream(self, stream_handle: int | None) -> None:
        self._check(self._L.fm_set_hip_stream(self._h, stream_handle))

    # -- hot path ------------------------------------------------------------
    def submit(self, frames: np.ndarray) -> None:
        """frames: uint8 [n][n_streams][H][W][3] (or [n_streams][H][W][3] for n = 1), host memory."""
        f = np.ascontiguousarray(frames, dtype=np.uint8)
        if f.ndim == 4:
            f = f[None]
        if f.shape[1:] != (self.n_streams,) + self.src_shape:
            raise ValueError(f"frames shape {f.shape} != [n][{self.n_streams}]{self.src_shape}")
        self._check(self._L.fm_submit(self._h, _ptr(f), f.shape[0], 0))
        self._inflight.append((f.shape[0], f))

    def submit_streams(self, frames, on_device: bool = False, n_frames: int | None = None) -> None:
        """One buffer per stream (fm_submit_streams): frames[s] = stream s's frames [n][H][W][3] -- host
        arrays, or device addresses (ints) with on_device and n_frames.  Same results as submit() of the
        frames gathered into [n][n_streams] order, without the host-side gather."""
        if len(frames) != self.n_streams:
            raise ValueError(f"{len(frames)} stream buffers for {self.n_streams} streams")
        if on_device:
            if n_frames is None:
                raise ValueError("n_frames is required for device buffers")
            ptrs = np.array([int(p) for p in frames], np.uint64)
            self._check(self._L.fm_submit_streams(self._h, _ptr(ptrs), int(n_frames), 1))
            self._inflight.append((int(n_frames), None))
            return
        arrs = []
        for f in frames:
            a = np.asarray(f)
            if a.dtype != np.uint8 or not a.flags.c_contiguous:
                a = np.ascontiguousarray(a, dtype=np.uint8)
            if a.ndim == 3:
                a = a[None]
            if a.shape[1:] != self.src_shape:
                raise ValueError(f"stream buffer shape {a.shape} != [n]{self.src_shape}")
            if arrs and a.shape[0] != arrs[0].shape[0]:
                raise ValueError("every stream buffer must hold the same number of frames")
            arrs.append(a)
        ptrs = np.array([a.ctypes.data for a in arrs], np.uint64)
        self._check(self._L.fm_submit_streams(self._h, _ptr(ptrs), arrs[0].shape[0], 0))
        self._inflight.append((arrs[0].shape[0], arrs))

    def submit_device(self, ptr: int, n_frames: int) -> None:
        """Frames already in device memory (e.g. a torch CUDA tensor's data_ptr()).

        Up to two batches may be in flight (submit batch i+1 before wait() for
        batch i): the contour pass of one overlaps the pixel kernel of the next."""
        self._check(self._L.fm_submit(self._h, C.c_void_p(ptr), n_frames, 1))
        self._inflight.append((n_frames, None))

    def submit_jpeg(self, decoder: "MJpegDecoder", jpegs) -> None:
        """Compressed frames (the decode side, fm.py:497-506): jpegs = n_frames x n_streams JPEG byte
        strings in [t][s] order (a flat sequence), decoded on the GPU into the batch, then processed
        as submit().  The byte strings may be dropped once this returns."""
        n = len(jpegs)
        if n % self.n_streams:
            raise ValueError(f"{n} JPEGs is not a multiple of n_streams={self.n_streams}")
        ptrs, sizes, keep = _jpeg_arrays(jpegs)
        self._check(self._L.fm_submit_jpeg(self._h, decoder._h, _ptr(ptrs), _ptr(sizes), n // self.n_streams))
        del keep
        self._inflight.append((n // self.n_streams, None))

    def wait(self) -> None:
        """Complete the oldest batch in flight; its results become readable."""
        self._check(self._L.fm_wait(self._h))
        if self._inflight:
            self.last_batch = self._inflight.pop(0)[0]
        self.generation += 1
        self._init = [True] * self.n_streams

    def fallbacks(self) -> int:
        """Frames of the last waited batch relabelled by the pixel-level fallback (diagnostics)."""
        return self._check(self._L.fm_last_fallbacks(self._h))

    def ccl_stats(self) -> dict:
        """Contour pass of the last waited batch: nodes taken from the shared pool, heavy tiles."""
        a, b = C.c_int32(), C.c_int32()
        self._check(self._L.fm_last_ccl_stats(self._h, C.byref(a), C.byref(b)))
        return {"shared_nodes": a.value, "heavy_tiles": b.value}

    def footprint(self) -> dict:
        """Bytes the context holds: device memory and page-locked host memory (fm_footprint)."""
        d, p = C.c_size_t(), C.c_size_t()
        self._check(self._L.fm_footprint(self._h, C.byref(d), C.byref(p)))
        return {"device_bytes": d.value, "pinned_bytes": p.value}

    def counts(self) -> np.ndarray:
        out = np.zeros((self.last_batch, self.n_streams), np.int32)
        self._check(self._L.fm_get_counts(self._h, _ptr(out)))
        return out

    def contours(self, frame: int, stream: int) -> list:
        """Every external contour of (frame, stream), in raster order of their start pixels.

        max_contours only sizes the first fetch: a frame with more contours is fetched
        whole, so len() is always the true count find_movement needs (fm.py:674-694)."""
        cap = self.max_contours
        while True:
            buf = (FMContour * cap)()
            n = self._check(self._L.fm_get_contours(self._h, frame, stream, C.cast(buf, C.c_void_p), cap))
            if n <= cap:
                return [Contour(c.x, c.y, c.w, c.h, (c.origin_x, c.origin_y), c.area2 / 2 if c.area2 >= 0 else None)
                        for c in buf[:n]]
            cap = n

    def mask(self, frame: int, stream: int) -> np.ndarray:
        out = np.empty(self.work_shape, np.uint8)
        self._check(self._L.fm_read_mask(self._h, frame, stream, _ptr(out)))
        return out

    def read_frame(self, frame: int, stream: int) -> np.ndarray:
        """The source frame (BGR) of (frame, stream) of the last waited batch, from the device."""
        out = np.empty(self.src_shape, np.uint8)
        self._check(self._L.fm_read_frame(self._h, frame, stream, _ptr(out)))
        return out

    def frame_device_ptr(self, frame: int, stream: int) -> int:
        """Device address of the source frame (BGR [H][W][3]) of (frame, stream) of the last waited
        batch, left in HBM (valid until the next wait)."""
        p = C.c_void_p()
        self._check(self._L.fm_frame_device(self._h, frame, stream, C.byref(p)))
        return int(p.value)

    def plane(self, which: int, frame: int, stream: int) -> np.ndarray:
        """gray / blur / frame_delta (h, w), or PLANE_SMALL: the resized BGR frame (h, w, 3) (fm.py:490)."""
        out = np.empty(self.work_shape + ((3,) if which == PLANE_SMALL else ()), np.uint8)
        self._check(self._L.fm_read_plane(self._h, which, frame, stream, _ptr(out)))
        return out

    def kernel_time_stats(self) -> dict:
        """{kernel: {ms, launches, stamped, ms_sq, busy_ms}} plus {"_unstamped": n}, from ONE fold of the launch
        stamps (fm_kernel_time_stats), so every figure covers the same launches."""
        N = 32
        names = (C.c_char_p * N)()
        ms, sms, sq, busy = (C.c_double * N)(), (C.c_double * N)(), (C.c_double * N)(), (C.c_double * N)()
        nl, ns = (C.c_int64 * N)(), (C.c_int64 * N)()
        un = C.c_int64(0)
        v = [C.cast(x, C.c_void_p) for x in (names, ms, nl, sms, ns, sq, busy)]
        n = self._check(self._L.fm_kernel_time_stats(self._h, *v, C.byref(un), N))
        out = {names[i].decode(): {"ms": ms[i], "launches": nl[i], "stamped_ms": sms[i], "stamped": ns[i],
                                   "ms_sq": sq[i], "busy_ms": busy[i]} for i in range(min(n, N))}
        out["_unstamped"] = int(un.value)
        return out

    def kernel_times(self) -> dict:
        """{kernel: (ms, launches)} since the last reset."""
        return {k: (v["ms"], v["launches"]) for k, v in self.kernel_time_stats().items() if k != "_unstamped"}

    def kernel_time_busy(self) -> dict:
        """{kernel: ms during which at least one of its stamped launches ran}."""
        return {k: v["busy_ms"] for k, v in self.kernel_time_stats().items() if k != "_unstamped"}

    def kernel_time_std(self) -> dict:
        """{kernel: standard deviation of its launch time in ms} over its stamped launches only (the pixel kernel
        and the resize; event-timed launches add to ms but not to ms_sq, so they are left out of both)."""
        out = {}
        for name, v in self.kernel_time_stats().items():
            if name == "_unstamped" or v["stamped"] < 1 or v["ms_sq"] <= 0:
                continue
            cnt = v["stamped"]
            out[name] = max(v["ms_sq"] / cnt - (v["stamped_ms"] / cnt) ** 2, 0.0) ** 0.5
        return out

    def reset_kernel_times(self) -> None:
        self._check(self._L.fm_reset_kernel_times(self._h))


class CascadeClassifier:
    """cv2.CascadeClassifier for HAAR cascades on the GPU (find_motion.py:396, :722-731).

    `CascadeClassifier(path)` reads the XML (find_motion_amd.cascade); `detectMultiScale`
    keeps OpenCV's signature and returns an (N, 4) int32 array of (x, y, w, h), or an
    empty tuple when nothing is found, as cv2 does.  `detect_batch` runs many images of
    one size in one call (the ROI frames of many streams)."""

    def __init__(self, path_or_cascade, device: int = 0):
        from .cascade import Cascade, parse
        cs = path_or_cascade if isinstance(path_or_cascade, Cascade) else parse(path_or_cascade)
        self.cascade = cs
        L = load()
        self._keep = [np.ascontiguousarray(a) for a in (
            cs.stage_ntrees, cs.stage_threshold, cs.tree_nodes, cs.node_left, cs.node_right, cs.node_feature,
            cs.node_threshold, cs.leaves, cs.feat_rects, cs.feat_weights, cs.feat_tilted)]
        k = self._keep
        d = FMHaarDesc(cs.win_w, cs.win_h, len(cs.stage_ntrees), len(cs.tree_nodes), len(cs.node_left),
                       len(cs.leaves), len(cs.feat_tilted), *[_ptr(a) for a in k])
        h = C.c_void_p()
        rc = L.fm_haar_create(int(device), C.byref(d), C.byref(h))
        self._h = h
        if rc != FM_OK:
            msg = L.fm_haar_last_error(h).decode() if h else ""
            L.fm_haar_destroy(h)
            self._h = None
            raise FMError(rc, f"fm_haar_create: {msg}")

    def empty(self) -> bool:
        return self._h is None

    def detect_batch(self, images: np.ndarray, scaleFactor=1.1, minNeighbors=5, minSize=(0, 0), maxSize=(0, 0),
                     cap: int = 256):
        """images: [n, H, W, 3] BGR or [n, H, W] gray u8 -> list of (k, 4) int32 arrays."""
        L = load()
        imgs = np.ascontiguousarray(images, np.uint8)
        ch = 3 if imgs.ndim == 4 else 1
        n, H, W = imgs.shape[:3]
        while True:
            rects = np.zeros((n, cap, 4), np.int32)
            counts = np.zeros(n, np.int32)
            rc = L.fm_haar_detect(self._h, _ptr(imgs), n, H, W, ch, 0, float(scaleFactor), int(minNeighbors),
                                  int(minSize[0]), int(minSize[1]), int(maxSize[0]), int(maxSize[1]),
                                  _ptr(rects), cap, _ptr(counts))
            if rc != FM_OK:
                raise FMError(rc, f"fm_haar_detect: {L.fm_haar_last_error(self._h).decode()}")
            if counts.max(initial=0) <= cap:
                return [rects[i, :counts[i]].copy() for i in range(n)]
            cap = int(counts.max())

    def detect_frames(self, frames: np.ndarray, roi_w: int = 300, scaleFactor=1.1, minNeighbors=5, cap: int = 256):
        """find_objects on raw BGR frames [n, H, W, 3]: INTER_AREA to width roi_w on the device, then
        detectMultiScale; rects are in ROI coordinates (as find_motion.py:724-729 stores them).
        `frames` is a host array, a contiguous uint8 torch tensor already on the detector's GPU
        (frames resident in HBM: no host round trip; torch's current stream is synchronised first),
        or a tuple (device address, n, H, W) of frames the engine left in HBM (fm_frame_device)."""
        L = load()
        if isinstance(frames, tuple):  # (device address, n, H, W): frames left in HBM by the engine
            ptr, n, H, W = frames
            return self._detect_frames(L, C.c_void_p(ptr), int(n), int(H), int(W), 1, roi_w, scaleFactor,
                                       minNeighbors, cap)
        if getattr(frames, "is_cuda", False):
            import torch
            if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3 or not frames.is_contiguous():
                raise ValueError("device frames must be a contiguous uint8 tensor [n, H, W, 3]")
            torch.cuda.current_stream(frames.device).synchronize()
            fr, ptr, on_dev = frames, C.c_void_p(frames.data_ptr()), 1
        else:
            fr = np.ascontiguousarray(frames, np.uint8)
            ptr, on_dev = _ptr(fr), 0
        n, H, W = (int(v) for v in fr.shape[:3])
        return self._detect_frames(L, ptr, n, H, W, on_dev, roi_w, scaleFactor, minNeighbors, cap)

    def detect_frame_list(self, ptrs, H: int, W: int, roi_w: int = 300, scaleFactor=1.1, minNeighbors=5,
                          cap: int = 256):
        """find_objects on raw BGR frames already in device memory at separate addresses (e.g. the ROI frames
        of many streams left in an engine's ring or input slots): `ptrs` = their device addresses, each
        frame [H, W, 3].  The resize reads them in place (fm_haar_detect_frame_list); rects in ROI
        coordinates.  The frames must be complete on the device (the caller synchronises its streams)."""
        L = load()
        n = len(ptrs)
        arr = (C.c_void_p * n)(*[int(p) for p in ptrs])
        rh = C.c_int32()
        while True:
            rects = np.zeros((n, cap, 4), np.int32)
            counts = np.zeros(n, np.int32)
            rc = L.fm_haar_detect_frame_list(self._h, C.cast(arr, C.c_void_p), n, int(H), int(W), int(roi_w),
                                             float(scaleFactor), int(minNeighbors), _ptr(rects), cap, _ptr(counts),
                                             C.byref(rh))
            if rc != FM_OK:
                raise FMError(rc, f"fm_haar_detect_frame_list: {L.fm_haar_last_error(self._h).decode()}")
            if counts.max(initial=0) <= cap:
                return [rects[i, :counts[i]].copy() for i in range(n)]
            cap = int(counts.max())

    def detect_frame_list_async(self, ptrs, H: int, W: int, roi_w: int = 300, scaleFactor=1.1, minNeighbors=5) -> int:
        """detect_frame_list queued on the detector's own stream without waiting (fm_haar_detect_frame_list_async);
        `collect` returns its results.  One detection in flight per detector; the frames must stay in place
        until it is collected.  Returns the number of frames queued."""
        L = load()
        n = len(ptrs)
        arr = (C.c_void_p * n)(*[int(p) for p in ptrs])
        rh = C.c_int32()
        rc = L.fm_haar_detect_frame_list_async(self._h, C.cast(arr, C.c_void_p), n, int(H), int(W), int(roi_w),
                                               float(scaleFactor), int(minNeighbors), C.byref(rh))
        if rc != FM_OK:
            raise FMError(rc, f"fm_haar_detect_frame_list_async: {L.fm_haar_last_error(self._h).decode()}")
        return n

    def collect(self, n: int, cap: int = 256):
        """The queued detection's results (waits for it): a list of [k, 4] rect arrays, one per frame."""
        L = load()
        while True:
            rects = np.zeros((n, cap, 4), np.int32)
            counts = np.zeros(n, np.int32)
            rc = L.fm_haar_collect(self._h, _ptr(rects), cap, _ptr(counts), int(n))
            if rc != FM_OK:
                raise FMError(rc, f"fm_haar_collect: {L.fm_haar_last_error(self._h).decode()}")
            if counts.max(initial=0) <= cap:
                return [rects[i, :counts[i]].copy() for i in range(n)]
            cap = int(counts.max())

    def _detect_frames(self, L, ptr, n, H, W, on_dev, roi_w, scaleFactor, minNeighbors, cap):
        rh = C.c_int32()
        while True:
            rects = np.zeros((n, cap, 4), np.int32)
            counts = np.zeros(n, np.int32)
            rc = L.fm_haar_detect_frames(self._h, ptr, n, H, W, on_dev, int(roi_w), float(scaleFactor),
                                         int(minNeighbors), _ptr(rects), cap, _ptr(counts), C.byref(rh))
            if rc != FM_OK:
                raise FMError(rc, f"fm_haar_detect_frames: {L.fm_haar_last_error(self._h).decode()}")
            if counts.max(initial=0) <= cap:
                return [rects[i, :counts[i]].copy() for i in range(n)]
            cap = int(counts.max())

    def detectMultiScale(self, image, scaleFactor=1.1, minNeighbors=5, flags=0, minSize=(0, 0), maxSize=(0, 0)):
        r = self.detect_batch(np.asarray(image)[None], scaleFactor, minNeighbors, minSize or (0, 0),
                              maxSize or (0, 0))[0]
        return r if len(r) else ()

    def candidates(self) -> np.ndarray:
        """Ungrouped candidates of image 0 of the last call (parity tests)."""
        L = load()
        n = L.fm_haar_candidates(self._h, None, 0)
        out = np.zeros((max(n, 1), 4), np.int32)
        L.fm_haar_candidates(self._h, _ptr(out), n)
        return out[:n]

    def last_ms(self) -> float:
        return float(load().fm_haar_last_ms(self._h))

    def close(self):
        if self._h:
            load().fm_haar_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _jpeg_arrays(jpegs):
    """(pointer array, size array, keep-alive list) for a sequence of JPEG byte strings."""
    keep = [np.frombuffer(j, np.uint8) if not isinstance(j, np.ndarray) else np.ascontiguousarray(j, np.uint8)
            for j in jpegs]
    ptrs = np.array([k.ctypes.data for k in keep], np.uint64)
    sizes = np.array([k.size for k in keep], np.uint64)
    return ptrs, sizes, keep


class MJpegDecoder:
    """The decode side on the GPU: baseline JPEG frames of an MJPEG stream ->
    BGR u8 frames as cv2.VideoCapture.read returns them (fm.py:497-506), libjpeg-turbo's default
    decode reproduced bit for bit (jpeg_idct_islow, fancy upsampling, integer YCbCr tables)."""

    def __init__(self, width: int, height: int, max_frames: int = 64, device: int = 0,
                 chunk_bits: int | None = None, spec_bits: int | None = None):
        L = load()
        h = C.c_void_p()
        rc = L.fm_mjpeg_create(int(device), int(width), int(height), int(max_frames), C.byref(h))
        self._h = h
        if rc != FM_OK:
            msg = L.fm_mjpeg_last_error(h).decode() if h else ""
            L.fm_mjpeg_destroy(h)
            self._h = None
            raise FMError(rc, f"fm_mjpeg_create: {msg}")
        self.width, self.height, self.max_frames = int(width), int(height), int(max_frames)
        if chunk_bits is not None or spec_bits is not None:  # fm_mjpeg_tune: speed only, same results
            rc = L.fm_mjpeg_tune(h, int(chunk_bits or 512), int(512 if spec_bits is None else spec_bits))
            if rc != FM_OK:
                msg = L.fm_mjpeg_last_error(h).decode()
                self.close()
                raise FMError(rc, f"fm_mjpeg_tune: {msg}")

    def decode(self, jpegs) -> np.ndarray:
        """JPEG byte strings -> BGR u8 [n, H, W, 3] (host)."""
        L = load()
        ptrs, sizes, keep = _jpeg_arrays(jpegs)
        out = np.empty((len(keep), self.height, self.width, 3), np.uint8)
        rc = L.fm_mjpeg_decode(self._h, _ptr(ptrs), _ptr(sizes), len(keep), _ptr(out), 0)
        if rc != FM_OK:
            raise FMError(rc, f"fm_mjpeg_decode: {L.fm_mjpeg_last_error(self._h).decode()}")
        return out

    def decode_device(self, jpegs, ptr: int) -> None:
        """JPEG byte strings -> BGR frames at device address ptr (synchronous)."""
        L = load()
        ptrs, sizes, keep = _jpeg_arrays(jpegs)
        rc = L.fm_mjpeg_decode(self._h, _ptr(ptrs), _ptr(sizes), len(keep), C.c_void_p(ptr), 1)
        if rc != FM_OK:
            raise FMError(rc, f"fm_mjpeg_decode: {L.fm_mjpeg_last_error(self._h).decode()}")

    def last_ms(self) -> float:
        return float(load().fm_mjpeg_last_ms(self._h))

    def close(self):
        if self._h:
            load().fm_mjpeg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
