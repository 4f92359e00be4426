"""ctypes wrapper over oracle/fm_oracle.c (the C restatement).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Each wrapper names the
reference call site it restates (fm.py = find_motion/find_motion.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libfm_oracle.so")
_lib = None

u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile the C restatement (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "fm_oracle.c")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        L.fmo_reflect101.argtypes = [C.c_int, C.c_int]
        L.fmo_area_tab_size.argtypes = [C.c_int, C.c_int]
        L.fmo_work_height.argtypes = [C.c_int, C.c_int, C.c_int]
        L.fmo_resize_area_bgr.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_int, C.c_int]
        L.fmo_bgr2gray.argtypes = [u8p, C.c_size_t, u8p]
        L.fmo_gauss_coeffs.argtypes = [C.c_int, i32p]
        L.fmo_gauss_blur.argtypes = [u8p, C.c_int, C.c_int, C.c_int, u8p]
        L.fmo_diff_thresh.argtypes = [u8p, f64p, C.c_size_t, C.c_int, u8p, u8p]
        L.fmo_accumulate.argtypes = [u8p, f64p, C.c_size_t, C.c_double]
        L.fmo_dilate5.argtypes = [u8p, C.c_int, C.c_int, u8p]
        L.fmo_find_contours_ext.argtypes = [u8p, C.c_int, C.c_int, i32p, f64p, C.c_int, C.c_void_p, C.c_int]
        L.fmo_process_frame.argtypes = [
            C.c_void_p, u8p, C.c_void_p, f64p, C.POINTER(C.c_int),
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, i32p, f64p, C.c_int,
        ]
        L.fmo_process_sequence.argtypes = [
            C.c_void_p, u8p, C.c_int, C.c_void_p, f64p, C.POINTER(C.c_int), C.c_void_p,
            i32p, i32p, C.c_void_p, C.c_int, C.c_int,
        ]
        L.fmo_run_streams.argtypes = [C.c_void_p, u8p, C.c_int, C.c_int, C.c_int, i32p, C.c_int]
        _lib = L
    return _lib


class _Cfg(C.Structure):
    _fields_ = [("H", C.c_int), ("W", C.c_int), ("h", C.c_int), ("w", C.c_int),
                ("ksize", C.c_int), ("thresh", C.c_int), ("alpha", C.c_double)]


def make_gaussian(box_size: int, blur_scale: int) -> int:
    """VideoMotion._make_gaussian (fm.py:478-484): k = int(box/scale), made odd."""
    k = int(box_size / blur_scale)
    return k + 1 if k % 2 == 0 else k


def work_height(H: int, W: int, box: int) -> int:
    """imutils.resize(width=box) height rule (fm.py:492): int(H * (box / float(W)))."""
    return int(H * (box / float(W)))


def resize_area_bgr(src: np.ndarray, w: int) -> np.ndarray:
    """imutils.resize(raw, width=w) -> cv2.resize(INTER_AREA) (fm.py:492)."""
    H, W, _ = src.shape
    h = work_height(H, W, w)
    out = np.empty((h, w, 3), np.uint8)
    if lib().fmo_resize_area_bgr(np.ascontiguousarray(src), H, W, out, h, w) != 0:
        raise ValueError("INTER_AREA upscaling is not part of the restated path")
    return out


def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(BGR2GRAY) (fm.py:493)."""
    out = np.empty(bgr.shape[:2], np.uint8)
    lib().fmo_bgr2gray(np.ascontiguousarray(bgr), out.size, out)
    return out


def gauss_coeffs(k: int) -> np.ndarray:
    """8-bit fixed-point Gaussian taps used by GaussianBlur(u8, (k,k), 0)."""
    out = np.zeros(k, np.int32)
    if lib().fmo_gauss_coeffs(k, out) != 0:
        raise ValueError(f"bad ksize {k}")
    return out


def gauss_blur(gray: np.ndarray, k: int) -> np.ndarray:
    """cv2.GaussianBlur(gray, (k,k), 0) (fm.py:494)."""
    out = np.empty_like(gray)
    if lib().fmo_gauss_blur(np.ascontiguousarray(gray), gray.shape[0], gray.shape[1], k, out) != 0:
        raise ValueError(f"bad ksize {k}")
    return out


def diff_thresh(blur: np.ndarray, bg: np.ndarray, t: int):
    """absdiff(blur, convertScaleAbs(bg)) and threshold(BINARY) (fm.py:246-257)."""
    delta = np.empty_like(blur)
    th = np.empty_like(blur)
    lib().fmo_diff_thresh(np.ascontiguousarray(blur), np.ascontiguousarray(bg), blur.size, int(t), delta, th)
    return delta, th


def accumulate(blur: np.ndarray, bg: np.ndarray, alpha: float) -> None:
    """cv2.accumulateWeighted(blur, bg, alpha), in place on bg (fm.py:659)."""
    assert bg.flags.c_contiguous and bg.dtype == np.float64
    lib().fmo_accumulate(np.ascontiguousarray(blur), bg, blur.size, float(alpha))


def dilate5(th: np.ndarray) -> np.ndarray:
    """cv2.dilate(thresh, None, iterations=2) (fm.py:266)."""
    out = np.empty_like(th)
    lib().fmo_dilate5(np.ascontiguousarray(th), th.shape[0], th.shape[1], out)
    return out


def find_contours_ext(mask: np.ndarray, cap: int = 1 << 16, with_points: bool = False, pts_cap: int = 4096):
    """cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) (fm.py:269-272).

    Returns a list of dicts {bbox:(x,y,w,h), area, origin:(x,y), npts[, points]}
    in scan order of the contours' start pixels.
    """
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    h, w = mask.shape
    rec = np.zeros((cap, 7), np.int32)
    areas = np.zeros(cap, np.float64)
    pts = None
    if with_points:
        pts = np.zeros((cap, pts_cap, 2), np.int32)
    n = lib().fmo_find_contours_ext(mask, h, w, rec, areas, cap,
                                    pts.ctypes.data if pts is not None else None, pts_cap)
    out = []
    for i in range(min(n, cap)):
        r = rec[i]
        d = {"bbox": (int(r[0]), int(r[1]), int(r[2]), int(r[3])), "area": float(areas[i]),
             "origin": (int(r[4]), int(r[5])), "npts": int(r[6])}
        if with_points:
            d["points"] = pts[i, : min(int(r[6]), pts_cap)].copy()
        out.append(d)
    if n > cap:
        raise RuntimeError("contour capacity exceeded")
    return out


@dataclass
class OracleConfig:
    H: int
    W: int
    box: int
    ksize: int
    thresh: int = 12
    alpha: float = 0.1

    @property
    def h(self) -> int:
        return work_height(self.H, self.W, self.box)

    @property
    def w(self) -> int:
        return self.box

    def _c(self) -> _Cfg:
        return _Cfg(self.H, self.W, self.h, self.w, self.ksize, self.thresh, self.alpha)


class OracleStream:
    """One stream's find_motion state (VideoMotion.ref_frame, fm.py:363,651-659)."""

    def __init__(self, cfg: OracleConfig, keep: np.ndarray | None = None):
        self.cfg = cfg
        self._c = cfg._c()
        self.bg = np.zeros((cfg.h, cfg.w), np.float64)
        self._init = C.c_int(0)
        self.keep = None if keep is None else np.ascontiguousarray(keep, dtype=np.uint8)

    @property
    def initialized(self) -> bool:
        return bool(self._init.value)

    def step(self, bgr: np.ndarray, cap: int = 4096) -> dict:
        """blur_frame + mask_off_areas + find_diff for one frame (fm.py:866-868)."""
        c = self.cfg
        assert bgr.shape == (c.H, c.W, 3) and bgr.dtype == np.uint8
        gray = np.empty((c.h, c.w), np.uint8)
        blur = np.empty_like(gray)
        delta = np.empty_like(gray)
        mask = np.empty_like(gray)
        rec = np.zeros((cap, 7), np.int32)
        areas = np.zeros(cap, np.float64)
        n = lib().fmo_process_frame(
            C.byref(self._c), np.ascontiguousarray(bgr),
            self.keep.ctypes.data if self.keep is not None else None,
            self.bg, C.byref(self._init),
            gray.ctypes.data, blur.ctypes.data, delta.ctypes.data, mask.ctypes.data,
            rec, areas, cap,
        )
        if n < 0:
            raise RuntimeError("oracle frame step failed")
        boxes = [tuple(int(v) for v in rec[i, :4]) for i in range(min(n, cap))]
        origins = [(int(rec[i, 4]), int(rec[i, 5])) for i in range(min(n, cap))]
        return {"gray": gray, "blur": blur, "delta": delta, "mask": mask, "count": int(n),
                "boxes": boxes, "origins": origins, "areas": areas[: min(n, cap)].copy()}


class _SeqResult:
    """Per-frame results of OracleStream.run: counts[F], boxes(f), origins(f), areas(f), masks{f: plane}."""

    def __init__(self, counts, rec, areas, masks):
        self.counts, self._rec, self._areas, self.masks = counts, rec, areas, masks

    def boxes(self, f: int) -> list:
        n = min(int(self.counts[f]), self._rec.shape[1])
        return [tuple(int(v) for v in self._rec[f, i, :4]) for i in range(n)]

    def origins(self, f: int) -> list:
        n = min(int(self.counts[f]), self._rec.shape[1])
        return [(int(self._rec[f, i, 4]), int(self._rec[f, i, 5])) for i in range(n)]

    def areas(self, f: int) -> np.ndarray:
        n = min(int(self.counts[f]), self._rec.shape[1])
        return self._areas[f, :n].copy()


def _run_sequence(self, frames: np.ndarray, cap: int = 4096, mask_frames=(), nthreads: int = 0) -> _SeqResult:
    """step() over frames [F][H][W][3] (one stream, in order), frames in parallel where
    find_diff's data flow allows it (fmo_process_sequence; identical arithmetic)."""
    c = self.cfg
    frames = np.ascontiguousarray(frames)
    assert frames.ndim == 4 and frames.shape[1:] == (c.H, c.W, 3) and frames.dtype == np.uint8
    F = frames.shape[0]
    counts = np.zeros(F, np.int32)
    rec = np.zeros((F, cap, 7), np.int32)
    areas = np.zeros((F, cap), np.float64)
    masks = {int(f): np.empty((c.h, c.w), np.uint8) for f in mask_frames}
    ptrs = (C.c_void_p * F)(*[masks[f].ctypes.data if f in masks else None for f in range(F)])
    rc = lib().fmo_process_sequence(
        C.byref(self._c), frames, F, self.keep.ctypes.data if self.keep is not None else None,
        self.bg, C.byref(self._init), ptrs, counts, rec, areas.ctypes.data, cap, int(nthreads))
    if rc < 0:
        raise RuntimeError("oracle sequence failed")
    if int(counts.max(initial=0)) > cap:
        raise RuntimeError("contour capacity exceeded")
    return _SeqResult(counts, rec, areas, masks)


OracleStream.run = _run_sequence


def run_streams(cfg: OracleConfig, frames: np.ndarray, nthreads: int = 0, n_streams: int | None = None):
    """CPU baseline, one thread per stream.  frames [S][F][H][W][3], or
    [F][H][W][3] replayed by each of n_streams streams.  Returns (counts[S][F], threads)."""
    shared = frames.ndim == 4
    if shared:
        S, F = int(n_streams or 1), frames.shape[0]
    else:
        S, F = frames.shape[:2]
    counts = np.zeros((S, F), np.int32)
    c = cfg._c()
    used = lib().fmo_run_streams(C.byref(c), np.ascontiguousarray(frames), S, F, int(nthreads), counts,
                                 1 if shared else 0)
    return counts, int(used)
