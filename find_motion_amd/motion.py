"""Drop-in VideoMotion / VideoFrame whose per-frame cv2 chain runs on MI355X.

Mirrors the reference's classes (find_motion/find_motion.py, "fm.py"):

* VideoFrame  (fm.py:230-291) -- same attributes: raw, frame, in_cache,
  contours, frame_delta, gray, thresh, blur, resized;
* VideoMotion (fm.py:294-926) -- same constructor arguments and methods,
  the same frame loop (find_motion, fm.py:852-904), the same movement /
  output state machine (find_movement fm.py:665-700, decide_output
  fm.py:549-589, cleanup_cache fm.py:592-601) and writer behaviour.

What changes is the hot path.  blur_frame / mask_off_areas / find_diff
(fm.py:487-494, 619-636, 638-662) no longer call cv2: the frames go through
the C ABI (include/find_motion_amd.h) into one fused HIP kernel plus a GPU
connected-components pass, and the results are bound back onto the
VideoFrame:

* frame.contours -- one Contour per external contour (len = the count
  find_movement adds up, fm.py:694); Contour.bbox is cv2.boundingRect;
* frame.thresh   -- the dilated threshold mask (fm.py:266), fetched from the
  device on first access;
* frame.gray / frame.blur / frame.frame_delta -- fetched on access when the
  engine keeps planes (show or debug), else None;
* VideoMotion.ref_frame -- the float64 background, read from the device on
  access.  The mask polygons are rasterised once per video (they are static)
  and applied inside the kernel, so mask_off_areas() has nothing left to do.

Capture: cv2.VideoCapture whenever OpenCV imports, as the reference does
(fm.py:413).  MJPEG AVIs are decoded on the GPU in front of the hot path
(videoio.MjpegAviCapture + fm_submit_jpeg) when the caller
opts in (gpu_decode=True) or OpenCV is absent: frame.raw is then fetched from
the device on first access (a frame the state machine writes, shows or runs a
cascade on), and an MJPG output receives the source's JPEG bytes unchanged
instead of a re-encode.  That decode equals libjpeg-turbo's (cv2.imdecode),
not FFmpeg's (cv2.VideoCapture's default backend): see videoio.

Extra keyword arguments (not in the reference): device (HIP ordinal),
batch (frames decoded ahead and processed per kernel launch; the per-frame
results and the decisions are identical for any batch -- only ref_frame is
then observed at batch boundaries), capture (a ready capture object),
gpu_decode (see above).

There is no CPU fallback: without the HIP library this module raises
NativeLibraryMissing at VideoMotion construction.
"""
from __future__ import annotations

import copy
import importlib.util
import logging
import math
import os
import typing
from collections import deque

import numpy as np

from . import videoio
from ._native import (PLANE_BLUR, PLANE_DELTA, PLANE_GRAY, CascadeClassifier, MJpegDecoder, MotionEngine,
                      rasterize_masks)
from .feeder import BatchFeeder

log = logging.getLogger("find_motion_amd")

BLACK = (0, 0, 0)
RED = (0, 0, 255)
GREEN = (0, 255, 0)

# fm.py:104-122
_CASCADES: dict = {}  # (path, device) -> CascadeClassifier

CASCADE_LOOKUP = {
    "frontalcatface": "Cat 1",
    "frontalcatface_extended": "Cat 2",
    "frontalface_alt": "Face 1",
    "frontalface_alt2": "Face 2",
    "frontalface_alt_tree": "Face 3",
    "frontalface_default": "Face 4",
    "fullbody": "Person",
    "lowerbody": "Legs",
    "profileface": "Face 5",
}


class VideoError(Exception):
    """fm.py:173-178"""


def make_gaussian_size(box_size: int, blur_scale: int) -> int:
    """VideoMotion._make_gaussian (fm.py:478-484)."""
    k = int(box_size / blur_scale)
    return k + 1 if k % 2 == 0 else k


class _Bound:
    """Where a frame's results live: (engine, batch generation, frame index in the batch, stream)."""

    __slots__ = ("engine", "gen", "t", "s")

    def __init__(self, engine, gen, t, s):
        self.engine, self.gen, self.t, self.s = engine, gen, t, s

    def fetch(self, what):
        eng = self.engine
        if eng.generation != self.gen:
            raise RuntimeError("frame results were overwritten by a later batch; read them before the next batch")
        if what == "thresh":
            return eng.mask(self.t, self.s)
        if not eng.keep_planes:
            return None
        return eng.plane({"gray": PLANE_GRAY, "blur": PLANE_BLUR, "frame_delta": PLANE_DELTA}[what], self.t, self.s)


class VideoFrame:
    """fm.py:230-291.  Holds one decoded frame and the hot path's results for it."""

    _LAZY = ("gray", "blur", "frame_delta", "thresh")

    def __init__(self, frame, show: bool = False, jpeg: bytes = None) -> None:
        self._raw = frame
        self.jpeg = jpeg  # MJPEG input: the compressed source frame (raw is decoded on the GPU)
        self._load = None  # MJPEG input: fetches raw on first access (VideoMotion.bind_results)
        self._show = show
        # fm.py:236 always copies raw; the copy is only drawn on (show), so it is made only then
        if frame is not None:
            self.frame = frame.copy() if show else frame
        self.in_cache = False
        self.contours: list = []
        self.resized = None
        self._bound: typing.Optional[_Bound] = None
        self._vals: dict = {}
        self.processed = False
        self.index = -1  # position in the source (set when the engine processes the frame)

    @property
    def raw(self):
        r = self._raw
        if r is None:
            if self._load is None:
                raise AttributeError("raw")
            r = self._raw = self._load()
        return r

    @raw.setter
    def raw(self, value):
        self._raw = value

    def __getattr__(self, name):
        # frame of an MJPEG input, made from raw on first access like fm.py:236
        d = self.__dict__
        if name == "frame" and d.get("_load") is not None:
            f = self.raw.copy() if d.get("_show") else self.raw
            d["frame"] = f
            return f
        raise AttributeError(name)

    def _get(self, name):
        if name in self._vals:
            return self._vals[name]
        b = self._bound
        if b is None:
            return None
        v = b.fetch(name)
        self._vals[name] = v
        return v

    gray = property(lambda s: s._get("gray"), lambda s, v: s._vals.__setitem__("gray", v))
    blur = property(lambda s: s._get("blur"), lambda s, v: s._vals.__setitem__("blur", v))
    frame_delta = property(lambda s: s._get("frame_delta"), lambda s, v: s._vals.__setitem__("frame_delta", v))
    thresh = property(lambda s: s._get("thresh"), lambda s, v: s._vals.__setitem__("thresh", v))

    # fm.py:246-276 compute on the device (VideoMotion.find_diff); on a frame the
    # engine has already processed these are no-ops that keep the reference's surface
    def diff(self, ref_frame) -> None:
        self._require()

    def threshold(self, thresh) -> None:
        self._require()

    def find_contours(self) -> None:
        self._require()

    def _require(self):
        if not self.processed:
            raise RuntimeError("VideoFrame ops run on the GPU: pass the frame through VideoMotion.blur_frame/find_diff")

    def cleanup(self) -> None:
        """fm.py:279-291"""
        for attr in ("frame", "contours"):
            if attr in self.__dict__:
                delattr(self, attr)
        self._vals.clear()
        self._bound = None
        if self.in_cache:
            return
        self._raw = self._load = self.jpeg = None


class VideoMotion:
    """fm.py:294-926 with the per-frame chain on the GPU (see the module docstring)."""

    DEFAULT_MIN_BOX_SCALE = 50  # -m / min_box_scale default (fm.py:300)
    # pylint: disable=too-many-instance-attributes,too-many-arguments
    def __init__(self, filename: typing.Union[str, int, None] = None, outdir: str = "", fps: int = 30,
                 box_size: int = 100, min_box_scale: int = DEFAULT_MIN_BOX_SCALE, cache_time: float = 2.0,
                 min_time: float = 0.5,
                 threshold: int = 7, avg: float = 0.1, blur_scale: int = 20,
                 mask_areas: list = None, show: bool = False,
                 codec: str = "MJPG", log_level: int = logging.INFO,
                 mem: bool = False, cleanup: bool = False,
                 multiprocess: bool = False,
                 cascades: typing.List[str] = None,
                 yolo_tiny: bool = False, *,
                 device: int = 0, batch: int = 1, capture=None, engine: MotionEngine = None,
                 stream: int = 0, keep_planes: bool = None, cascade_dir: str = None,
                 pipeline_depth: int = None, gpu_decode: bool = None) -> None:
        self.filename = filename
        if self.filename is None and capture is None:
            raise Exception("Filename required")
        self.log = logging.getLogger("find_motion_amd.VideoMotion")
        self.log.setLevel(log_level)
        self.multiprocess = multiprocess
        self.outfile = None
        self.outfiles = 0
        self.outfile_name = ""
        self.outdir = os.path.normpath(outdir)
        self.fps = fps
        self.box_size = box_size
        self.min_box_scale = min_box_scale
        self.min_area = -1
        self.max_area = -1
        self.area_filter = False  # max_area < min_area: fm.py:684 filters by contourArea
        self.gaussian_scale = blur_scale
        self.cache_frames = int(cache_time * fps)
        self.min_movement_frames = int(min_time * fps)
        self.delta_thresh = threshold
        self.avg = avg
        self.mask_areas = mask_areas if mask_areas is not None else []
        self.show = show
        self.cascade_names = cascades
        self.cascade_dir = cascade_dir
        self.device = int(device)
        self.codec = codec
        self.debug = log_level == logging.DEBUG
        self.mem = mem
        self.cleanup_flag = cleanup
        self.cascades = None
        self._load_cascades()
        self.tiny = yolo_tiny
        self.amount_of_frames = -1
        self.frame_width = -1
        self.frame_height = -1
        self.scale = -1.0
        self.current_frame: typing.Optional[VideoFrame] = None
        self.frame_cache: typing.Deque[VideoFrame] = deque()
        self.wrote_frames: typing.Optional[bool] = False
        self.err_msg = ""
        self.movement = False
        self.movement_decay = 0
        self.movement_counter = 0
        self.object_counter = 0
        self.last_objects: typing.Dict[str, typing.List] = {}
        self.seen_objects: typing.Set[str] = set()
        # MI355X engine
        self.device = int(device)
        self.batch = max(1, int(batch))
        self.keep_planes = (show or self.debug) if keep_planes is None else bool(keep_planes)
        self._engine = engine
        self._own_engine = engine is None
        self._pipe = None  # BatchFeeder iterator of read() (single-stream engine)
        # batches in flight on the GPU ahead of the frame being consumed (None: fm_max_inflight);
        # 1 keeps ref_frame readable after every batch (the engine is idle when a batch is handed out)
        self.pipeline_depth = pipeline_depth
        self._stream = int(stream)
        self._capture = capture
        self.gpu_decode = gpu_decode
        self._ahead: typing.Deque[VideoFrame] = deque()
        self.frames_read = 0
        self._jpeg_dec = None  # one-frame GPU decoder for raw frames of batches already overwritten
        self.written_indices: typing.List[int] = []  # source frame indices written, in write order
        self._calc_min_area()
        self._make_gaussian()
        self.loaded = self._load_video()

    # -- init (fm.py:383-484) ------------------------------------------------
    def _load_cascades(self) -> None:
        """fm.py:383-399: the named cascades, read from haarcascade_<name>.xml and run on the GPU
        (find_motion_amd.CascadeClassifier).  Files are looked up in `cascade_dir`, $FM_HAARCASCADES,
        the installed reference package's haarcascades/ (FIND_MOTION_PATH), then cv2.data."""
        self.cascades = dict()
        if self.cascade_names is None:
            return
        names = copy.copy(CASCADE_LOOKUP) if "ALL" in self.cascade_names else {
            c: CASCADE_LOOKUP[c] for c in self.cascade_names if c in CASCADE_LOOKUP}
        dirs = [d for d in (self.cascade_dir, os.environ.get("FM_HAARCASCADES")) if d]
        spec = importlib.util.find_spec("find_motion")
        if spec is not None and spec.origin:
            dirs.append(os.path.join(os.path.dirname(spec.origin), "haarcascades"))
        cv2 = videoio.cv2
        if cv2 is not None and hasattr(cv2, "data"):
            dirs.append(cv2.data.haarcascades)
        for c, title in names.items():
            path = next((os.path.join(d, f"haarcascade_{c}.xml") for d in dirs
                         if os.path.isfile(os.path.join(d, f"haarcascade_{c}.xml"))), None)
            if path is None:
                self.log.warning("cascade %s not found in %s: skipped", c, dirs)
                continue
            key = (os.path.realpath(path), self.device)
            if key not in _CASCADES:  # one device copy per file and device, shared by every stream
                _CASCADES[key] = CascadeClassifier(path, device=self.device)
            self.cascades[title] = _CASCADES[key]

    def _calc_min_area(self) -> None:
        """fm.py:402-406"""
        self.min_area = int(math.pow(self.box_size / self.min_box_scale, 2))

    def _make_gaussian(self) -> None:
        """fm.py:478-484"""
        g = make_gaussian_size(self.box_size, self.gaussian_scale)
        self.gaussian = (g, g)

    def _load_video(self) -> bool:
        """fm.py:409-424, plus engine creation and the one-time mask rasterisation."""
        self.cap = videoio.open_capture(self._capture if self._capture is not None else self.filename, self.device,
                                        self.gpu_decode)
        self.frame_cache = deque(maxlen=self.cache_frames)
        try:
            self._get_video_info()
        except VideoError as e:
            self.log.error(str(e))
            return False
        self.scale = self.box_size / self.frame_width
        self.max_area = int((self.frame_width * self.frame_height) / 2 * self.scale)
        # the contourArea filter of fm.py:684 can skip a contour only when max_area < min_area:
        # then the engine traces every external contour's border on the GPU for its area
        self.area_filter = self.max_area < self.min_area
        if self._engine is None:
            self._engine = MotionEngine(n_streams=1, src_w=self.frame_width, src_h=self.frame_height,
                                        box_size=self.box_size, ksize=self.gaussian[0], threshold=self.delta_thresh,
                                        avg=self.avg, max_batch=self.batch, keep_planes=self.keep_planes,
                                        device=self.device, contour_area=self.area_filter)
        if self.mask_areas:
            h, w = self._engine.work_shape
            self._engine.set_mask(self._stream, rasterize_masks(h, w, self.scale, self.mask_areas))
        return True

    def _get_video_info(self) -> None:
        """fm.py:427-444"""
        self.amount_of_frames = int(self.cap.get(videoio.CAP_PROP_FRAME_COUNT))
        self.frame_width = int(self.cap.get(videoio.CAP_PROP_FRAME_WIDTH))
        self.frame_height = int(self.cap.get(videoio.CAP_PROP_FRAME_HEIGHT))
        if self.frame_width == 0 or self.frame_height == 0:
            broken = "width" if self.frame_width == 0 else "height"
            raise VideoError("Video info malformed - {} is 0: {}".format(broken, self.filename))
        if self.amount_of_frames == 0:
            log.warning("Video info malformed - frames reported as 0")

    @property
    def engine(self) -> MotionEngine:
        return self._engine

    # -- background state (VideoMotion.ref_frame, fm.py:363, 414, 651-659) ----
    @property
    def ref_frame(self):
        """float64 background after the most recent batch (None before the first frame)."""
        eng = self._engine
        if eng is None or not eng.initialized(self._stream):
            return None
        return eng.background(self._stream)

    @ref_frame.setter
    def ref_frame(self, value):
        eng = self._engine
        if eng is None:
            return
        if value is None:
            eng.reset(self._stream)
        else:
            eng.set_background(self._stream, np.asarray(value, dtype=np.float64))

    # -- I/O (fm.py:497-546) ---------------------------------------------------
    def read(self) -> bool:
        """fm.py:497-506.  Frames are decoded ahead by a BatchFeeder thread into page-locked
        batches of `batch` frames, up to fm_max_inflight batches in flight on the GPU; read()
        hands out the processed frames one by one, in order."""
        if not self._ahead:
            eng = self._engine
            if eng.n_streams != 1:
                raise RuntimeError("a shared multi-stream engine is driven by StreamGroup")
            if self._pipe is None:
                self._pipe = iter(BatchFeeder(eng, [self.cap], self.batch, self.pipeline_depth))
            b = next(self._pipe, None)
            if b is None:
                return False
            vfs = self.make_frames(b, 0)
            self.bind_results(vfs, eng, 0)
            self._ahead.extend(vfs)
        self.current_frame = self._ahead.popleft()
        return True

    def make_frames(self, b, stream: int) -> list:
        """VideoFrames of stream `stream` of a waited feeder batch (JPEG batches: raw fetched lazily)."""
        if b.jpegs is not None:
            return [VideoFrame(None, self.show, jpeg=j) for j in b.frames[stream]]
        return [VideoFrame(r, self.show) for r in b.frames[stream]]

    def _raw_loader(self, eng, gen: int, t: int, s: int, jpeg: bytes):
        def load():
            if eng.generation == gen:  # the batch's decoded frame is still in the engine's input slot
                return eng.read_frame(t, s)
            if self._jpeg_dec is None:
                self._jpeg_dec = MJpegDecoder(self.frame_width, self.frame_height, 1, device=self.device)
            return videoio.decode_one(self._jpeg_dec, jpeg)
        return load

    def bind_results(self, vfs, eng, stream: int) -> None:
        for t, vf in enumerate(vfs):
            if vf.jpeg is not None and vf._raw is None:
                vf._load = self._raw_loader(eng, eng.generation, t, stream, vf.jpeg)
            vf._bound = _Bound(eng, eng.generation, t, stream)
            vf.contours = eng.contours(t, stream)
            vf.processed = True
            vf.index = self.frames_read
            self.frames_read += 1

    def _make_outfile(self) -> None:
        """fm.py:447-475"""
        self.outfiles += 1
        if self.outfiles > 1 and self.outfile is not None:
            self.outfile.release()
        outname = str(self.filename) + "_" + str(self.outfiles)
        if self.outdir in ("", "."):
            self.outfile_name = outname + "_motion.avi"
        else:
            self.outfile_name = os.path.join(self.outdir, os.path.basename(outname)) + "_motion.avi"
        self.outfile = videoio.open_writer(self.outfile_name, self.codec, self.fps,
                                           (self.frame_width, self.frame_height),
                                           jpeg=hasattr(self.cap, "read_jpeg"))

    def output_frame(self, frame: VideoFrame = None) -> None:
        """fm.py:509-530"""
        frame = self.current_frame if frame is None else frame
        if self.show and videoio.cv2 is not None:
            videoio.cv2.imshow("frame", frame.frame)
        self._write_frame(frame)

    def output_raw_frame(self, frame: np.ndarray = None, index: int = -1) -> None:
        """fm.py:533-546"""
        self._write(frame, index)

    def _write_frame(self, frame: VideoFrame) -> None:
        self._write(lambda: frame.raw, getattr(frame, "index", -1), getattr(frame, "jpeg", None))

    def _put(self, raw, jpeg) -> None:
        if jpeg is not None and hasattr(self.outfile, "write_jpeg"):
            self.outfile.write_jpeg(jpeg)  # MJPEG in, MJPG out: the source's bytes, no re-encode
        else:
            self.outfile.write(raw() if callable(raw) else raw)

    def _write(self, raw, index, jpeg=None):
        if not self.wrote_frames:
            self._make_outfile()
            self.wrote_frames = True
        try:
            self._put(raw, jpeg)
        except Exception as e:  # noqa: BLE001 (fm.py:527-530)
            self.log.warning("Having to create output file due to exception: {}".format(e))
            self._make_outfile()
            self._put(raw, jpeg)
        self.written_indices.append(index)

    # -- the hot path (fm.py:487-494, 619-636, 638-662) ------------------------
    def blur_frame(self, frame: VideoFrame = None) -> None:
        """resize -> cvtColor -> GaussianBlur: runs (fused with the rest) on the GPU at read()."""
        frame = self.current_frame if frame is None else frame
        if not frame.processed:
            if self._ahead:
                raise RuntimeError("cannot process an external frame while decoded frames are pending")
            self._process_external(frame)

    def _process_external(self, frame: VideoFrame) -> None:
        if self._pipe is not None:
            raise RuntimeError("cannot process an external frame while the decode-ahead pipeline is running")
        eng = self._engine
        eng.submit(np.asarray(frame.raw, dtype=np.uint8)[None, None])
        eng.wait()
        self.bind_results([frame], eng, self._stream)

    def mask_off_areas(self, frame: VideoFrame = None):
        """Masks are rasterised once per video (_load_video) and applied inside the fused kernel."""
        return None

    def find_diff(self, frame: VideoFrame = None) -> None:
        """absdiff/threshold/accumulateWeighted/dilate/findContours: done on the GPU with blur_frame."""
        frame = self.current_frame if frame is None else frame
        if not frame.processed:
            raise Exception("Blur frame is None")  # fm.py:648-649

    # -- consumer state machine (fm.py:549-601, 665-700) -----------------------
    def find_movement(self, frame: VideoFrame = None) -> None:
        """fm.py:665-700.  The area filter of fm.py:684 can only skip a contour when
        max_area < min_area (area_filter): then contour.area is the GPU-traced contourArea."""
        frame = self.current_frame if frame is None else frame
        self.movement = False
        self.movement_decay -= 1 if self.movement_decay > 0 else 0
        if frame.contours is not None and len(frame.contours) > 0:
            for contour in frame.contours:
                if self.area_filter and self.max_area < contour.area < self.min_area:
                    continue
                if self.show:
                    self.draw_box(self.make_box(contour, frame), frame)
                self.movement_counter += 1
                self.movement = True
        if not self.movement:
            self.movement_counter = 0

    def decide_output(self) -> None:
        """fm.py:549-589"""
        if (self.movement_counter >= self.min_movement_frames) or (self.movement_decay > 0):
            if self.movement:
                self.movement_decay = self.cache_frames
                for frame in self.frame_cache:
                    if frame is not None:
                        self._write_frame(frame)  # output_raw_frame(frame.raw), fm.py:557
                        if self.cleanup_flag:
                            frame.in_cache = False
                            frame.cleanup()
                self.frame_cache.clear()
            objects = self.find_objects()
            if objects:
                self.seen_objects.update(objects)
            if self.show:
                self.draw_text()
            self.output_frame()
        else:
            if self.cleanup_flag:
                self.cleanup_cache()
            self.frame_cache.append(self.current_frame)
            self.current_frame.in_cache = True

    def cleanup_cache(self) -> None:
        """fm.py:592-601"""
        if len(self.frame_cache) == self.cache_frames and self.cache_frames > 0:
            f = self.frame_cache.popleft()
            if f is not None:
                f.in_cache = False
                f.cleanup()

    def is_open(self) -> bool:
        """fm.py:604-608"""
        return bool(self._ahead) or self.cap.isOpened()

    @staticmethod
    def scale_area(area, scale: float) -> list:
        """fm.py:611-616"""
        return [(int(a[0] * scale), int(a[1] * scale)) for a in area]

    # -- objects (fm.py:703-762): Haar needs OpenCV; cvlib YOLO is not available offline
    def find_objects(self, frame: VideoFrame = None, width=300, skip=15, scaleFactor=1.1, minNeighbours=5,
                     confidence=0.25) -> typing.Set[str]:
        frame = self.current_frame if frame is None else frame
        self.object_counter += 1
        if self.object_counter != skip:
            return set()
        self.object_counter = 0
        self.last_objects = {}
        if self.cascades:
            # frame.resized = imutils.resize(frame.raw, width=width) happens on the device inside
            # detect_frames (INTER_AREA); rects are in ROI coordinates as in the reference
            lazy = getattr(frame, "_raw", True) is None and getattr(frame, "_load", None) is not None
            src = None if lazy else frame.raw[None]
            b = getattr(frame, "_bound", None)
            if src is None and b is not None and b.engine.generation == b.gen:
                # an MJPEG frame decoded on the GPU, its batch still current: the cascade reads it
                # where the decoder left it (fm_frame_device), no round trip through host memory
                H, W = b.engine.src_shape[:2]
                src = (b.engine.frame_device_ptr(b.t, b.s), 1, H, W)
            elif src is None:
                src = frame.raw[None]
            for title, cascade in self.cascades.items():
                found = cascade.detect_frames(src, width, scaleFactor, minNeighbours)[0]
                for rect in found:
                    self.last_objects.setdefault(title, []).append(VideoMotion.make_area_from_rect(tuple(int(v) for v in rect)))
        return set(self.last_objects.keys())

    # -- display (fm.py:765-821): only with OpenCV and --show
    @staticmethod
    def find_centre(area) -> typing.Tuple[int, int]:
        return ((area[0][0] + area[1][0]) // 2, (area[0][1] + area[1][1]) // 2)

    def draw_text(self, frame: VideoFrame = None) -> None:
        frame = self.current_frame if frame is None else frame
        if videoio.cv2 is not None:
            videoio.cv2.putText(frame.frame, "Status: {}".format("motion" if self.movement else "quiet"), (10, 20),
                                videoio.cv2.FONT_HERSHEY_SIMPLEX, 0.5, RED, 2)

    def make_box(self, contour, frame: VideoFrame = None):
        """fm.py:787-792: boundingRect -> ((x, y), (x + w, y + h))"""
        return VideoMotion.make_area_from_rect(contour.bbox)

    @staticmethod
    def make_area_from_box(object_tuple):
        (x1, y1, x2, y2) = object_tuple
        return ((x1, y1), (x2, y2))

    @staticmethod
    def make_area_from_rect(object_tuple):
        (x, y, w, h) = object_tuple
        return ((x, y), (x + w, y + h))

    def draw_box(self, area, frame: VideoFrame = None) -> None:
        frame = self.current_frame if frame is None else frame
        if videoio.cv2 is not None:
            videoio.cv2.rectangle(frame.frame, *self.scale_area(area, 1 / self.scale), GREEN, 2)

    @staticmethod
    def key_pressed(key: str) -> bool:
        """fm.py:816-821 (waitKey only exists with OpenCV)."""
        cv2 = videoio.cv2
        return cv2 is not None and (cv2.waitKey(1) & 0xFF) == ord(key)

    def show_frames(self) -> None:
        cv2 = videoio.cv2
        if cv2 is None:
            return
        cf = self.current_frame
        for name in ("thresh", "gray", "blur", "raw"):
            img = getattr(cf, name, None)
            if img is not None:
                cv2.imshow(name, img)

    def cleanup(self) -> None:
        """fm.py:824-849, plus releasing the device context."""
        if self._pipe is not None:  # stop the decoder thread, drain batches in flight
            self._pipe.close()
            self._pipe = None
        if self.cap is not None:
            self.cap.release()
        if self.outfile is not None:
            self.outfile.release()
        if self.cleanup_flag and self.current_frame is not None:
            self.current_frame.in_cache = False
            self.current_frame.cleanup()
            for frame in self.frame_cache:
                if frame is not None:
                    frame.in_cache = False
                    frame.cleanup()
            self.frame_cache.clear()
        if self._own_engine and self._engine is not None:
            self._engine.close()
            self._engine = None
        if self._jpeg_dec is not None:
            self._jpeg_dec.close()
            self._jpeg_dec = None

    # -- main loop (fm.py:852-904) ---------------------------------------------
    def step(self) -> None:
        """Everything the loop does with one frame after the hot path (fm.py:870-892)."""
        try:
            self.find_movement()
        except Exception as e:  # noqa: BLE001 (fm.py:873-876)
            self.log.error("find_movement: {}".format(e))
        self.decide_output()
        if self.show:
            self.show_frames()
        self.current_frame.cleanup()

    def find_motion(self) -> tuple:
        while self.is_open():
            if not self.read():
                break
            self.blur_frame()
            self.mask_off_areas()
            self.find_diff()
            self.step()
            if self.show and VideoMotion.key_pressed("q"):
                self.wrote_frames = None
                self.err_msg = "Closing video at user request"
                break
        self.cleanup()
        return self.wrote_frames, self.err_msg, tuple(self.seen_objects)


def run_vid(filename, **kwargs) -> tuple:
    """fm.py:1021-1037 (the unbound seen_objects of the reference's error path is None here)."""
    seen_objects = None
    try:
        vid = VideoMotion(filename=filename, **kwargs)
        if vid.loaded:
            wrote_frames, err_msg, seen_objects = vid.find_motion()
        else:
            wrote_frames = None
            err_msg = "Video did not load successfully"
            vid.cleanup()
    except Exception as e:  # noqa: BLE001
        err_msg = "Error processing video {}: {}".format(filename, e)
        wrote_frames = None
    return (wrote_frames, filename, err_msg, seen_objects)


class StreamGroup:
    """S same-sized videos on ONE device, batched into one launch per frame step.

    The reference runs one video per worker process (run_pool, fm.py:1054-1122).
    On MI355X the streams of a device share one fm_ctx with one background
    model per stream, so one fused launch covers T frames of all S streams.
    Each stream keeps its own VideoMotion state machine and writer; results
    are gathered per stream as run_vid returns them.
    """

    def __init__(self, filenames: list, batch: int = 8, device: int = 0, captures: list = None, engine=None,
                 **kwargs):
        self.filenames = list(filenames)
        S = len(self.filenames)
        if S == 0:
            raise ValueError("More than 0 files needed")
        caps = [videoio.open_capture(c if c is not None else f, device, kwargs.get("gpu_decode"))
                for f, c in zip(self.filenames, captures or [None] * S)]
        w = {int(c.get(videoio.CAP_PROP_FRAME_WIDTH)) for c in caps}
        h = {int(c.get(videoio.CAP_PROP_FRAME_HEIGHT)) for c in caps}
        if len(w) != 1 or len(h) != 1:
            raise VideoError("StreamGroup streams must share one frame size")
        W, H = w.pop(), h.pop()
        box = kwargs.get("box_size", 100)
        blur_scale = kwargs.get("blur_scale", 20)
        show = kwargs.get("show", False)
        dbg = kwargs.get("log_level", logging.INFO) == logging.DEBUG
        self.batch = max(1, int(batch))
        make = engine if engine is not None else MotionEngine  # engine: a factory with MotionEngine's signature
        mbs = kwargs.get("min_box_scale", VideoMotion.DEFAULT_MIN_BOX_SCALE)
        area_filter = int(W * H / 2 * (box / W)) < int(math.pow(box / mbs, 2))  # as _load_video decides
        self.engine = make(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=make_gaussian_size(box, blur_scale),
                           threshold=kwargs.get("threshold", 7), avg=kwargs.get("avg", 0.1), max_batch=self.batch,
                           keep_planes=show or dbg, device=device, contour_area=area_filter)
        self.videos = [VideoMotion(filename=f, capture=c, engine=self.engine, stream=s, batch=self.batch, **kwargs)
                       for s, (f, c) in enumerate(zip(self.filenames, caps))]

    def find_motion(self) -> list:
        """Decode-ahead into page-locked batches (BatchFeeder), up to fm_max_inflight batches in
        flight, each waited batch consumed frame by frame by every stream's state machine."""
        caps = [v.cap if v.loaded else videoio.ArrayCapture([]) for v in self.videos]
        for b in BatchFeeder(self.engine, caps, self.batch):
            for s, v in enumerate(self.videos):
                if not b.frames[s]:
                    continue
                vfs = v.make_frames(b, s)
                v.bind_results(vfs, self.engine, s)
                for vf in vfs:
                    v.current_frame = vf
                    v.step()
        out = []
        for f, v in zip(self.filenames, self.videos):
            v.cleanup()
            out.append((v.wrote_frames if v.loaded else None, f, v.err_msg if v.loaded else
                        "Video did not load successfully", tuple(v.seen_objects) if v.loaded else None))
        self.engine.close()
        return out
