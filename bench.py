#!/usr/bin/env python3
"""bench.py — frames/s of the MI355X motion hot path on synthetic 1080p.

Workload (BASELINE.json configs[1]): one 1080p stream per GPU through the
fused pixel kernel in "mode F" (-B 1920 -b 384: box = frame width, 5x5
Gaussian), the reference's CLI defaults otherwise (-t 12 -a 0.1).  A "step"
is one fm_submit + fm_wait of --batch consecutive frames per stream, read
from a device-resident ring of synthetic frames (the background model keeps
evolving across the ring).  Multi-GPU: one process per GPU (torchrun), each
on its own streams; no collective on the data path (the reference's only
parallelism is one video per worker, find_motion.py:1071-1075).  RCCL is used
only for the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line on rank 0 (driver contract), with a "roofline" object
for the dominant kernel (HIP-event timing inside the library, on the stream
the kernels run on) and a "cpu_baseline" object (the C restatement in
oracle/, OpenMP, one thread per stream, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# eight hardware queues per process (find_motion_amd.use_hw_queues, the CLI's setting), before torch makes the
# first HIP call, whatever the environment holds (the GPU box exports HIP's default, 4): with 4 the input
# stream shares an in-order queue with a contour stream (mode D 498 -> 591 k frames/s at 8, MJPEG-fed 74 ->
# 84 k, the headline unchanged; profiles/r04s_hwq_ab.txt).  FM_BENCH_HW_QUEUES picks another count; the value
# in effect is recorded in the JSON line
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("FM_BENCH_HW_QUEUES", "8")

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
PCIE_GBS = 63.0  # PCIe Gen5 x16, one direction
CONFIG5_MASKS = [((0, 0), (639, 359)), ((3839, 2159), (3200, 2159), (3839, 1600))]
METRIC = "frames/sec on 1080p synthetic video at 1/2/4/8 MI355X; achieved HBM GB/s %peak"
# kernels the engine times by in-kernel stamps on every launch (fm_capi.cpp KernelTimer::stamp)
STAMPED = ("pix", "pix_init", "resize_area", "resize_area_fast", "small_blur", "small_scan")


def algorithmic_bytes(kernel: str, cfg: dict) -> float | None:
    """Algorithmic HBM bytes of ONE launch of `kernel` (DESIGN.md 'Kernels')."""
    S, T = cfg["streams_per_gpu"], cfg["frames_per_step"]
    H, W, h, w = cfg["H"], cfg["W"], cfg["h"], cfg["w"]
    if kernel in ("fused", "pix"):
        # one launch = T frames of every stream: per frame BGR read 3 B + dilated mask write 1 B;
        # per batch the f64 background read + write 16 B (held in registers across the batch)
        return S * T * h * w * (3 + 1) + S * h * w * 16
    if kernel == "pixel":
        # one launch = one frame of every stream: BGR read 3 B + mask write 1 B + f64 background r/w 16 B
        return S * h * w * (3 + 1 + 16)
    if kernel in ("resize_area", "resize_area_fast"):
        return S * T * (H * W * 3 + h * w * 3)
    return None


def moved_bytes(kernel: str, cfg: dict) -> float | None:
    """Bytes ONE launch of the pixel kernel must move as it is built (not §8(d)'s accounting): the BGR
    read (3 B/px-frame), the threshold bits it writes instead of a u8 mask (1/8 B/px-frame), 32 B of tile
    flags per 64x64 tile-frame, and the f64 background read + written once per launch (16 B/px)."""
    if kernel not in ("fused", "pix"):
        return None
    S, T, h, w = cfg["streams_per_gpu"], cfg["frames_per_step"], cfg["h"], cfg["w"]
    tiles = ((h + 63) // 64) * ((w + 63) // 64)
    return S * T * (h * w * (3 + 1 / 8) + tiles * 32) + S * h * w * 16


def path_bytes_per_frame(cfg: dict) -> int:
    """SURVEY.md §8(d) algorithmic bytes of the whole path per frame: mode D 3·W·H + 17·h·w (BGR frame read,
    resized image, mask and the reference's per-frame f64 background traffic); mode F W·H·(4 + 16/T)."""
    H, W, h, w, T = cfg["H"], cfg["W"], cfg["h"], cfg["w"], cfg["frames_per_step"]
    if (h, w) != (H, W):
        return 3 * W * H + 17 * h * w
    return int(h * w * (4 + 16 / T))


def pmc_traffic(kernel: str, cfg: dict) -> tuple[int | None, str | None, dict | None]:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (profiles/traffic.json,
    written by tools/traffic.py from FETCH_SIZE / WRITE_SIZE passes of this same workload), and the SQ
    counter ratios of those passes (what bounds the kernel), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None, None
    entries = t.get("entries", [t])  # one entry per profiled workload (tools/traffic.py)
    # the most recent profile of this workload (entries are appended round by round)
    e = next((e for e in reversed(entries) if e.get("workload") == cfg["workload"] and kernel in e.get("kernels", {})),
             None)
    if e is None:
        return None, None, None
    k = e["kernels"][kernel]
    return int(k["traffic_bytes"]), e.get("source"), k.get("sq")


def config_name(S: int, W: int, H: int, mode: str, k: int, haar: bool = False, world: int = 1) -> str:
    """Which BASELINE.json config the run's shape is (configs[1] is the headline; the others are the parity
    configurations run at their quoted perf shapes), so a line is never filed under the wrong one.  S is
    streams per GPU, world the number of ranks (one GPU each): 8 streams per GPU on 8 GPUs is configs[3]
    (64 x 1080p sharded 8 per GPU, find_motion.py:1054-1122)."""
    md = "" if mode == "F" else " (mode D)"
    if (W, H) == (1920, 1080):
        if S == 1:
            return ("configs[1]" if world == 1 else f"configs[1] x {world} GPUs") + md
        if S == 8:
            if world == 1:
                return "configs[2]" + md
            if world == 8:
                return "configs[3]" + md
            return f"configs[3] family: 8 streams per GPU x {world} GPUs" + md
        return f"{S} x 1080p streams per GPU x {world} GPU(s) (configs[2]/[3] family)" + md
    if (W, H) == (3840, 2160) and k == 21:
        return ("configs[4]" if haar else "configs[4] geometry (no Haar stage)") + ("" if world == 1 else f" x {world} GPUs")
    return "custom shape"


def workload_name(S: int, W: int, H: int, mode: str, box: int, blur_scale: int, k: int, T: int, R: int,
                  ring_period: int, haar: bool = False, world: int = 1) -> str:
    """The line's config.workload (also the key of the workload's PMC entry in profiles/traffic.json)."""
    return (f"{config_name(S, W, H, mode, k, haar, world)}: {S}x{W}x{H} stream(s) per GPU, mode {mode} "
            f"(-B {box} -b {blur_scale}, k {k}), {T} frames/stream/step from a {R}-frame device-resident ring"
            + (f" cycling {ring_period} synthetic frames" if ring_period < R else ""))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg: dict, frames_host: np.ndarray, n_frames: int) -> dict:
    """The oracle (C restatement, not OpenCV) on a bounded sample of the same workload, per SURVEY.md §8d:
    P worker threads, one stream each (run_pool's one video per worker, find_motion.py:1071-1075), frames
    pre-generated in RAM, 10 warm-up frames, the median of 5 timed runs; plus one thread on one stream."""
    import oracle

    aff = len(os.sched_getaffinity(0))
    # P = len(sched_getaffinity(0)), capped by OMP_NUM_THREADS: the GPU box sets it to the CPU share of
    # one GPU (16) and allows no larger worker pools
    cap = int(os.environ.get("OMP_NUM_THREADS") or aff)
    threads = max(1, min(aff, cap))
    ocfg = oracle.OracleConfig(H=cfg["H"], W=cfg["W"], box=cfg["box"], ksize=cfg["ksize"],
                               thresh=cfg["threshold"], alpha=cfg["avg"])
    seq = np.ascontiguousarray(frames_host[:n_frames])
    warm = np.ascontiguousarray(frames_host[:10])
    oracle.run_streams(ocfg, warm, threads, n_streams=threads)  # 10 warm-up frames per worker
    runs = []
    used = threads
    for _ in range(5):
        t0 = time.perf_counter()
        _, used = oracle.run_streams(ocfg, seq, threads, n_streams=threads)
        runs.append(time.perf_counter() - t0)
    dt = float(np.median(runs))
    t0 = time.perf_counter()
    oracle.run_streams(ocfg, seq, 1, n_streams=1)
    single = n_frames / (time.perf_counter() - t0)
    return {"value": round(threads * n_frames / dt, 2), "unit": "frames/s", "cores": used, "kind": "port",
            "single_stream_1_core": round(single, 2),
            # SURVEY §8d asks for P = the affinity; on the GPU box the affinity lists the whole machine's CPUs while
            # one GPU's share of them is OMP_NUM_THREADS (16), the largest worker pool the box allows per GPU
            "cores_rule": (f"P = min(affinity {aff}, OMP_NUM_THREADS {cap}): the host CPUs one GPU's job may use"
                           if cap < aff else f"P = affinity ({aff})"),
            "sample": f"{threads} workers x 1 stream x {n_frames} frames {cfg['W']}x{cfg['H']} box {cfg['box']} "
                      f"k {cfg['ksize']}, median of 5 runs after 10 warm-up frames ({aff} CPUs in affinity, "
                      f"OMP_NUM_THREADS cap {cap}); CPU restatement of the OpenCV chain, not OpenCV "
                      f"(oracle/fm_oracle.c, gcc -O3 -march=x86-64-v3; cv2 is not installed); CPU: {cpu_model()}"}


def mjpeg_fed(eng, host: np.ndarray, T: int, S: int, quality: int = 75) -> dict | None:
    """Frames/s through BatchFeeder's JPEG mode (host parse + compressed H2D + GPU decode + hot path),
    the decoder's kernels alone (HIP events), and Pillow's libjpeg-turbo decode on one host core."""
    try:
        from PIL import Image
    except ImportError:
        return None
    import io

    import torch

    from find_motion_amd import MJpegDecoder, videoio
    from find_motion_amd.feeder import BatchFeeder
    R, H, W = host.shape[0], host.shape[2], host.shape[3]
    enc = []
    for t in range(min(R, 64)):  # host: the ring's distinct frames
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(host[t, 0][..., ::-1])).save(b, "JPEG", quality=quality)
        enc.append(b.getvalue())
    dec = MJpegDecoder(W, H, max_frames=T * S, device=eng.device)
    dst = torch.empty((T * S, H, W, 3), dtype=torch.uint8, device="cuda")
    jp = [enc[i % len(enc)] for i in range(T * S)]
    dec.decode_device(jp, dst.data_ptr())
    kms = []
    for _ in range(3):
        dec.decode_device(jp, dst.data_ptr())
        kms.append(dec.last_ms())
    dec.close()
    del dst
    n = max(32 * T, 2048)  # long enough that the feeder's fill and drain (about two batches) stay small
    for _ in BatchFeeder(eng, [videoio.JpegListCapture(enc[:2]) for _ in range(S)], T):  # warm-up
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in BatchFeeder(eng, [videoio.JpegListCapture([enc[i % len(enc)] for i in range(n)]) for _ in range(S)], T):
        pass
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    for j in enc[:16]:
        np.asarray(Image.open(io.BytesIO(j)))
    cpu_fps = 16 / (time.perf_counter() - t1)
    return {"frames_per_s": round(n * S / dt, 1), "frames": n * S, "jpeg_quality": quality,
            "bytes_per_frame": int(np.mean([len(j) for j in enc])),
            "decoder_kernels_ms_per_batch": round(float(np.median(kms)), 3),
            "decoder_kernels_frames_per_s": round(T * S / (float(np.median(kms)) / 1e3), 1),
            "libjpeg_turbo_1core_frames_per_s": round(cpu_fps, 1),
            "mode": "BatchFeeder JPEG mode: JPEG bytes -> host parse -> H2D -> GPU Huffman/IDCT/colour -> hot path"}


class RoiSelector:
    """Which frames of one stream reach the cascade, by the reference's rule: find_movement counts the
    contours (fm.py:665-700), decide_output writes the frame when movement_counter >= min_movement_frames
    or movement_decay > 0 and then calls find_objects (fm.py:549-575), whose counter runs the cascades on
    every 15th call (skip = 15, fm.py:703-713).  VideoMotion defaults: fps 30, cache_time 2.0 (decay 60
    frames), min_time 0.5 (15 contour-frames)."""

    def __init__(self, fps: int = 30, cache_time: float = 2.0, min_time: float = 0.5, skip: int = 15):
        self.cache_frames, self.min_frames, self.skip = int(cache_time * fps), int(min_time * fps), skip
        self.counter = self.decay = self.obj = 0

    def step(self, count: int) -> bool:
        movement = count > 0
        self.decay -= 1 if self.decay > 0 else 0
        self.counter = self.counter + int(count) if movement else 0
        if self.counter >= self.min_frames or self.decay > 0:
            if movement:
                self.decay = self.cache_frames
            self.obj += 1
            if self.obj == self.skip:
                self.obj = 0
                return True
        return False


def spawn_ranks(n: int) -> int:
    """bench.py --gpus N without a launcher: start N ranks of this script (one per GPU, RANK = LOCAL_RANK =
    device ordinal, rendezvous on 127.0.0.1) before any GPU call in this process, and return the worst
    exit status.  Rank 0's stdout carries the JSON line."""
    import signal
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, abs(p.wait()))
            if rc:
                break
    finally:
        for p in procs:  # a failed rank: stop the others (exact child PIDs)
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
            rc = max(rc, abs(p.returncode or 0))
    return rc


def synthetic_ring(W: int, H: int, S: int, R: int, P: int, streams: list, local: int, paint=None):
    """Host frames [P][S][H][W][3] (the ring's distinct synthetic frames, generated on a thread pool: each
    frame is independent of the others; `paint(frame)` then draws into each) and the device ring
    [R][S][H][W][3], slot t holding frame t % P."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from find_motion_amd.synthetic import SyntheticVideo
    vids = [SyntheticVideo(W, H, stream=g) for g in streams]
    host = np.empty((P, S, H, W, 3), np.uint8)

    def gen(i: int) -> None:
        host[i // S, i % S] = vids[i % S].frame(i // S)
        if paint is not None:
            paint(host[i // S, i % S])

    with ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1))) as ex:
        list(ex.map(gen, range(P * S)))
    uniq = torch.from_numpy(host).to(f"cuda:{local}")
    ring = torch.empty((R, S, H, W, 3), dtype=torch.uint8, device=f"cuda:{local}")
    for t in range(R):
        ring[t].copy_(uniq[t % P])
    del uniq
    return host, ring


def roofline_of(ktimes: dict, cfg: dict, ms_per_step: float, kstd: dict | None = None,
                kbusy: dict | None = None) -> dict | None:
    """Roofline of the dominant kernel from the engine's per-kernel times (every pixel / resize launch
    timed by in-kernel stamps: first workgroup's start to last wave's end).  In mode D the dominant
    kernel is the INTER_AREA resize, the one kernel there that streams whole frames (the pixel kernel's
    100 x 56 work image is two tiles: latency, not bandwidth)."""
    dom = max(ktimes.items(), key=lambda kv: kv[1][0])[0] if ktimes else None
    for rk in ("resize_area", "resize_area_fast"):
        if rk in ktimes and ktimes[rk][1] > 0:
            dom = rk
    if dom is None:
        return None
    ms, n = ktimes[dom]
    avg_s = ms / 1e3 / max(n, 1)
    nbytes = algorithmic_bytes(dom, cfg)
    if nbytes is None or avg_s <= 0:
        return None
    # launches of one kernel may overlap (mode D's resizes of consecutive batches run on two input streams): the
    # kernel's throughput is then its bytes over the time at least one launch ran (the union of the windows)
    busy = (kbusy or {}).get(dom)
    overlap = bool(busy and busy < ms * (1 - 1e-3))
    eff_s = busy / 1e3 / max(n, 1) if overlap else avg_s
    ach = nbytes / eff_s / 1e9
    traffic, tsrc, sq = pmc_traffic(dom, cfg)
    # "bound" is the roofline the kernel is priced against (byte/integer stencils + an f64
    # recurrence: no contraction, no MFMA).  What actually limits it is read from the SQ
    # counters of the committed profile: "limiter" below.
    roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": int(nbytes), "avg_launch_us": round(avg_s * 1e6, 3), "launches_timed": int(n),
            "timing": ("every launch of the timed steps, in-kernel s_memrealtime stamps (first workgroup start, "
                       "last wave end; 100 MHz)") if dom in STAMPED else "HIP events around one launch in four",
            # the launches of one stream are serialised, so each is at most a step: a larger figure is a
            # timing fault, never a kernel fraction
            "launch_le_step": bool(eff_s * 1e3 <= ms_per_step * (1 + 1e-6))}
    if overlap:
        roof["launches_overlap"] = True
        roof["busy_us_per_launch"] = round(eff_s * 1e6, 3)
        roof["frac_per_launch_duration"] = round(nbytes / avg_s / 1e9 / HBM_PEAK_GBS, 4)
        roof["timing"] += ("; launches overlap, so achieved = bytes / (the union of the launch windows / launches), "
                           "busy_us_per_launch")
    if kstd and dom in kstd:
        roof["launch_std_us"] = round(1e3 * kstd[dom], 2)
    if not roof["launch_le_step"]:
        print(f"[bench] WARNING: {dom} averages {eff_s * 1e6:.1f} us per launch, more than the "
              f"{ms_per_step * 1e3:.1f} us step", file=sys.stderr)
    mv = moved_bytes(dom, cfg)
    if mv is not None:  # the same launches priced on the bytes the kernel must move as built
        roof["moved_bytes_per_launch"] = int(mv)
        roof["frac_moved"] = round(mv / eff_s / 1e9 / HBM_PEAK_GBS, 4)
    if traffic is not None:
        roof["traffic_source"] = f"{tsrc}: 2 x FETCH_SIZE + WRITE_SIZE per launch (gfx950 16-B read correction)"
    if sq:
        roof["limiter"] = (f"issue and latency, not HBM bandwidth: of SQ_WAVE_CYCLES, {sq['wait_inst_any_frac']:.0%} "
                           f"issue stalls (SQ_WAIT_INST_ANY), {sq['wait_any_frac']:.0%} parked on s_waitcnt / the "
                           f"frame barrier (SQ_WAIT_ANY), {sq['active_inst_any_frac']:.0%} issuing; "
                           f"{sq['valu_insts'] / 1e6:.1f}M VALU, {sq['salu_insts'] / 1e6:.1f}M SALU, "
                           f"{sq['lds_insts'] / 1e6:.1f}M LDS wave-instructions per launch ({tsrc})")
    return roof


def face_painter(W: int, H: int):
    """configs[4]'s Haar stage timed on frames that contain faces: the cartoon frontal face of the Haar
    tests (tests/haar_cases.py draw_faces, which the reference's frontalface_default cascade detects) drawn
    into every synthetic frame, at the place and size it has in the 3840x2160 fixture frame."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from haar_cases import draw_faces
    cx, cy, r = int(1024 * W / 3840), int(1024 * H / 2160), int(576 * W / 3840)
    x0, x1, y0, y1 = max(0, cx - r), min(W, cx + r), max(0, cy - int(1.2 * r)), min(H, cy + int(1.2 * r))
    patch = draw_faces(np.empty((y1 - y0, x1 - x0, 3), np.uint8), [(cx - x0, cy - y0, r)], seed=1)

    def paint(frame: np.ndarray) -> None:
        frame[y0:y1, x0:x1] = patch
    return paint


def run_leg(args, mode: str, S: int, T: int, steps: int, warmup: int, pl, local: int, active: bool, backend: str,
            haar: bool = False, masks: bool = False, ring_frames: int | None = None, shape: tuple | None = None,
            blur_scale: int | None = None, ring_period: int | None = None) -> dict:
    """One workload: S streams per GPU of synthetic frames in a device-resident ring, `warmup` untimed then
    `steps` timed steps (one step = one batch of T frames per stream submitted and one completed), the
    barrier + synchronize on both sides, max over ranks.  Returns the line's figures and the live engine."""
    import torch

    from find_motion_amd import MotionEngine, dist, make_gaussian, work_height
    world = pl.world
    W, H = (args.width, args.height) if shape is None else shape
    box, bscale = (W, W // 5) if mode == "F" else (100, 20)
    if mode == "F" and W == 1920:
        bscale = 384
    if blur_scale is None and args.blur_scale is not None and shape is None:
        blur_scale = args.blur_scale
    blur_scale = bscale if blur_scale is None else blur_scale
    k = make_gaussian(box, blur_scale)
    ring_frames = args.ring if ring_frames is None else ring_frames
    ring_period = args.ring_period if ring_period is None else ring_period
    R = max(ring_frames - ring_frames % T, T)
    cfg = {"workload": workload_name(S, W, H, mode, box, blur_scale, k, T, R, ring_period, haar, world),
           "streams_per_gpu": S, "frames_per_step": T, "W": W, "H": H, "box": box, "ksize": k,
           "h": work_height(H, W, box), "w": box, "threshold": 12, "avg": 0.1, "parallelism": f"streams x {world} GPUs"}

    # synthetic ring [R][S][H][W][3] on the device, distinct streams per rank (stream s -> rank s // S):
    # ring slot t holds synthetic frame t % P; only the P distinct frames exist on the host (at 8 streams a
    # host copy of the whole ring would be 12.7 GB per rank)
    P = max(1, min(ring_period, R))
    paint = face_painter(W, H) if haar else None
    host, ring = synthetic_ring(W, H, S, R, P, dist.rank_streams(pl, S), local, paint)
    frame_bytes = S * H * W * 3

    eng = MotionEngine(n_streams=S, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1,
                       max_batch=T, max_contours=1 << 14,
                       profile=False if args.no_ktimes else True if args.all_ktimes else "pix", device=local)
    footprint = dict(eng.footprint(), ring_bytes=R * frame_bytes)
    if masks or haar:  # mask_off_areas (fm.py:611-636): rasterised once, applied in the pixel kernel
        from find_motion_amd import rasterize_masks
        keep = rasterize_masks(cfg["h"], cfg["w"], box / W, CONFIG5_MASKS)
        for s in range(S):
            eng.set_mask(s, keep)
        cfg["masks"] = [list(map(list, m)) for m in CONFIG5_MASKS]
    base = ring.data_ptr()
    n_batches = R // T

    # Pipelined like a live decoder feeding the engine: up to max_inflight batches are
    # submitted before the oldest one's results are collected, so the contour passes
    # of consecutive batches overlap each other and the next pixel kernels.  A step =
    # one batch submitted + one batch completed; all timed batches are submitted and
    # completed inside the timed region.
    depth = eng.max_inflight

    hostt = {"submit": 0.0, "wait": 0.0}  # host seconds in fm_submit / fm_wait (is the loop host-bound?)

    def submit(i: int) -> None:
        t = time.perf_counter()
        eng.submit_device(base + (i % n_batches) * T * frame_bytes, T)
        hostt["submit"] += time.perf_counter() - t

    ccl = {"heavy_tiles": 0, "shared_nodes_max": 0, "fallback_frames": 0, "batches": 0}

    # configs[4]'s object-ROI stage: the frames find_objects hands to the cascade, gathered from the ring
    # (still in HBM) after each waited batch and detected in one call (INTER_AREA to 300 px + detectMultiScale)
    det, sel = None, [RoiSelector() for _ in range(S)]
    hs = {"calls": 0, "roi_frames": 0, "detections": 0, "wall_s": 0.0, "device_ms": 0.0, "pending": 0}
    if haar:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from golden_cases import load_frontalface  # the reference's cascade, as committed fixture arrays

        from find_motion_amd import CascadeClassifier
        det = CascadeClassifier(load_frontalface()[0], device=local)

    def collect() -> None:
        if hs["pending"]:
            found = det.collect(hs["pending"])
            hs["device_ms"] += det.last_ms()
            hs["detections"] += sum(len(f) for f in found)
            hs["pending"] = 0

    def objects(i: int, last: bool) -> None:
        # find_objects' detections feed only the seen-objects set (never the written-frame decision,
        # fm.py:549-575, 703-731), so batch i's are queued on the detector's stream and collected after batch
        # i + 1 is waited: the sweep overlaps the next batches' kernels and the host loop
        cnt = eng.counts()
        base_t = (i % n_batches) * T
        pick = [(t, s) for t in range(T) for s in range(S) if sel[s].step(int(cnt[t, s]))]
        t0 = time.perf_counter()
        collect()
        if pick:
            # the ROI frames where they lie in the ring (written before the timed region): no gather copy
            det.detect_frame_list_async([ring[base_t + t, s].data_ptr() for t, s in pick], H, W, 300, 1.1, 5)
            hs["pending"] = len(pick)
            hs["calls"] += 1
            hs["roi_frames"] += len(pick)
        if last:
            collect()
        hs["wall_s"] += time.perf_counter() - t0

    def run(first: int, n: int) -> None:
        for i in range(min(depth, n)):
            submit(first + i)
        for i in range(n):
            t = time.perf_counter()
            eng.wait()  # completes batch i and frees its slot
            hostt["wait"] += time.perf_counter() - t
            if det is not None:
                objects(first + i, i == n - 1)
            st = eng.ccl_stats()  # two mapped-memory words: no device sync
            ccl["heavy_tiles"] += st["heavy_tiles"]
            ccl["shared_nodes_max"] = max(ccl["shared_nodes_max"], st["shared_nodes"])
            ccl["fallback_frames"] += eng.fallbacks()
            ccl["batches"] += 1
            if i + depth < n:
                submit(first + i + depth)

    run(0, warmup)
    eng.reset_kernel_times()
    ccl.update(heavy_tiles=0, shared_nodes_max=0, fallback_frames=0, batches=0)
    hostt.update(submit=0.0, wait=0.0)

    dist.barrier(active)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hs.update(calls=0, roi_frames=0, detections=0, wall_s=0.0, device_ms=0.0, pending=0)
    run(warmup, steps)
    torch.cuda.synchronize()
    dist.barrier(active)
    wall = time.perf_counter() - t0
    elapsed = dist.max_over_ranks(wall, active, device=f"cuda:{local}" if backend == "nccl" else "cpu")
    if det is not None:
        det.close()

    kst = eng.kernel_time_stats()  # one fold of the launch stamps: sums, spreads and busy time over the same launches
    unstamped = kst.pop("_unstamped")
    ktimes = {k: (v["ms"], v["launches"]) for k, v in kst.items()}
    # stamped launches: the spread of the launch time over the timed steps
    kstd = {k: max(v["ms_sq"] / v["stamped"] - (v["stamped_ms"] / v["stamped"]) ** 2, 0.0) ** 0.5
            for k, v in kst.items() if v["stamped"] > 0 and v["ms_sq"] > 0}
    kbusy = {k: v["busy_ms"] for k, v in kst.items()}  # the union of each kernel's launch windows
    total_frames = world * S * T * steps
    ms_per_step = 1e3 * elapsed / steps
    kernels = {name: {"avg_us": round(1e3 * ms / max(n, 1), 3), "launches": int(n), "total_ms": round(ms, 3),
                      **({"std_us": round(1e3 * kstd[name], 2)} if name in kstd else {}),
                      **({"busy_ms": round(kbusy[name], 3)} if kbusy.get(name) and kbusy[name] < ms * (1 - 1e-3) else {})}
               for name, (ms, n) in ktimes.items()}
    del ring
    return {"cfg": cfg, "eng": eng, "host": host, "P": P, "wall": wall, "elapsed": elapsed, "unstamped": int(unstamped),
            "value": total_frames / elapsed, "ms_per_step": ms_per_step,
            "roofline": roofline_of(ktimes, cfg, ms_per_step, kstd, kbusy), "kernels": kernels, "haar": hs, "det": det,
            "footprint": footprint, "ccl": ccl,
            "host_us_per_step": {k: round(1e6 * v / steps, 1) for k, v in hostt.items()}}


def haar_summary(hs: dict, wall: float) -> dict:
    return {"cascade": "haarcascade_frontalface_default (reference XML as tests/golden fixture arrays)",
            "rule": "every 15th written frame per stream (find_objects skip=15, fm.py:549-575, 703-731)",
            "calls": hs["calls"], "roi_frames": hs["roi_frames"], "detections": hs["detections"],
            "wall_ms": round(1e3 * hs["wall_s"], 3), "device_ms": round(hs["device_ms"], 3),
            "share_of_step_time": round(hs["wall_s"] / wall, 4),
            "overlap": "each batch's detection queued on the detector's stream, collected after the next "
                       "batch is waited (host time in the loop: wall_ms)",
            "frames": "synthetic frames with a cartoon frontal face drawn in (tests/haar_cases.py draw_faces)"}


def side_leg(args, mode: str, S: int, T: int, pl, local: int, active: bool, backend: str, steps: int = 60,
             warmup: int | None = None, **kw) -> dict:
    """A compact figure of another configuration for the same JSON line (mode D, the reference CLI's
    default -B 100; configs[2], 8 streams per GPU; configs[4], 4 x 4K with k 21, masks and the Haar stage):
    value, step time, its own roofline."""
    # mode D / configs[2]: 60 timed steps whatever the headline's K: a step's batch is submitted and completed
    # inside the timed region, so the pipeline's fill and drain (the last batch's pixel stage and contour pass
    # after its resize, ~0.3 ms in mode D) is a fixed cost that 20 steps of ~0.32 ms amortise ~3x less than 60 do
    warmup = max(2, min(args.warmup, 5)) if warmup is None else warmup
    leg = run_leg(args, mode, S, T, steps, warmup, pl, local, active, backend, **kw)
    leg["eng"].close()
    out = {"workload": leg["cfg"]["workload"], "value": round(leg["value"], 2), "unit": "frames/s",
           "steps": steps, "warmup": warmup, "ms_per_step": round(leg["ms_per_step"], 4), "roofline": leg["roofline"],
           "kernels": leg["kernels"], "host_us_per_step": leg["host_us_per_step"], "path_hbm_frac": round(leg["value"] / pl.world * path_bytes_per_frame(leg["cfg"])
                                                            / 1e9 / HBM_PEAK_GBS, 4)}
    if leg["det"] is not None:
        out["haar_stage"] = haar_summary(leg["haar"], leg["wall"])
    if "masks" in leg["cfg"]:
        out["masks"] = leg["cfg"]["masks"]
    del leg
    import torch
    torch.cuda.empty_cache()
    return out


# mode D (-B 100 -b 20, the reference CLI's default, find_motion.py:1474); configs[2] (8 x 1080p streams on one
# GPU, 128 frames per stream per step); configs[4]: 4 x 3840x2160 streams, -B 3840 -b 183 (k 21), the polygon
# masks, 64 frames per stream per step from a 64-frame ring cycling 16 synthetic frames, with the frontalface
# cascade on every 15th written frame (faces drawn in), and the same geometry without the Haar stage
_C4 = dict(shape=(3840, 2160), blur_scale=183, ring_frames=64, ring_period=16, steps=20, warmup=10)
SIDE_LEGS = {"mode_d": ("D", 1, None, {}), "configs2": ("F", 8, 128, {}),
             "configs4": ("F", 4, 64, dict(_C4, haar=True)), "configs4_no_haar": ("F", 4, 64, dict(_C4, masks=True))}


def side_child(name: str, args) -> dict:
    """Run side leg `name` in a child process (bench.py --side-leg NAME) and return its JSON object."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--side-leg", name, "--warmup", str(args.warmup),
           "--batch", str(args.batch)] + (["--all-ktimes"] if args.all_ktimes else []) + (["--no-ktimes"] if args.no_ktimes else [])
    env = {k: v for k, v in os.environ.items() if k != "FM_BENCH_PG"}  # no group of its own beside the parent's
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"side leg {name} exited {r.returncode}"}
    return json.loads(lines[-1])


def rank_devices(local: int, pl, active: bool) -> list:
    """[{rank, device, pci_bus_id, name}] of every rank, gathered on rank 0 through the process group (so
    the line records how many ranks the group really held and which device each ran on)."""
    import torch

    from find_motion_amd import dist
    pr = torch.cuda.get_device_properties(local)
    bus = None
    if getattr(pr, "pci_bus_id", None) is not None:
        bus = f"{getattr(pr, 'pci_domain_id', 0):04x}:{pr.pci_bus_id:02x}:{getattr(pr, 'pci_device_id', 0):02x}"
    me = {"rank": pl.rank, "device": local, "pci_bus_id": bus, "name": pr.name,
          "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}
    return dist.gather_to_root(me, pl, active) or []


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["F", "D"], default="F",
                    help="F: -B 1920 -b 384 (full-resolution fused kernel); D: reference default -B 100 -b 20")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--blur-scale", type=int, default=None,
                    help="-b override (config 5: --width 3840 --height 2160 --blur-scale 183 -> k 21)")
    ap.add_argument("--streams", type=int, default=1, help="streams per GPU")
    # 256 frames per launch: r02 (60 steps) 64 326k, 128 357k, 160 368k, 192 376k, 224 364k, 256 375k frames/s;
    # round 3 with the labelling gate and 6 slots at the driver's 20 steps, 3 alternating rounds: 192 396.3k,
    # 256 412.3k, 320 415.0k -- each batch boundary costs a pixel-kernel tail and a dependent launch, and the
    # last batch's contour chain after the last pixel launch is a smaller share of 20 longer steps
    ap.add_argument("--batch", type=int, default=256, help="frames per stream per step (one pixel-kernel launch)")
    ap.add_argument("--ring", type=int, default=256, help="device-resident frames per stream")
    ap.add_argument("--ring-period", type=int, default=64,
                    help="synthetic frames in the ring's cycle: ring slot t holds frame t %% period")
    ap.add_argument("--cpu-frames", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-fed", action="store_true", help="also time PCIe-fed submits (stderr only)")
    ap.add_argument("--no-host-fed", action="store_true", help="skip the host-fed decode-ahead pipeline figure")
    ap.add_argument("--no-ktimes", action="store_true", help="no HIP event timing at all (no roofline)")
    ap.add_argument("--no-mjpeg", action="store_true", help="skip the MJPEG-fed (GPU decode) figure")
    ap.add_argument("--masks", action="store_true",
                    help="configs[4]'s polygon masks on every stream: a rectangle and a triangle in 3840x2160 frame "
                         "coordinates, given in the MASK_SCHEMA form (find_motion.py:86-100), the polygons of the "
                         "configs[4] parity tests; implied by --haar")
    ap.add_argument("--haar", action="store_true",
                    help="configs[4]: run the reference's frontalface_default cascade on every 15th written frame "
                         "of each stream (find_objects, fm.py:549-575, 703-731) inside the timed steps")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the mode D and configs[2] figures the default (1-GPU, configs[1]) line carries")
    ap.add_argument("--side-leg", choices=sorted(SIDE_LEGS), default=None,
                    help="(internal) run one side leg of the default line and print its JSON object")
    ap.add_argument("--all-ktimes", action="store_true",
                    help="HIP events around every kernel (perturbs the pipeline); default: pixel kernel only")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    from find_motion_amd import dist

    pl = dist.placement_from_env()
    if pl.world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={pl.world} (launch {args.gpus} ranks, or none)")
    rank, world, local = pl.rank, pl.world, pl.local_rank

    import torch

    # rehearsal only (one GPU box): FM_BENCH_DEVICE pins every rank to one device and
    # FM_BENCH_BACKEND=gloo replaces RCCL (which refuses two ranks on one device)
    if os.environ.get("FM_BENCH_DEVICE") is not None:
        local = int(os.environ["FM_BENCH_DEVICE"])
    backend = os.environ.get("FM_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    # FM_BENCH_PG=1: a process group even at one rank (the N>1 path's RCCL calls on a one-GPU box)
    active = dist.init(pl, backend, torch.device("cuda", local), force=os.environ.get("FM_BENCH_PG") == "1")

    if args.side_leg:  # one side leg of the default line, in a process of its own (side_child)
        mode, S_, T_, kw = SIDE_LEGS[args.side_leg]
        print(json.dumps(side_leg(args, mode, S_, T_ or args.batch, pl, local, active, backend, **kw)), flush=True)
        return
    leg = run_leg(args, args.mode, args.streams, args.batch, args.steps, args.warmup, pl, local, active, backend,
                  haar=args.haar, masks=args.masks)
    cfg, eng, host, P, wall, elapsed = leg["cfg"], leg["eng"], leg["host"], leg["P"], leg["wall"], leg["elapsed"]
    S, T, W, H = cfg["streams_per_gpu"], cfg["frames_per_step"], cfg["W"], cfg["H"]
    value, roof, kernels, haar, det = leg["value"], leg["roofline"], leg["kernels"], leg["haar"], leg["det"]
    footprint, ccl, depth = leg["footprint"], leg["ccl"], eng.max_inflight

    # measured device copy peak (for reference beside the spec)
    try:
        a = torch.empty(1 << 28, dtype=torch.uint8, device=f"cuda:{local}")
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        copy_gbs = 10 * 2 * a.numel() / (e0.elapsed_time(e1) / 1e3) / 1e9
        if roof is not None:
            roof["copy_peak_measured"] = round(copy_gbs, 1)
        del a, b
    except Exception:
        pass

    if args.host_fed:
        # PCIe-inclusive rates (never `value`): pageable numpy batches, then page-locked
        # batches from the engine (asynchronous DMA on the input stream, overlapped with
        # the previous batches' kernels), pipelined like the device-resident loop
        host_batch = np.ascontiguousarray(np.stack([host[t % P] for t in range(T)]))
        t0 = time.perf_counter()
        for _ in range(5):
            eng.submit(host_batch)
            eng.wait()
        hf = 5 * S * T / (time.perf_counter() - t0)
        pinned = [eng.host_buffer(T) for _ in range(min(depth, 2))]
        for k, pb in enumerate(pinned):
            for t in range(T):
                pb[t] = host[(k * T + t) % P]
        n_hf = 8

        def run_pinned() -> None:
            for i in range(min(depth, n_hf)):
                eng.submit(pinned[i % len(pinned)])
            for i in range(n_hf):
                eng.wait()
                if i + depth < n_hf:
                    eng.submit(pinned[(i + depth) % len(pinned)])

        run_pinned()  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_pinned()
        torch.cuda.synchronize()
        hp = n_hf * S * T / (time.perf_counter() - t0)
        print(f"[bench] host-fed frames/s per GPU: pageable H2D {hf:.1f}, pinned + hipMemcpyAsync overlap {hp:.1f} "
              f"({hp * S * H * W * 3 / 1e9 / S:.1f} GB/s of frames over PCIe)", file=sys.stderr)

    # Host-fed, end to end through the drop-in's decode-ahead pipeline (find_motion_amd.feeder.BatchFeeder):
    # frames pre-decoded in RAM (decode excluded, as in the CPU baseline) copied by a decoder thread into
    # page-locked batches, fm_max_inflight batches in flight, every batch waited and its contours read.
    # PCIe-inclusive, so it is reported beside `value`, never as it.
    host_fed = None
    # per-GPU figure, measured in the 1-GPU run only: every rank would page-lock (depth + 2) batches of
    # T frames (≈21 GB at 10 slots x 256 frames of 1080p), ≈170 GB of pinned host memory on an 8-GPU node
    if not args.no_host_fed and world == 1:
        from find_motion_amd import videoio
        from find_motion_amd.feeder import BatchFeeder

        # batches of Th frames per stream, 3 in flight + 2 being filled / consumed: ~1 GB page-locked
        # (1080p: 32 frames x 1 stream, 4 x 8 streams; each copy is still ~200 MB, PCIe-bound as at 128)
        Th = max(1, min(T, (32 * 1920 * 1080) // (S * H * W)))
        depth_hf = min(3, eng.max_inflight)
        n_hf = max(8 * Th, 512 // S)
        caps = [videoio.ArrayCapture([host[t % P, s] for t in range(n_hf)]) for s in range(S)]
        warm = [videoio.ArrayCapture([host[t % P, s] for t in range(2 * Th)]) for s in range(S)]
        bufs = BatchFeeder.make_buffers(eng, Th, depth_hf)  # page-locked once, outside the timed run
        for _ in BatchFeeder(eng, warm, Th, depth=depth_hf, buffers=bufs):
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ncont = 0
        for b in BatchFeeder(eng, caps, Th, depth=depth_hf, buffers=bufs):
            ncont += int(eng.counts().sum())
        dt = time.perf_counter() - t0
        gbs = n_hf * S * H * W * 3 / dt / 1e9
        host_fed = {"frames_per_s": round(n_hf * S / dt, 1), "gb_per_s": round(gbs, 2),
                    "pcie_frac": round(gbs / PCIE_GBS, 3), "frames": n_hf * S, "batch": Th, "in_flight": depth_hf,
                    "pinned_bytes": int(len(bufs) * Th * S * H * W * 3),
                    "mode": "BatchFeeder: pre-decoded frames -> page-locked batches -> hipMemcpyAsync + kernels"}
        del bufs

    # MJPEG-fed (the decode side): the synthetic frames as baseline JPEGs (Pillow,
    # quality 75, 4:2:0, no restart markers), read by BatchFeeder in JPEG mode: compressed bytes parsed on
    # the host, copied to the GPU, decoded there (fm_submit_jpeg) in front of the hot path.  Beside
    # `value`, never as it; libjpeg-turbo (Pillow) on one host core is the CPU decode rate it replaces.
    mjpeg = None
    if not args.no_mjpeg and world == 1:  # a per-GPU figure: measured in the 1-GPU run only
        mjpeg = mjpeg_fed(eng, host, T, S)

    eng.close()
    ranks = rank_devices(local, pl, active)  # (collective: every rank)

    # Side configurations in the same line (per-GPU figures, the 1-GPU run only, after the headline's
    # timed steps): mode D (-B 100 -b 20, the reference CLI's default, find_motion.py:1474) and configs[2]
    # (8 x 1080p streams batched on one GPU), each with its own roofline
    # Each leg runs in a process of its own (started as a child, after this one's GPU work), as a job of that
    # workload would: a process that already created and destroyed several engines' streams maps a new
    # detector's stream onto hardware queues differently, and configs[4]'s Haar leg then read 32-57 k against
    # 67 k in a fresh process (round 6, profiles/r06/r06c*_default_bench.log)
    side = None
    default_shape = args.mode == "F" and S == 1 and (W, H) == (1920, 1080) and not args.haar
    if world == 1 and default_shape and not args.no_side:
        side = {name: side_child(name, args) for name in SIDE_LEGS}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, host.reshape(P * S, H, W, 3), min(args.cpu_frames, P * S))

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(leg["ms_per_step"], 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8+f64",
               "data": "synthetic (find_motion_amd/synthetic.py, SURVEY.md §8d)", "config": cfg,
               "roofline": roof, "cpu_baseline": cpu, "kernels": kernels, "side_configs": side,
               # launches that found the stamp ring full between two folds (timed by events on one in four, or not)
               "unstamped_launches": leg["unstamped"],
               "ranks": {"world_size_seen": dist.world_size(active), "devices": ranks,
                         "group_backend": backend if active else None}, "host_fed_per_gpu": host_fed,
               "mjpeg_fed_per_gpu": mjpeg, "footprint_per_gpu": footprint,
               "hw_queues_per_process": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
               "haar_stage": None if det is None else haar_summary(haar, wall),
               "path_hbm": {"bytes_per_frame": path_bytes_per_frame(cfg),
                            "achieved": round(value / world * path_bytes_per_frame(cfg) / 1e9, 1), "unit": "GB/s",
                            "frac": round(value / world * path_bytes_per_frame(cfg) / 1e9 / HBM_PEAK_GBS, 4),
                            "note": "whole-path frames/s per GPU x SURVEY.md §8(d) bytes per frame"},
               "contour_pass": {"heavy_tiles_per_batch": round(ccl["heavy_tiles"] / max(ccl["batches"], 1), 2),
                                "shared_nodes_max": ccl["shared_nodes_max"],
                                "fallback_frames": ccl["fallback_frames"]},
               "host_us_per_step": leg["host_us_per_step"]}
        print(json.dumps(out), flush=True)
    dist.finalize(active)


if __name__ == "__main__":
    main()
