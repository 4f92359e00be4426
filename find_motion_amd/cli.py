"""Command line with the reference's flag surface (fm.py:1448-1489) plus GPU placement.

    python -m find_motion_amd [files] -i DIR -o DIR -c cfg.ini -B 100 -b 20 -t 12 -a 0.1 ...
                              [--gpus N] [--device D] [--batch T] [--group] [--gpu-decode]

Everything the reference's `run` does around the hot path is kept in its
shape (INI overriding the CLI, masks from literals and a JSON file, mtime
ordering with HH:MM priority windows, progress.log resume), compactly; the
per-video work is find_motion_amd.motion.run_vid (or StreamGroup).

Parallelism: the reference runs -J worker processes, one video each
(run_pool, fm.py:1054-1122).  Here the unit of placement is the GPU: with
--gpus N the files are split into N contiguous shards (stream s -> GPU
s // ceil(S/N)), one worker process per GPU, each pinned with
HIP_VISIBLE_DEVICES before it touches the device; results come back to the
parent as run_vid tuples (the host-side gather of fm.py:1087).  There is no
collective: videos are independent.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
import typing
from argparse import ArgumentParser, Namespace
from ast import literal_eval
from configparser import ConfigParser

log = logging.getLogger("find_motion_amd")

LINE_BUFFERED = 1


def get_args(parser: ArgumentParser) -> None:
    """fm.py:1448-1489, plus --gpus/--device/--batch/--group."""
    parser.add_argument("files", nargs="*", help="Video files to find motion in")
    parser.add_argument("--config", "-c", help="Config in INI format")
    parser.add_argument("--cameras", nargs="*", type=int, help="0-indexed number of camera to stream from")
    parser.add_argument("--input-dir", "-i", help="Input directory to process")
    parser.add_argument("--output-dir", "-o", default="", help="Output directory for processed files")
    parser.add_argument("--ignore-progress", "-I", action="store_true", default=False, help="Ignore progress log")
    parser.add_argument("--ignore-drive", "-D", action="store_true", default=False,
                        help="Ignore drive letter in progress log")
    parser.add_argument("--codec", "-k", default="MP42", help="Codec to write files with")
    parser.add_argument("--fps", "-f", type=int, default=30, help="Frames per second of input files")
    parser.add_argument("--time_order", "-to", nargs="*",
                        help='Time ranges in priority order for processing. Express as "HH:MM-HH:MM"')
    parser.add_argument("--masks", "-m", nargs="*", type=literal_eval, help="Areas to mask off in video")
    parser.add_argument("--masks_file", help="File holding mask coordinates (JSON)")
    parser.add_argument("--cascade-object", "-O", nargs="*", type=str,
                        help="Specific types of objects to detect using haar cascades (slow!)")
    parser.add_argument("--yolo-tiny", "-yt", action="store_true", help="Use fast common object detection")
    parser.add_argument("--blur-scale", "-b", type=int, default=20,
                        help="Scale of gaussian blur size compared to video width (used as 1/blur_scale)")
    parser.add_argument("--box-size", "-B", type=int, default=100, help="Pixel size to scale the video to for processing")
    parser.add_argument("--min-box-scale", "-mbs", type=int, default=50,
                        help="Scale of minimum motion compared to video width (used as 1/min_box_scale")
    parser.add_argument("--threshold", "-t", type=int, default=12, help="Threshold for change in grayscale")
    parser.add_argument("--mintime", "-M", type=float, default=0.5, help="Minimum time for motion, in seconds")
    parser.add_argument("--cachetime", "-C", type=float, default=1.0, help="How long to cache, in seconds")
    parser.add_argument("--avg", "-a", type=float, default=0.1,
                        help="How much to weight the most recent frame in the running average")
    parser.add_argument("--processes", "-J", default=1, type=int, help="Number of processors to use")
    parser.add_argument("--progress", "-p", action="store_true", help="Show progress bar")
    parser.add_argument("--show", "-s", action="store_true", default=False, help="Show video processing")
    parser.add_argument("--cleanup", "-cu", action="store_true",
                        help="Cleanup used frames (do not wait for garbage collection)")
    parser.add_argument("--mem", "-u", action="store_true", help="Run memory usage")
    parser.add_argument("--debug", "-d", action="store_true", help="Debug")
    parser.add_argument("--test", "-T", action="store_true", help="Test which files or camera streams would be processed")
    # MI355X placement
    parser.add_argument("--gpus", type=int, default=1, help="GPUs to shard the videos over (one process per GPU)")
    parser.add_argument("--device", type=int, default=0, help="HIP device for a single-GPU run")
    parser.add_argument("--batch", type=int, default=8, help="Frames per stream decoded ahead per kernel launch")
    parser.add_argument("--group", action="store_true",
                        help="Batch same-sized videos of a GPU's shard into one launch (StreamGroup)")
    parser.add_argument("--gpu-decode", action="store_true", default=None,
                        help="Decode MJPEG AVIs on the GPU (libjpeg-turbo-exact) even when OpenCV is present")


def process_config(config_file: str, args: Namespace) -> Namespace:
    """fm.py:1418-1445: the INI [settings] section overrides the command line."""
    config = ConfigParser()
    config.read(config_file)
    for setting, value in config["settings"].items():
        setting = setting.replace("-", "_")
        use_value: typing.Any = value
        if setting in ("processes", "blur_scale", "min_box_scale", "threshold", "fps", "box_size", "gpus", "batch"):
            use_value = int(value)
        if setting in ("mintime", "cachetime", "avg"):
            use_value = float(value)
        if setting in ("mem", "progress", "debug", "show", "ignore_progress", "ignore_drive", "yolo_tiny", "group",
                       "gpu_decode"):
            if value not in ("True", "False"):
                raise ValueError("{} must be True or False".format(setting))
            use_value = value == "True"
        if setting in ("masks", "cameras", "time_order"):
            use_value = literal_eval(value)
        setattr(args, setting, use_value)
    return args


def _valid_masks(masks) -> bool:
    """MASK_SCHEMA (fm.py:86-100): a list of polygons of >= 2 [int, int] points."""
    return isinstance(masks, list) and all(
        isinstance(m, list) and len(m) >= 2 and all(
            isinstance(p, list) and len(p) == 2 and all(isinstance(v, int) and not isinstance(v, bool) for v in p)
            for p in m) for m in masks)


def read_masks(masks_file: str) -> list:
    """fm.py:1269-1284"""
    try:
        with open(masks_file, "r") as mf:
            masks = json.load(mf)
        if not _valid_masks(masks):
            raise ValueError("masks do not match MASK_SCHEMA")
        return [tuple(tuple(c) for c in m) for m in masks]
    except Exception as e:  # noqa: BLE001
        log.error("Masks file not read ({}): {}".format(masks_file, e))
        return []


def find_files(directory) -> typing.List[str]:
    """fm.py:929-933"""
    if directory is None:
        return []
    return [os.path.normpath(os.path.abspath(os.path.join(d, f))) for d, _, fs in os.walk(directory) for f in fs
            if f != "progress.log"]


def verify_files(file_list) -> typing.List[str]:
    """fm.py:936-940"""
    return [os.path.normpath(os.path.abspath(f)) for f in (file_list or []) if os.path.isfile(f)]


def process_times(time_order):
    """fm.py:1401-1415"""
    times = []
    for slot in time_order or []:
        try:
            a, b = (time.strptime(t, "%H:%M") for t in slot.split("-"))
        except ValueError as e:
            log.error("Time interval {} misparsed: {}".format(slot, e))
            continue
        times.append((a, b))
    return times


def _clock(st) -> tuple:
    return (st.tm_hour, st.tm_min, st.tm_sec)  # ClockTime ordering (fm.py:984-1018)


def sort_files_by_time(file_list, priority_intervals) -> list:
    """fm.py:943-981: by mtime, files whose mtime (UTC clock) falls in a priority window first."""
    files = sorted(((f, os.path.getmtime(f)) for f in file_list), key=lambda f: f[1])
    out, seen = [], set()
    for lo, hi in priority_intervals:
        for f in files:
            if _clock(lo) <= _clock(time.gmtime(f[1])) < _clock(hi) and f not in seen:
                out.append(f)
                seen.add(f)
    out.extend(f for f in files if f not in seen)
    return out


def get_progress(log_file: str) -> set:
    """fm.py:1040-1051"""
    try:
        with open(log_file, "r") as fh:
            return {line.split(" // ")[0].strip() for line in fh}
    except FileNotFoundError:
        return set()


def process_progress(files, log_file: str, ignore_drive: bool = False):
    """fm.py:1389-1398 (ignore_drive compares paths without their drive, which the reference intends)."""
    done = get_progress(log_file)
    if ignore_drive:
        done = {os.path.splitdrive(d)[1] for d in done}
        return [f for f in files if os.path.splitdrive(f[0])[1] not in done]
    return [f for f in files if f[0] not in done]


def set_log_file(input_dir=None, output_dir=None) -> str:
    """fm.py:1287-1288"""
    return os.path.normpath(os.path.join(output_dir if output_dir else input_dir if input_dir is not None else ".",
                                         "progress.log"))


def shard(items: list, n: int) -> typing.List[list]:
    """Contiguous blocks: item s -> shard s // ceil(S / n)."""
    n = max(1, int(n))
    per = -(-len(items) // n) if items else 0
    return [items[i * per:(i + 1) * per] for i in range(n)]


def _job_kwargs(args) -> dict:
    """fm.py:1323-1331"""
    return dict(outdir=args.output_dir, mask_areas=args.masks, show=args.show, codec=args.codec,
                log_level=logging.DEBUG if args.debug else logging.INFO, mem=args.mem, cleanup=args.cleanup,
                blur_scale=args.blur_scale, box_size=args.box_size, min_box_scale=args.min_box_scale,
                threshold=args.threshold, avg=args.avg, fps=args.fps, min_time=args.mintime,
                cache_time=args.cachetime, multiprocess=args.processes > 1, cascades=args.cascade_object,
                yolo_tiny=args.yolo_tiny, gpu_decode=getattr(args, "gpu_decode", None))


def run_shard(files: list, kwargs: dict, device: int, batch: int, group: bool) -> list:
    """One GPU's share of the videos: run_vid per file, or one StreamGroup for the whole shard."""
    from .motion import StreamGroup, run_vid

    if not files:
        return []
    if group and len(files) > 1:
        try:
            return StreamGroup(files, batch=batch, device=device, **kwargs).find_motion()
        except Exception as e:  # noqa: BLE001 - e.g. mixed frame sizes: fall back to one video at a time
            log.warning("StreamGroup not usable for this shard ({}); processing videos one by one".format(e))
    return [run_vid(f, device=device, batch=batch, **kwargs) for f in files]


def _shard_worker(args_tuple):
    files, kwargs, gpu, batch, group = args_tuple
    os.environ["HIP_VISIBLE_DEVICES"] = str(gpu)  # before anything touches the device
    return run_shard(files, kwargs, 0, batch, group)


def run_sharded(files: list, kwargs: dict, gpus: int, batch: int, group: bool) -> list:
    """One process per GPU over contiguous shards; results gathered in file order."""
    kwargs = dict(kwargs)
    device = kwargs.pop("device", 0)
    shards = shard(files, gpus)
    if gpus <= 1:
        return run_shard(files, kwargs, device, batch, group)
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    with ctx.Pool(processes=gpus) as pool:
        parts = pool.map(_shard_worker, [(s, kwargs, g, batch, group) for g, s in enumerate(shards)])
    return [r for p in parts for r in p]


def run(args: Namespace, print_help: typing.Callable = lambda: None) -> list:
    """fm.py:1291-1385 (secondary entry point for embedding)."""
    if args.config:
        process_config(args.config, args)
    if args.debug or args.test:
        log.setLevel(logging.DEBUG)
    if not args.files and not args.input_dir and not args.cameras:
        print_help()
        sys.exit(2)
    if args.output_dir and not os.path.isdir(args.output_dir):
        os.mkdir(args.output_dir)
    masks = list(args.masks) if args.masks else []
    if args.masks_file:
        masks.extend(read_masks(args.masks_file))
    args.masks = masks
    log_file = set_log_file(args.input_dir, args.output_dir)
    kwargs = _job_kwargs(args)
    if args.cameras:
        sources = list(args.cameras)
    else:
        files = sort_files_by_time(verify_files(args.files) + find_files(args.input_dir),
                                   process_times(args.time_order))
        if not args.ignore_progress:
            files = process_progress(files, log_file, args.ignore_drive)
        if args.test:
            for f in files:
                log.info("would process %s", f[0])
            sys.exit(0)
        sources = [f[0] for f in files]
    if not sources:
        log.error("More than 0 files needed")
        return []
    kwargs["device"] = args.device
    results = run_sharded(sources, kwargs, args.gpus, args.batch, args.group)
    with open(log_file, "a+", LINE_BUFFERED) as progress_log:
        for wrote_frames, filename, err_msg, seen_objects in results:
            if err_msg:
                log.error("Error processing {}: {}".format(filename, err_msg))
            elif not args.cameras:
                print("{} // {}".format(filename, seen_objects), file=progress_log)
            else:
                print("Finished streaming from camera {}".format(filename), file=progress_log)
    return results


def hw_queues_from_env(env=None) -> tuple:
    """(count, force) for use_hw_queues: FM_HW_QUEUES, when set, is validated (1..32, HIP's accepted range)
    and forced over any GPU_MAX_HW_QUEUES; otherwise an exported GPU_MAX_HW_QUEUES is honoured and 8 is
    the default (with HIP's 4 the input stream shares an in-order queue with a contour stream)."""
    env = os.environ if env is None else env

    def checked(name: str, v: str) -> int:
        try:
            n = int(v)
        except ValueError:
            raise SystemExit(f"{name}={v!r}: expected an integer in 1..32") from None
        if not 1 <= n <= 32:
            raise SystemExit(f"{name}={n}: expected an integer in 1..32")
        return n

    v = env.get("FM_HW_QUEUES")
    if v is None:
        # an exported GPU_MAX_HW_QUEUES is kept (use_hw_queues does not force), but only a value HIP accepts
        if env.get("GPU_MAX_HW_QUEUES") is not None:
            checked("GPU_MAX_HW_QUEUES", env["GPU_MAX_HW_QUEUES"])
        return 8, False
    return checked("FM_HW_QUEUES", v), True


def main(argv=None) -> None:
    from . import use_hw_queues
    n, force = hw_queues_from_env()
    use_hw_queues(n, force=force)  # before any HIP call (inherited by --gpus workers)
    if int(os.environ["GPU_MAX_HW_QUEUES"]) < 8:
        log.info("GPU_MAX_HW_QUEUES=%s from the environment (FM_HW_QUEUES=8 gives each pipeline stream its own "
                 "hardware queue)", os.environ["GPU_MAX_HW_QUEUES"])
    parser = ArgumentParser(description="Find motion and objects in video (MI355X)")
    get_args(parser)
    args = parser.parse_args(argv)
    logging.basicConfig()
    if args.debug:
        log.setLevel(logging.DEBUG)
    run(args, parser.print_help)
