#!/usr/bin/env python3
"""Throughput of the object-ROI stage (fm_haar_detect_frames): 1080p raw frames ->
INTER_AREA to width 300 -> HAAR cascade detectMultiScale(1.1, 5), batched.

The cascade is synthetic with frontalface_default's shape (24x24 window, 25
stages with its per-stage tree counts, ~2.7k stumps; the reference's cascade files are not on the GPU box) and
the frames are synthetic scenes with bright squares; stage thresholds are
calibrated to pass about half of the windows reaching each stage, so the
rejection profile resembles, but is not, a trained cascade's: the line reports windows/s and the stage-0 pass
rate next to frames/s.  A CPU figure comes from oracle/haar.py on a few frames
(numpy restatement, not OpenCV).

Usage: python tools/bench_haar.py [--frames 64] [--iters 20] [--cpu-frames 1] [--frontalface]

--frontalface runs the reference's own cascade (config 5) from its committed fixture arrays.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

# frontalface_default.xml: weak classifiers per stage
FACE_DEFAULT_TREES = [9, 16, 27, 32, 52, 53, 62, 72, 83, 91, 99, 115, 127, 135, 136, 137, 159, 155, 169, 196, 197,
                      181, 199, 211, 200]


def face_shaped_cascade(seed=0):
    from find_motion_amd.cascade import THRESHOLD_EPS, Cascade
    from haar_cases import make_cascade
    parts = [make_cascade(seed * 100 + i, win=(24, 24), stages=2, trees=t, tight=0.3)
             for i, t in enumerate(FACE_DEFAULT_TREES)]
    # stage 0 of part 0 (centre-surround) then stage 1 of every part
    p0 = parts[0]
    rects, wts, tl = [p0.feat_rects[:1]], [p0.feat_weights[:1]], [p0.feat_tilted[:1]]
    ntrees, sthr, tnodes = [1], [p0.stage_threshold[0]], [1]
    left, right, feat, nthr, leaves = [0], [-1], [0], [p0.node_threshold[0]], list(p0.leaves[:2])
    nf = 1
    for p in parts[:-1]:
        k = int(p.stage_ntrees[1])
        ntrees.append(k)
        sthr.append(p.stage_threshold[1])
        tnodes += [1] * k
        left += [0] * k
        right += [-1] * k
        feat += list(range(nf, nf + k))
        nthr += list(p.node_threshold[1:1 + k])
        leaves += list(p.leaves[2:2 + 2 * k])
        rects.append(p.feat_rects[p.node_feature[1:1 + k]])
        wts.append(p.feat_weights[p.node_feature[1:1 + k]])
        tl.append(p.feat_tilted[p.node_feature[1:1 + k]])
        nf += k
    _ = THRESHOLD_EPS
    return Cascade(24, 24, np.asarray(ntrees, np.int32), np.asarray(sthr, np.float32), np.asarray(tnodes, np.int32),
                   np.asarray(left, np.int32), np.asarray(right, np.int32), np.asarray(feat, np.int32),
                   np.asarray(nthr, np.float32), np.asarray(leaves, np.float32), np.concatenate(rects),
                   np.concatenate(wts), np.concatenate(tl))


def calibrate(cs, img, keep=0.5):
    """Set every stage's threshold after stage 0 to the `keep` quantile of its sums over the
    windows that reach it (scale 1 of a calibration frame), so windows drop out stage by stage
    the way a trained cascade rejects them (about half per stage) instead of all-or-nothing."""
    from oracle import haar
    g = haar.bgr2gray(img)
    S, Q, T = haar.integrals(g, cs.has_tilted)
    gy, gx = np.meshgrid(np.arange(0, g.shape[0] + 1 - cs.win_h, 2), np.arange(0, g.shape[1] + 1 - cs.win_w, 2),
                         indexing="ij")
    xs, ys = gx.ravel(), gy.ravel()
    W, H = cs.win_w, cs.win_h
    area = float((W - 2) * (H - 2))
    vs = haar._rect_sum(S, xs, ys, (1, 1, W - 2, H - 2), False).astype(np.float64)
    vq = (haar._rect_sum(Q, xs, ys, (1, 1, W - 2, H - 2), False).astype(np.int64) & 0xFFFFFFFF).astype(np.float64)
    nf = area * vq - vs * vs
    ok = nf > 0
    vnf = np.ones(len(xs), np.float32)
    vnf[ok] = (1.0 / np.sqrt(nf[ok])).astype(np.float32)
    alive = np.nonzero(ok & (area * vnf.astype(np.float64) < 0.1))[0]
    ni = li = 0
    thr = cs.stage_threshold.copy()
    for si in range(cs.n_stages):
        tot = np.zeros(len(alive))
        for _ in range(int(cs.stage_ntrees[si])):
            f = int(cs.node_feature[ni])
            tl = bool(cs.feat_tilted[f])
            I = T if tl else S
            v = None
            for j in range(3):
                if j == 2 and cs.feat_weights[f, j] == 0:
                    continue
                t = (np.float32(cs.feat_weights[f, j]) *
                     haar._rect_sum(I, xs[alive], ys[alive], cs.feat_rects[f, j], tl).astype(np.float32))
                v = t if v is None else (v + t).astype(np.float32)
            v = (v * vnf[alive]).astype(np.float32)
            tot += np.where(v < cs.node_threshold[ni], cs.leaves[li], cs.leaves[li + 1])
            ni += 1
            li += 2
        if si > 0 and len(alive):
            thr[si] = np.float32(np.quantile(tot, 1 - keep))
        alive = alive[tot >= thr[si]]
    cs.stage_threshold = thr.astype(np.float32)
    return cs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64, help="raw 1080p frames per call (ROI frames of many streams)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu-frames", type=int, default=1)
    ap.add_argument("--cascade", default=None, help="a real haarcascade_*.xml instead of the synthetic one")
    ap.add_argument("--frontalface", action="store_true",
                    help="the reference's haarcascade_frontalface_default (parsed arrays in tests/golden)")
    args = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, then libfm_hip: DESIGN §1)
    from find_motion_amd import CascadeClassifier
    from haar_cases import make_image

    from haar_cases import make_image as _mi
    if args.frontalface:
        from golden_cases import load_frontalface
        cs = load_frontalface()[0]
        args.cascade = "haarcascade_frontalface_default (tests/golden/cascade_frontalface_default.npz)"
    elif args.cascade:
        from find_motion_amd.cascade import parse
        cs = parse(args.cascade)
    else:
        cs = calibrate(face_shaped_cascade(), _mi(1000, 300, 168))
    W, H = 1920, 1080
    frames = np.empty((args.frames, H, W, 3), np.uint8)
    ys = (np.arange(H) * 169) // H
    xs = (np.arange(W) * 300) // W
    for i in range(args.frames):
        frames[i] = make_image(i, 300, 169)[ys][:, xs]
    det = CascadeClassifier(cs)
    print("frames ready", file=sys.stderr, flush=True)
    det.detect_frames(frames, 300, 1.1, 5)  # warm-up (allocations, tables)
    print(f"warm-up: {det.last_ms():.3f} ms device, {len(det.candidates())} candidates in frame 0", file=sys.stderr,
          flush=True)
    gpu_ms = []
    t0 = time.perf_counter()
    for it in range(args.iters):
        out = det.detect_frames(frames, 300, 1.1, 5)
        gpu_ms.append(det.last_ms())
        print(f"iter {it}: {gpu_ms[-1]:.3f} ms device", file=sys.stderr, flush=True)
    wall = time.perf_counter() - t0
    n = args.frames * args.iters
    # windows per ROI frame and stage-0 pass rate, from the restatement's geometry
    from oracle import haar
    geo = haar.scale_geometry(300, 168, cs.win_w, cs.win_h, haar.scale_list(300, 168, cs.win_w, cs.win_h, 1.1))
    nwin = sum(((g["ww"] + g["ystep"] - 1) // g["ystep"]) * ((g["ylim"] + g["ystep"] - 1) // g["ystep"])
               for g in geo)
    res = {"metric": "ROI frames/s through find_objects (1080p raw -> 300 px ROI -> detectMultiScale 1.1/5)",
           "value": round(n / wall, 1), "unit": "frames/s", "frames_per_call": args.frames,
           "device_ms_per_call": round(float(np.mean(gpu_ms)), 3),
           "device_frames_per_s": round(args.frames / (np.mean(gpu_ms) / 1e3), 1),
           "windows_per_frame": nwin, "detections_frame0": int(len(out[0])),
           "cascade": (args.cascade if args.cascade else "synthetic, frontalface_default shape") +
                      f" ({cs.win_w}x{cs.win_h}, {cs.n_stages} stages, {len(cs.tree_nodes)} trees)",
           "note": "wall includes the H2D copy of the raw frames (PCIe); device_ms covers gray..eval kernels"}
    if args.cpu_frames > 0:
        import oracle as orc
        t0 = time.perf_counter()
        for i in range(args.cpu_frames):
            haar.detect_multiscale(cs, orc.resize_area_bgr(frames[i], 300), 1.1, 5)
        res["cpu_baseline"] = {"value": round(args.cpu_frames / (time.perf_counter() - t0), 2), "unit": "frames/s",
                               "cores": 1, "kind": "port",
                               "sample": f"{args.cpu_frames} frames, oracle/haar.py (numpy), not OpenCV"}
    # frames already resident in HBM (the motion path's ring / the MJPEG decoder's output): no H2D copy
    dev = torch.from_numpy(frames).to("cuda:0")
    det.detect_frames(dev, 300, 1.1, 5)
    t0 = time.perf_counter()
    for it in range(args.iters):
        det.detect_frames(dev, 300, 1.1, 5)
    res["resident_frames_per_s"] = round(n / (time.perf_counter() - t0), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
