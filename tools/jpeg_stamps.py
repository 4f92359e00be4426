#!/usr/bin/env python3
"""Summarise k_jpeg_huff's per-tile phase stamps (dev build, FM_JPEG_STAMPS=<file>): durations of
phase 0 (speculative decode + in-wave fix-up), the look-back wait, the fix-up + scan after it, and
the writing decode, in microseconds (s_memrealtime, 100 MHz).  Usage: tools/jpeg_stamps.py <file>"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 6).astype(np.int64)
t0 = a[:, 0][a[:, 0] > 0].min()
st, p0, lb, sc, end = (a[:, i] for i in range(5))
ok = (st > 0) & (end > 0)
print(f"tiles {len(a)}, complete {ok.sum()}")
us = lambda x: x / 100.0  # noqa: E731  (10 ns ticks)
def q(name, v):
    v = v[v >= 0]
    print(f"{name:28s} median {us(np.median(v)):8.1f}  p90 {us(np.percentile(v, 90)):8.1f}  max {us(v.max()):8.1f} us")
q("start (since first tile)", st[ok] - t0)
q("phase 0", (p0 - st)[ok & (p0 > 0)])
waited = ok & (lb > 0)
q("look-back wait", (lb - p0)[waited])
q("fix-up + scan", (sc - np.where(lb > 0, lb, p0))[ok & (p0 > 0)])
q("writing decode", (end - sc)[ok & (sc > 0)])
q("end (since first tile)", end[ok] - t0)
