#!/usr/bin/env python3
"""Summarise FM_PTS k_pix workgroup stamps: span, per-workgroup durations, start skew, CU co-residency.

Usage: tools/pts.py <file> [frames_per_launch]
Each workgroup wrote [hw_id | xcc_id << 32, realtime start, realtime end (100 MHz), memtime cycles].
"""
import sys
from collections import defaultdict

import numpy as np


def main(path, T=32):
    raw = np.fromfile(path, dtype=np.uint64)
    nwg = raw.size // 36
    ph = raw[nwg * 4:].reshape(nwg, 8, 4).astype(np.float64) if raw.size == nwg * 36 else None
    v = raw[:nwg * 4].reshape(-1, 4) if ph is not None else raw.reshape(-1, 4)
    if ph is not None and ph.sum() > 0:
        tot = ph.sum(axis=2)
        print("k_pix5 per-wave phase cycles per launch (mean over workgroups; waves 0..7):")
        for k, name in enumerate(["barrier", "chain", "taps", "gray+st+ld"]):
            print(f"  {name:11s} " + " ".join(f"{x:9.0f}" for x in ph[:, :, k].mean(axis=0)))
        print("  total       " + " ".join(f"{x:9.0f}" for x in tot.mean(axis=0)))
    v = v[v[:, 1] > 0]
    hw = (v[:, 0] & 0xFFFFFFFF).astype(np.int64)
    xcc = (v[:, 0] >> np.uint64(32)).astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    t0 = v[:, 1].astype(np.int64)
    t1 = v[:, 2].astype(np.int64)
    cyc = v[:, 3].astype(np.float64)
    base = t0.min()
    s_us = (t0 - base) / 100.0
    e_us = (t1 - base) / 100.0
    d_us = e_us - s_us
    print(f"workgroups {len(v)}  span {e_us.max():.1f} us  (frames/launch {T})")
    q = lambda a: " ".join(f"{x:.1f}" for x in np.percentile(a, [0, 10, 50, 90, 100]))
    print(f"start  us p0/10/50/90/100: {q(s_us)}")
    print(f"end    us p0/10/50/90/100: {q(e_us)}")
    print(f"dur    us p0/10/50/90/100: {q(d_us)}")
    print(f"clock GHz (memtime cycles / duration) median {np.median(cyc / (d_us * 1e3)):.2f}")
    print(f"per-frame us (median dur / T): {np.median(d_us) / T:.2f}")
    slots = defaultdict(list)
    for i in range(len(v)):
        slots[(xcc[i], se[i], sh[i], cu[i])].append(i)
    cnt = np.bincount([len(x) for x in slots.values()])
    print(f"CUs used {len(slots)}; workgroups per CU histogram {dict(enumerate(cnt.tolist()))}")
    per_xcc = np.bincount(xcc, minlength=8)
    print(f"workgroups per XCC {per_xcc.tolist()}")
    # max concurrency per CU
    conc = []
    for ids in slots.values():
        ev = sorted([(s_us[i], 1) for i in ids] + [(e_us[i], -1) for i in ids])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        conc.append(m)
    print(f"max co-resident workgroups per CU histogram {dict(enumerate(np.bincount(conc).tolist()))}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 32)
