#!/usr/bin/env python3
"""Per-launch summary of FM_PTS + FM_PTS_RING k_pix5 workgroup stamps (dev build): was a long launch
long because some workgroups started late (dispatch) or because some ran slowly (shared CUs)?

Usage: tools/pts_ring.py <file> <workgroups_per_launch>
Each launch record: [nwg][4] u64 = (hw_id | xcc_id << 32, realtime start, realtime end (100 MHz), memtime
cycles), then [nwg][8][4] per-wave phase cycles (zero unless built with FM_P5_PHASES=1).
"""
import sys
from collections import Counter

import numpy as np


def main(path, nwg):
    raw = np.fromfile(path, dtype=np.uint64)
    rec = nwg * 36
    nl = raw.size // rec
    prev_end = None
    print(" launch  span  gap  start>5us  start_max  dur_p50  dur_max  late(end>p50+60): start / dur   cu2+")
    for L in range(nl):
        v = raw[L * rec:L * rec + nwg * 4].reshape(nwg, 4)
        v = v[v[:, 1] > 0]
        if len(v) == 0:
            continue
        t0 = v[:, 1].astype(np.int64)
        t1 = v[:, 2].astype(np.int64)
        base = t0.min()
        s = (t0 - base) / 100.0
        e = (t1 - base) / 100.0
        d = e - s
        hw = (v[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        xcc = (v[:, 0] >> np.uint64(32)).astype(np.int64) & 0xF
        cu = [(int(x), int((h >> 13) & 7), int((h >> 12) & 1), int((h >> 8) & 0xF)) for x, h in zip(xcc, hw)]
        per_cu = Counter(cu)
        late = np.where(e > np.median(e) + 60)[0]
        lt = " ".join(f"{s[i]:.0f}/{d[i]:.0f}" for i in late[np.argsort(-e[late])][:6])
        gap = (base - prev_end) / 100.0 if prev_end is not None else float("nan")
        prev_end = t1.max()
        print(f"{L:7d} {e.max():5.0f} {gap:5.0f} {int((s > 5).sum()):9d} {s.max():10.1f} {np.median(d):8.0f} {d.max():8.0f}"
              f"  {len(late):3d}: {lt:40s} {sum(1 for c in per_cu.values() if c > 2)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
