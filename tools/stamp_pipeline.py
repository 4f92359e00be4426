#!/usr/bin/env python3
"""stamp_pipeline.py LOG -- per-batch pipeline from the dev build's launch stamps (FM_STAMP_DUMP=1: every
stamped launch's first-workgroup start and last-wave end, s_memrealtime ticks of 10 ns, in launch order).
Prints, for the last batches, when each stage ran relative to the batch's resize start (us), and the gaps
on the input stream between consecutive resizes."""
import sys
from collections import defaultdict


def main(path, last=20):
    seq = defaultdict(list)
    for line in open(path):
        p = line.split()
        if len(p) == 4 and p[0] == "kstamp":
            seq[p[1]].append((int(p[2]), int(p[3])))
    names = [n for n in ("resize_area", "small_blur", "small_scan", "pix", "chain_regions", "chain_counts", "frame_contours") if seq.get(n)]
    n = min(len(seq[k]) for k in names)
    rows = [{k: seq[k][len(seq[k]) - n + i] for k in names} for i in range(n)][-last:]
    first = names[0]
    print("batch  " + "  ".join(f"{k:>22s}" for k in names) + "   (us from the batch's first-stage start: start-end)")
    for i, r in enumerate(rows):
        t0 = r[first][0]
        print(f"{i:5d}  " + "  ".join(f"{(r[k][0] - t0) / 100:9.1f}-{(r[k][1] - t0) / 100:9.1f}" for k in names))
    for k in names:
        g = [(rows[i + 1][k][0] - rows[i][k][1]) / 100 for i in range(len(rows) - 1)]
        d = [(r[k][1] - r[k][0]) / 100 for r in rows]
        print(f"{k:14s} duration avg {sum(d) / len(d):7.1f} us; gap to the next launch avg {sum(g) / max(len(g), 1):7.1f} "
              f"min {min(g, default=0):7.1f} max {max(g, default=0):7.1f}")
    last_stage = "chain_counts" if "chain_counts" in names else "frame_contours" if "frame_contours" in names else None
    if last_stage:
        lag = [(r[last_stage][1] - r[first][0]) / 100 for r in rows]
        print(f"batch latency ({first} start -> chain end): avg {sum(lag) / len(lag):.1f} us, max {max(lag):.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
