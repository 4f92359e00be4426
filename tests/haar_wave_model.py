"""Wave-level cost of k_hdetect's window sweep, from the oracle's per-window failing stages (round 6).

Not a test: `python tests/haar_wave_model.py` prints, for the committed frontalface ROI fixture, how many
stump evaluations the sweep issues per *wave* (64 lanes each, whether live or not) under the phase layouts
profiles/r06/r06p_haar_phases_ab.txt compares, against the live-lane count. A wave issues a stage's stumps
when any of its lanes is still alive at that stage.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def stage_counts():
    """Per scale: stages each window evaluates, on the k_hdetect window grid."""
    from golden_cases import load_frontalface
    from oracle import haar
    cs, z = load_frontalface()
    g = haar.bgr2gray(z["roi_image"])
    h, w = g.shape
    out = []
    for geo in haar.scale_geometry(w, h, cs.win_w, cs.win_h, haar.scale_list(w, h, cs.win_w, cs.win_h, 1.1)):
        if geo["ww"] == 0 or geo["ylim"] <= 0:
            continue
        im = haar.resize_linear_exact(g, geo["sw"], geo["sh"])
        S, Q, T = haar.integrals(im, cs.has_tilted)
        st = geo["ystep"]
        gy, gx = np.meshgrid(np.arange(0, geo["ylim"], st), np.arange(0, geo["ww"], st), indexing="ij")
        res = haar.eval_windows(cs, S, Q, T, gx.ravel(), gy.ravel()).reshape(gy.shape)
        # (eval_windows gives -1 for flat windows and stage-1 rejects alike: both priced as two stages)
        out.append(np.where(res > 0, cs.n_stages, -res + 1))
    return np.asarray(cs.stage_ntrees, int), out


def wave_stumps(nt, grids, compact_at=(), split=4, spread_tail=True, tile=16):
    """(head, tail) wave-stumps: phases end at the stages in compact_at and at split; the tail's survivors
    either spread over the tile's 4 waves (survivor k -> wave k % 4) or packed into the first waves."""
    head = tail = 0
    for nst in grids:
        for by in range(0, nst.shape[0], tile):
            for bx in range(0, nst.shape[1], tile):
                blk = np.zeros((tile, tile), int)
                part = nst[by:by + tile, bx:bx + tile]
                blk[:part.shape[0], :part.shape[1]] = part
                lanes = blk.ravel()
                waves = [lanes[64 * i:64 * i + 64] for i in range(tile * tile // 64)]
                for s in range(split):
                    if s in compact_at:
                        surv = lanes[lanes > s]
                        waves = [surv[64 * i:64 * i + 64] for i in range((len(surv) + 63) // 64)]
                    head += sum(64 * nt[s] for wv in waves if (wv > s).any())
                surv = lanes[lanes > split]
                tw = [surv[i::4] for i in range(4)] if spread_tail else \
                     [surv[64 * i:64 * i + 64] for i in range((len(surv) + 63) // 64)]
                tail += sum(64 * nt[s] for wv in tw for s in range(split, len(nt)) if (wv > s).any())
    return head, tail


if __name__ == "__main__":
    nt, grids = stage_counts()
    cum = np.concatenate([[0], np.cumsum(nt)])
    live = sum(int(cum[np.minimum(gd, len(nt))].sum()) for gd in grids)
    print("live lane-stumps", live)
    for name, kw in [("round 5/6 product: head 4 per thread, tail spread", dict()),
                     ("tail packed", dict(spread_tail=False)),
                     ("compaction after 1, 2, 4 + tail packed", dict(compact_at=(1, 2), spread_tail=False))]:
        hd, tl = wave_stumps(nt, grids, **kw)
        print(f"{name}: head {hd}, tail {tl}, total {hd + tl}")
