"""Debug: where the GPU dilated mask differs from the oracle (mode F small case)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import oracle
from find_motion_amd import MotionEngine, make_gaussian
from find_motion_amd.synthetic import batch

W, H, box = 160, 120, 160
k = make_gaussian(box, 32)
eng = MotionEngine(n_streams=1, src_w=W, src_h=H, box_size=box, ksize=k, threshold=12, avg=0.1, max_batch=3,
                   keep_planes=True)
cfg = oracle.OracleConfig(H=H, W=W, box=box, ksize=k)
orc = oracle.OracleStream(cfg)
fr = batch(W, H, 1, 0, 3)
eng.submit(fr); eng.wait()
for t in range(3):
    ref = orc.step(fr[t, 0])
    got = eng.mask(t, 0)
    th = (ref["delta"] > 12)
    bad = np.argwhere(got != ref["mask"])
    print("frame", t, "bad", len(bad), "thresh px", th.sum(), "got on", (got > 0).sum(), "ref on", (ref["mask"] > 0).sum())
    if len(bad):
        ys, xs = bad[:, 0], bad[:, 1]
        print(" rows", np.unique(ys)[:40], "cols", np.unique(xs)[:80])
        print(" extra", ((got > 0) & (ref["mask"] == 0)).sum(), "missing", ((got == 0) & (ref["mask"] > 0)).sum())
