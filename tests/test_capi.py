"""The C-ABI library (find_motion_amd/libfm_hip.so) on a machine without a GPU.

Checks that the library loads, exports every entry point include/*.h declares,
and that its host-only parts behave: the mask rasteriser that replaces
mask_off_areas (fm.py:611-636) and argument validation of fm_create (no
device call is made for invalid parameters).  No compute call is made here.
"""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

from find_motion_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names.update(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(fm_[a-z_0-9]+)\s*\(", src, flags=re.M))
    return names


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("fm_create", "fm_destroy", "fm_submit", "fm_wait", "fm_get_counts", "fm_get_contours",
              "fm_read_mask", "fm_read_background", "fm_set_mask", "fm_last_error", "fm_rasterize_masks"):
        assert n in names
    assert names == set(_native.EXPORTED), names ^ set(_native.EXPORTED)


def test_library_loads_and_exports_every_declared_symbol():
    L = _native.load()
    for n in declared_functions():
        assert hasattr(L, n), n
    assert L.fm_abi_version() == 1


def test_fm_create_rejects_bad_params_without_touching_the_device():
    L = _native.load()
    h = C.c_void_p()
    for kw in (dict(ksize=4), dict(ksize=0), dict(n_streams=0), dict(box_size=0), dict(max_batch=0)):
        p = dict(device=0, n_streams=1, src_w=64, src_h=48, box_size=64, ksize=5, threshold=12, avg=0.1,
                 max_batch=1, max_contours=16, flags=0)
        p.update(kw)
        rc = L.fm_create(C.byref(h), C.byref(_native.FMParams(*p.values())))
        assert rc == _native.FM_EINVAL, kw
        assert L.fm_last_error(None)
    p = _native.FMParams(0, 1, 64, 48, 128, 5, 12, 0.1, 1, 16, 0)  # box > width: INTER_AREA upscaling
    assert L.fm_create(C.byref(h), C.byref(p)) == _native.FM_ENOTSUP
    assert not h.value


def test_null_context_calls_fail_cleanly():
    L = _native.load()
    assert L.fm_wait(None) == _native.FM_EINVAL
    assert L.fm_submit(None, None, 1, 0) == _native.FM_EINVAL
    assert L.fm_reset_stream(None, 0) == _native.FM_EINVAL
    L.fm_destroy(None)


# --- mask rasteriser (mask_off_areas, fm.py:619-636) --------------------------

def rect_keep(h, w, scale, p0, p1):
    """cv2.rectangle(blur, p0, p1, BLACK, FILLED) after scale_area (fm.py:616): inclusive, clipped."""
    (x0, y0), (x1, y1) = [(int(x * scale), int(y * scale)) for x, y in (p0, p1)]
    keep = np.ones((h, w), np.uint8)
    xa, xb = sorted((x0, x1))
    ya, yb = sorted((y0, y1))
    keep[max(ya, 0):max(yb + 1, 0), max(xa, 0):max(xb + 1, 0)] = 0
    return keep


@pytest.mark.parametrize("p0,p1,scale", [((0, 0), (10, 5), 1.0), ((10, 5), (0, 0), 1.0), ((3, 3), (3, 3), 1.0),
                                         ((-5, -5), (4, 200), 1.0), ((0, 0), (639, 359), 0.5),
                                         ((100, 50), (1900, 1000), 100 / 1920), ((30, 20), (200, 300), 1.0)])
def test_rectangle_is_inclusive_box(p0, p1, scale):
    h, w = 40, 64
    got = _native.rasterize_masks(h, w, scale, [[p0, p1]])
    np.testing.assert_array_equal(got, rect_keep(h, w, scale, p0, p1))


def test_triangle_known_answer():
    # fillConvexPoly((0,0),(4,0),(0,4)): the Bresenham hypotenuse hits x + y == 4, the fill x + y <= 4
    keep = _native.rasterize_masks(8, 8, 1.0, [[(0, 0), (4, 0), (0, 4)]])
    yy, xx = np.mgrid[:8, :8]
    np.testing.assert_array_equal(keep == 0, (xx + yy) <= 4)


def test_convex_polygon_covers_interior_and_stays_near_hull():
    h, w = 60, 80
    tri = [(70, 5), (10, 30), (60, 55)]
    keep = _native.rasterize_masks(h, w, 1.0, [tri])
    yy, xx = np.mgrid[:h, :w].astype(np.float64)

    orient = np.sign((tri[1][0] - tri[0][0]) * (tri[2][1] - tri[0][1]) - (tri[1][1] - tri[0][1]) * (tri[2][0] - tri[0][0]))

    def inside(margin):
        """pixel centres at least `margin` px inside every edge (negative: outside allowance)"""
        ok = np.ones((h, w), bool)
        for i in range(3):
            (ax, ay), (bx, by) = tri[i], tri[(i + 1) % 3]
            dist = orient * ((bx - ax) * (yy - ay) - (by - ay) * (xx - ax)) / np.hypot(bx - ax, by - ay)
            ok &= dist >= margin
        return ok

    assert (keep[inside(1.0)] == 0).all()      # interior masked
    assert (keep[~inside(-1.5)] == 1).all()    # nothing far outside masked


def test_config5_masks_and_union():
    masks = [[(0, 0), (639, 359)], [(3839, 2159), (3200, 2159), (3839, 1600)]]
    keep = _native.rasterize_masks(2160 // 8, 3840 // 8, 1 / 8, masks)
    assert keep[:44, :79].sum() == 0 and keep[45:, 80:].min() == 0  # rect + triangle region
    assert keep[100, 200] == 1 and keep[-1, -1] == 0
    none = _native.rasterize_masks(10, 10, 1.0, [])
    assert none.all()


def test_polygon_with_one_point_rejected():
    with pytest.raises(_native.FMError):
        _native.rasterize_masks(10, 10, 1.0, [[(1, 1)]])


def test_import_leaves_hw_queues_alone():
    """Importing the package does not touch GPU_MAX_HW_QUEUES (it would change the queue setup of every HIP
    user in the process); use_hw_queues() is the explicit opt-in the CLI and bench.py make."""
    import os
    import subprocess
    import sys
    code = ("import os, find_motion_amd as f; a = os.environ.get('GPU_MAX_HW_QUEUES'); "
            "b = f.use_hw_queues(); print(a, b, os.environ['GPU_MAX_HW_QUEUES'])")
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["None", "8", "8"], out.stdout + out.stderr


def test_use_hw_queues_env_wins_unless_forced():
    """A GPU_MAX_HW_QUEUES already in the environment stays (use_hw_queues()), unless forced, as the CLI and
    bench.py do: machines commonly export HIP's default 4, which serialises the input stream behind a
    contour stream."""
    import os
    import subprocess
    import sys
    code = ("import os, find_motion_amd as f; a = f.use_hw_queues(); b = f.use_hw_queues(8, force=True); "
            "print(a, b, os.environ['GPU_MAX_HW_QUEUES'])")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["4", "8", "8"], out.stdout + out.stderr


def test_cli_hw_queues_honours_env_and_validates():
    """The CLI forces FM_HW_QUEUES when it is set (validated to HIP's 1..32); otherwise an exported
    GPU_MAX_HW_QUEUES is honoured and 8 is only the default."""
    from find_motion_amd.cli import hw_queues_from_env
    assert hw_queues_from_env({}) == (8, False)
    assert hw_queues_from_env({"GPU_MAX_HW_QUEUES": "4"}) == (8, False)  # use_hw_queues keeps the 4
    assert hw_queues_from_env({"FM_HW_QUEUES": "16", "GPU_MAX_HW_QUEUES": "4"}) == (16, True)
    for bad in ("abc", "0", "33", "-1"):
        with pytest.raises(SystemExit, match="FM_HW_QUEUES"):
            hw_queues_from_env({"FM_HW_QUEUES": bad})
        # an exported GPU_MAX_HW_QUEUES is kept only when HIP would accept it
        with pytest.raises(SystemExit, match="GPU_MAX_HW_QUEUES"):
            hw_queues_from_env({"GPU_MAX_HW_QUEUES": bad})
