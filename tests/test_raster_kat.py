"""Known answers for the mask rasteriser without cv2 (mask_off_areas, fm.py:611-636).

fm_rasterize_masks restates OpenCV's FillConvexPoly (imgproc drawing.cpp, shift 0, LINE_8):
every edge drawn by the 8-connected LineIterator (left to right, clipped), then a
scanline fill between the two active edges in 16.16 fixed point.  OpenCV itself is
not importable here, so these pin the restatement by properties that hold for that
rule independently of how it is coded:

* an axis-aligned box given as four points fills exactly the inclusive box,
  clipped to the image (the two-point form is cv2.rectangle FILLED, fm.py:627-630);
* 45-degree right triangles in all four orientations fill exactly a half-square
  (the Bresenham diagonal and the fixed-point DDA are both exact at slope 1);
* the LINE_8 iterator picks, on each column of an x-major edge, the pixel nearest
  the ideal line with ties toward the start point: y - y0 = ceil(k*dy/dx - 1/2)
  (checked against a literal re-run of the iterator below, then used as the known
  answer for the config-5 triangle's hypotenuse, find_motion.py:86-100);
* the fill is invariant under rotating the vertex list (and reversing it, while
  no edge is clipped), contains
  every lattice point strictly inside the polygon, and never reaches a pixel
  farther than one pixel (L-inf) from it.
No GPU needed.
"""
import numpy as np
import pytest

from find_motion_amd import _native


def masked(h, w, polys, scale=1.0):
    return _native.rasterize_masks(h, w, scale, polys) == 0


@pytest.mark.parametrize("box,size", [(((2, 3), (9, 7)), (12, 14)), (((-5, -2), (6, 4)), (10, 10)),
                                      (((3, 4), (20, 30)), (8, 9)), (((0, 0), (0, 0)), (3, 3))])
def test_axis_box_four_points_is_inclusive_box_clipped(box, size):
    (x0, y0), (x1, y1) = box
    h, w = size
    want = np.zeros((h, w), bool)
    want[max(y0, 0):max(min(y1, h - 1) + 1, 0), max(x0, 0):max(min(x1, w - 1) + 1, 0)] = True
    quad = [(x0, y0), (x1, y0), (x1, y1), (x0, y1)]
    np.testing.assert_array_equal(masked(h, w, [quad]), want)
    np.testing.assert_array_equal(masked(h, w, [[(x0, y0), (x1, y1)]]), want)  # cv2.rectangle FILLED


@pytest.mark.parametrize("n", [1, 4, 9])
def test_diagonal_triangles_four_orientations(n):
    h = w = n + 3
    yy, xx = np.mgrid[:h, :w]
    inside = (xx <= n) & (yy <= n)
    cases = {
        ((0, 0), (n, n), (0, n)): (xx <= yy),            # below the main diagonal
        ((0, 0), (n, 0), (n, n)): (xx >= yy),            # above it
        ((n, 0), (n, n), (0, n)): (xx + yy >= n),        # below the anti-diagonal
        ((0, 0), (n, 0), (0, n)): (xx + yy <= n),        # above it
    }
    for tri, want in cases.items():
        np.testing.assert_array_equal(masked(h, w, [list(tri)]), want & inside, err_msg=str(tri))


def _line8(p, q):
    """OpenCV LineIterator(connectivity 8, leftToRight) re-run literally: every step moves one pixel along
    the major axis and one along the minor axis when err < 0 (err = dx - 2dy, += 2dx - 2dy or -2dy)."""
    if q[0] < p[0]:
        p, q = q, p
    (x0, y0), (x1, y1) = p, q
    dx, dy = x1 - x0, y1 - y0
    sy = 1 if dy >= 0 else -1
    dy = abs(dy)
    vert = dy > dx
    if vert:
        dx, dy = dy, dx
    err, out, x, y = dx - 2 * dy, [], x0, y0
    for _ in range(dx + 1):
        out.append((x, y))
        plus = err < 0
        err += -2 * dy + (2 * dx if plus else 0)
        if vert:
            x, y = x + (1 if plus else 0), y + sy
        else:
            x, y = x + 1, y + (sy if plus else 0)
    return out


@pytest.mark.parametrize("dx,dy", [(639, -559), (7, 3), (10, 5), (13, -13), (40, 1), (5, 0)])
def test_line8_is_nearest_pixel_ties_to_start(dx, dy):
    x0, y0 = 100, 600
    pts = _line8((x0, y0), (x0 + dx, y0 + dy))
    s = 1 if dy >= 0 else -1
    ady = abs(dy)
    want = [(x0 + k, y0 + s * -((-(2 * k * ady - dx)) // (2 * dx))) for k in range(dx + 1)]  # ceil(k dy/dx - 1/2)
    assert pts == want


def test_config5_triangle_edges_and_rows():
    """MASK_SCHEMA triangle (3839,2159), (3200,2159), (3839,1600) at 4K, scale 1 (find_motion.py:86-100):
    its hypotenuse pixels are the nearest-pixel line (ties to the left end), the right and bottom edges
    are the image border, and every row's masked span runs from the hypotenuse to x = 3839."""
    H, W = 2160, 3840
    m = masked(H, W, [[(3839, 2159), (3200, 2159), (3839, 1600)]])
    dx, dy = 639, 559  # left end (3200, 2159) -> (3839, 1600): y decreases
    hyp = [(3200 + k, 2159 + -((-(2 * k * dy - dx)) // (2 * dx)) * -1) for k in range(dx + 1)]
    assert all(m[y, x] for x, y in hyp)
    assert hyp[0] == (3200, 2159) and hyp[-1] == (3839, 1600)
    # known answers: first pixels of the line and the leftmost masked column of some rows
    assert hyp[:6] == [(3200, 2159), (3201, 2158), (3202, 2157), (3203, 2156), (3204, 2156), (3205, 2155)]
    left = {y: int(np.argmax(m[y])) for y in (1600, 1601, 1700, 1879, 1880, 2000, 2158, 2159)}
    assert left == {1600: 3839, 1601: 3838, 1700: 3725, 1879: 3520, 1880: 3519, 2000: 3382, 2158: 3201, 2159: 3200}
    first = {}
    for x, y in hyp:
        first[y] = min(first.get(y, x), x)
    for y in range(1600, 2160):  # contiguous spans from the hypotenuse to the right border
        xs = np.flatnonzero(m[y])
        assert xs[0] == first[y] and xs[-1] == 3839 and len(xs) == 3840 - xs[0], y
    assert not m[:1600].any() and m.sum() == sum(3840 - left_x for left_x in
                                                 (int(np.argmax(m[y])) for y in range(1600, 2160)))


def _convex_polys(rng, n, vmin=-6, vmax=46):
    out = []
    while len(out) < n:
        pts = rng.integers(vmin, vmax, (12, 2))
        # convex hull (monotone chain), counter-clockwise in image coordinates
        pts = sorted(set(map(tuple, pts.tolist())))
        if len(pts) < 3:
            continue

        def cross(o, a, b):
            return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])

        lo, hi = [], []
        for p in pts:
            while len(lo) >= 2 and cross(lo[-2], lo[-1], p) <= 0:
                lo.pop()
            lo.append(p)
        for p in reversed(pts):
            while len(hi) >= 2 and cross(hi[-2], hi[-1], p) <= 0:
                hi.pop()
            hi.append(p)
        hull = lo[:-1] + hi[:-1]
        if len(hull) >= 3:
            out.append(hull)
    return out


def test_convex_polygons_rotation_reversal_inside_and_tight():
    rng = np.random.default_rng(7)
    H, W = 40, 40
    yy, xx = np.mgrid[:H, :W]
    polys = _convex_polys(rng, 60) + _convex_polys(rng, 60, 0, 40)  # clipped ones, then inside the image
    assert sum(all(0 <= c < 40 for pt in p for c in pt) for p in polys) >= 60
    for poly in polys:
        base = masked(H, W, [poly])
        # clipLine cuts an edge from its first end point, so a reversed vertex list is the same fill only
        # while no edge needs clipping
        inside_img = all(0 <= x < W and 0 <= y < H for x, y in poly)
        for r in range(len(poly)):
            rot = poly[r:] + poly[:r]
            np.testing.assert_array_equal(masked(H, W, [rot]), base, err_msg=f"rotation {r} of {poly}")
            if inside_img:
                np.testing.assert_array_equal(masked(H, W, [rot[::-1]]), base, err_msg=f"reversal of {rot}")
        # strictly inside (all edge cross products of one sign) -> filled
        P = np.array(poly, np.int64)
        Q = np.roll(P, -1, axis=0)
        cr = np.stack([(q[0] - p[0]) * (yy - p[1]) - (q[1] - p[1]) * (xx - p[0]) for p, q in zip(P, Q)])
        strict = (cr > 0).all(0) | (cr < 0).all(0)
        assert base[strict].all(), poly
        # filled -> within one pixel (L-inf) of the closed polygon: some point of the 3x3 square around it
        # is inside or on the polygon
        near = np.zeros_like(strict)
        for ddy in (-1, 0, 1):
            for ddx in (-1, 0, 1):
                c2 = np.stack([(q[0] - p[0]) * (yy + ddy - p[1]) - (q[1] - p[1]) * (xx + ddx - p[0])
                               for p, q in zip(P, Q)])
                near |= (c2 >= 0).all(0) | (c2 <= 0).all(0)
        assert not (base & ~near).any(), poly
