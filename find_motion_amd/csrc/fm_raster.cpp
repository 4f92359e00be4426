// fm_raster.cpp — host rasteriser for mask_off_areas (fm.py:611-636).
//
// The reference draws every mask polygon onto frame.blur in every frame:
//   2 points  -> cv2.rectangle(blur, p0, p1, BLACK, cv2.FILLED)   fm.py:627-630
//   >= 3      -> cv2.fillConvexPoly(blur, pts, BLACK)              fm.py:632-635
// after scaling each point by int(v * scale) (scale_area, fm.py:611-616).
// Drawing 0 does not depend on the image, so the union of the polygons is
// rasterised once per video into a keep-mask that the pixel kernel applies.
//
// OpenCV's FILLED rectangle is FillConvexPoly over its four corners, so both
// go through the restatement of imgproc drawing.cpp FillConvexPoly (shift 0,
// LINE_8): every edge drawn with the 8-connected Bresenham LineIterator
// (clipped by clipLine), then a scanline fill between the two active edges
// in 16.16 fixed point.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/find_motion_amd.h"

namespace {

constexpr int XY_SHIFT = 16;
constexpr int64_t XY_ONE = 1ll << XY_SHIFT;

struct P64 {
    int64_t x, y;
};

struct Canvas {
    uint8_t* img;
    int w, h;
    void hline(int x1, int x2, int y) {
        for (int x = x1; x <= x2; x++) img[(size_t)y * w + x] = 0;
    }
};

bool clip_line(int64_t width, int64_t height, P64& a, P64& b) {
    const int64_t right = width - 1, bottom = height - 1;
    if (width <= 0 || height <= 0) return false;
    int64_t &x1 = a.x, &y1 = a.y, &x2 = b.x, &y2 = b.y;
    int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        int64_t t;
        if (c1 & 12) {
            t = c1 < 8 ? 0 : bottom;
            x1 += (int64_t)((double)(t - y1) * (x2 - x1) / (y2 - y1));
            y1 = t;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            t = c2 < 8 ? 0 : bottom;
            x2 += (int64_t)((double)(t - y2) * (x2 - x1) / (y2 - y1));
            y2 = t;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                t = c1 == 1 ? 0 : right;
                y1 += (int64_t)((double)(t - x1) * (y2 - y1) / (x2 - x1));
                x1 = t;
                c1 = 0;
            }
            if (c2) {
                t = c2 == 1 ? 0 : right;
                y2 += (int64_t)((double)(t - x2) * (y2 - y1) / (x2 - x1));
                x2 = t;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

// cv::Line with LINE_8: LineIterator(img, pt1, pt2, 8, leftToRight = true).
void draw_line(Canvas& cv, P64 p1, P64 p2) {
    if ((uint64_t)p1.x >= (uint64_t)cv.w || (uint64_t)p2.x >= (uint64_t)cv.w || (uint64_t)p1.y >= (uint64_t)cv.h ||
        (uint64_t)p2.y >= (uint64_t)cv.h) {
        if (!clip_line(cv.w, cv.h, p1, p2)) return;
    }
    int64_t dx = p2.x - p1.x, dy = p2.y - p1.y;
    int sx = 1, sy = 1;
    if (dx < 0) {  // leftToRight: swap the end points
        dx = -dx;
        dy = -dy;
        std::swap(p1, p2);
    }
    if (dy < 0) {
        dy = -dy;
        sy = -1;
    }
    const bool vert = dy > dx;
    if (vert) {
        std::swap(dx, dy);
        std::swap(sx, sy);
    }
    // connectivity 8
    int64_t err = dx - (dy + dy);
    const int64_t plusDelta = dx + dx, minusDelta = -(dy + dy);
    int minusShift = sx, plusShift = 0, minusStep = 0, plusStep = sy;
    const int64_t count = dx + 1;
    if (vert) {
        std::swap(plusStep, plusShift);
        std::swap(minusStep, minusShift);
    }
    int64_t x = p1.x, y = p1.y;
    for (int64_t i = 0; i < count; i++) {
        cv.img[(size_t)y * cv.w + x] = 0;
        const int64_t m = err < 0 ? -1 : 0;
        err += minusDelta + (plusDelta & m);
        x += minusShift + (plusShift & m);
        y += minusStep + (plusStep & m);
    }
}

void fill_convex_poly(Canvas& cv, const std::vector<P64>& v) {
    const int npts = (int)v.size();
    if (npts <= 0) return;
    struct Edge {
        int idx, di;
        int64_t x, dx;
        int ye;
    } edge[2];
    const int shift = 0;
    const int delta = 1 << shift >> 1;  // 0
    const int64_t delta1 = XY_ONE >> 1, delta2 = XY_ONE >> 1;
    int imin = 0, edges = npts;
    int64_t xmin = v[0].x, xmax = v[0].x, ymin = v[0].y, ymax = v[0].y;
    P64 p0 = v[npts - 1];
    p0.x <<= XY_SHIFT - shift;
    p0.y <<= XY_SHIFT - shift;
    for (int i = 0; i < npts; i++) {
        P64 p = v[i];
        if (p.y < ymin) {
            ymin = p.y;
            imin = i;
        }
        ymax = std::max(ymax, p.y);
        xmax = std::max(xmax, p.x);
        xmin = std::min(xmin, p.x);
        p.x <<= XY_SHIFT - shift;
        p.y <<= XY_SHIFT - shift;
        draw_line(cv, {p0.x >> XY_SHIFT, p0.y >> XY_SHIFT}, {p.x >> XY_SHIFT, p.y >> XY_SHIFT});
        p0 = p;
    }
    xmin = (xmin + delta) >> shift;
    xmax = (xmax + delta) >> shift;
    ymin = (ymin + delta) >> shift;
    ymax = (ymax + delta) >> shift;
    if (npts < 3 || (int)xmax < 0 || (int)ymax < 0 || (int)xmin >= cv.w || (int)ymin >= cv.h) return;
    ymax = std::min<int64_t>(ymax, cv.h - 1);
    edge[0].idx = edge[1].idx = imin;
    int y = (int)ymin;
    edge[0].ye = edge[1].ye = y;
    edge[0].di = 1;
    edge[1].di = npts - 1;
    edge[0].x = edge[1].x = -XY_ONE;
    edge[0].dx = edge[1].dx = 0;
    do {
        for (int i = 0; i < 2; i++) {
            if (y >= edge[i].ye) {
                int idx0 = edge[i].idx, di = edge[i].di;
                int idx = idx0 + di;
                if (idx >= npts) idx -= npts;
                int ty = 0;
                for (; edges-- > 0;) {
                    ty = (int)((v[idx].y + delta) >> shift);
                    if (ty > y) {
                        int64_t xs = v[idx0].x, xe = v[idx].x;
                        xs <<= XY_SHIFT - shift;
                        xe <<= XY_SHIFT - shift;
                        edge[i].ye = ty;
                        edge[i].dx = ((xe - xs) * 2 + ((int64_t)ty - y)) / (2 * ((int64_t)ty - y));
                        edge[i].x = xs;
                        edge[i].idx = idx;
                        break;
                    }
                    idx0 = idx;
                    idx += di;
                    if (idx >= npts) idx -= npts;
                }
            }
        }
        if (edges < 0) break;
        if (y >= 0) {
            int left = 0, right = 1;
            if (edge[0].x > edge[1].x) {
                left = 1;
                right = 0;
            }
            int xx1 = (int)((edge[left].x + delta1) >> XY_SHIFT);
            int xx2 = (int)((edge[right].x + delta2) >> XY_SHIFT);
            if (xx2 >= 0 && xx1 < cv.w) {
                if (xx1 < 0) xx1 = 0;
                if (xx2 >= cv.w) xx2 = cv.w - 1;
                cv.hline(xx1, xx2, y);
            }
        }
        edge[0].x += edge[0].dx;
        edge[1].x += edge[1].dx;
    } while (++y <= (int)ymax);
}

}  // namespace

extern "C" int fm_rasterize_masks(int h, int w, double scale, const int32_t* xy, const int32_t* npts, int n_polys,
                                  uint8_t* keep) {
    if (h < 1 || w < 1 || !keep || n_polys < 0 || (n_polys > 0 && (!xy || !npts))) return FM_EINVAL;
    std::memset(keep, 1, (size_t)h * w);
    Canvas cv{keep, w, h};
    size_t off = 0;
    for (int i = 0; i < n_polys; i++) {
        const int n = npts[i];
        if (n < 2) return FM_EINVAL;
        std::vector<P64> pts(n);
        for (int j = 0; j < n; j++) {
            // scale_area: int(a * scale) truncates toward zero
            pts[j].x = (int64_t)(int)((double)xy[2 * (off + j)] * scale);
            pts[j].y = (int64_t)(int)((double)xy[2 * (off + j) + 1] * scale);
        }
        off += n;
        if (n == 2) {
            const P64 a = pts[0], b = pts[1];
            std::vector<P64> r = {a, {b.x, a.y}, b, {a.x, b.y}};
            fill_convex_poly(cv, r);
        } else {
            fill_convex_poly(cv, pts);
        }
    }
    return FM_OK;
}
