/*
 * fm_oracle.c — CPU restatement of the per-frame motion chain of find_motion.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the MI355X
 * HIP path in find_motion_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * PARITY STATUS: "parity unpinned" by the reference itself.  The reference
 * (find_motion/find_motion.py) has no tests, no fixtures and no golden data,
 * and the library that holds the arithmetic (opencv-python, unpinned,
 * requirements.txt:4) is not installed in this image.  Every function below
 * restates the OpenCV 4.x CPU semantics of one call site of the reference and
 * is pinned by analytic known-answer tests (tests/test_oracle_kat.py) and by
 * an independent numpy/scipy restatement (oracle/oracle_np.py).
 *
 * Call sites restated (reference = /root/reference/find_motion/find_motion.py):
 *   fmo_resize_area_bgr     imutils.resize(raw, width=box) -> cv2.resize(INTER_AREA)   fm.py:492
 *   fmo_bgr2gray            cv2.cvtColor(small, COLOR_BGR2GRAY)                        fm.py:493
 *   fmo_gauss_coeffs/_blur  cv2.GaussianBlur(gray, (k,k), 0)                            fm.py:494, k from fm.py:478-484
 *   (mask)                  cv2.rectangle / cv2.fillConvexPoly on blur                  fm.py:619-636
 *   fmo_diff_thresh         absdiff(blur, convertScaleAbs(ref)) ; threshold(BINARY)     fm.py:246-257
 *   fmo_accumulate          cv2.accumulateWeighted(blur, ref, avg)                      fm.py:659
 *   fmo_dilate5             cv2.dilate(thresh, None, iterations=2)                      fm.py:266
 *   fmo_find_contours_ext   cv2.findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)        fm.py:269-272
 *   fmo_process_frame       the find_diff() ordering: init, diff, thresh, accumulate,
 *                           dilate, contours                                             fm.py:638-662
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------- */
/* cvRound (round half to even, the SSE cvtsd2si default) for doubles/floats */
static inline int rne_d(double v) { return (int)nearbyint(v); }
static inline int rne_f(float v) { return (int)nearbyintf(v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* BORDER_REFLECT_101 index mapping (OpenCV borderInterpolate). */
int fmo_reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p - 1 + 1;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* ------------------------------------------------------------------------- */
/* INTER_AREA resize (A1/A2).  dsize given => inv = d/s, scale = 1/inv.       */
typedef struct { int di, si; float alpha; } area_tab_t;

static int area_tab(int ssize, int dsize, double scale, area_tab_t* tab)
{
    int k = 0;
    for (int dx = 0; dx < dsize; dx++) {
        double fsx1 = dx * scale;
        double fsx2 = fsx1 + scale;
        double cellWidth = fmin(scale, ssize - fsx1);
        int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
        if (sx2 > ssize - 1) sx2 = ssize - 1;
        if (sx1 > sx2) sx1 = sx2;
        if (sx1 - fsx1 > 1e-3) {
            tab[k].di = dx; tab[k].si = sx1 - 1;
            tab[k++].alpha = (float)((sx1 - fsx1) / cellWidth);
        }
        for (int sx = sx1; sx < sx2; sx++) {
            tab[k].di = dx; tab[k].si = sx;
            tab[k++].alpha = (float)(1.0 / cellWidth);
        }
        if (fsx2 - sx2 > 1e-3) {
            tab[k].di = dx; tab[k].si = sx2;
            tab[k++].alpha = (float)(fmin(fmin(fsx2 - sx2, 1.), cellWidth) / cellWidth);
        }
    }
    return k;
}

/* Exported for tests: number of tab entries for (ssize -> dsize). */
int fmo_area_tab_size(int ssize, int dsize)
{
    double inv = (double)dsize / ssize, scale = 1. / inv;
    area_tab_t* t = (area_tab_t*)malloc(sizeof(area_tab_t) * (size_t)ssize * 2);
    int n = area_tab(ssize, dsize, scale, t);
    free(t);
    return n;
}

/* imutils.resize width rule: h = int(H * (box / float(W))). */
int fmo_work_height(int H, int W, int box)
{
    double r = (double)box / (double)W;
    return (int)(H * r);
}

/* Returns 0 ok, -1 unsupported (upscaling => OpenCV falls back to bilinear). */
int fmo_resize_area_bgr(const uint8_t* src, int H, int W, uint8_t* dst, int h, int w)
{
    const int cn = 3;
    if (h == H && w == W) { memcpy(dst, src, (size_t)H * W * cn); return 0; }
    double inv_x = (double)w / W, inv_y = (double)h / H;
    double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
    if (!(scale_x >= 1 && scale_y >= 1)) return -1;
    int isx = (int)lrint(scale_x), isy = (int)lrint(scale_y);
    int fast = fabs(scale_x - isx) < 2.220446049250313e-16 && fabs(scale_y - isy) < 2.220446049250313e-16;
    if (fast) {
        /* resizeAreaFast: integer box average. 2x2 => (sum+2)>>2; else cvRound(sum*(1.f/area)). */
        int area = isx * isy;
        float fscale = 1.f / (float)area;
        for (int dy = 0; dy < h; dy++)
            for (int dx = 0; dx < w; dx++)
                for (int c = 0; c < cn; c++) {
                    int sum = 0;
                    for (int yy = 0; yy < isy; yy++)
                        for (int xx = 0; xx < isx; xx++)
                            sum += src[((size_t)(dy * isy + yy) * W + (dx * isx + xx)) * cn + c];
                    int v = (isx == 2 && isy == 2) ? ((sum + 2) >> 2) : rne_f((float)sum * fscale);
                    dst[((size_t)dy * w + dx) * cn + c] = sat_u8(v);
                }
        return 0;
    }
    area_tab_t* xt = (area_tab_t*)malloc(sizeof(area_tab_t) * (size_t)W * 2);
    area_tab_t* yt = (area_tab_t*)malloc(sizeof(area_tab_t) * (size_t)H * 2);
    int nx = area_tab(W, w, scale_x, xt);
    int ny = area_tab(H, h, scale_y, yt);
    float* buf = (float*)malloc(sizeof(float) * (size_t)w * cn);
    float* sum = (float*)calloc((size_t)w * cn, sizeof(float));
    int prev_dy = yt[0].di;
    for (int j = 0; j < ny; j++) {
        float beta = yt[j].alpha;
        int dy = yt[j].di, sy = yt[j].si;
        const uint8_t* S = src + (size_t)sy * W * cn;
        for (int i = 0; i < w * cn; i++) buf[i] = 0.f;
        for (int k = 0; k < nx; k++) {
            int sxn = xt[k].si * cn, dxn = xt[k].di * cn;
            float a = xt[k].alpha;
            for (int c = 0; c < cn; c++) {
                volatile float prod = (float)S[sxn + c] * a; /* separate mul and add */
                buf[dxn + c] = buf[dxn + c] + prod;
            }
        }
        if (dy != prev_dy) {
            uint8_t* D = dst + (size_t)prev_dy * w * cn;
            for (int i = 0; i < w * cn; i++) {
                D[i] = sat_u8(rne_f(sum[i]));
                sum[i] = beta * buf[i];
            }
            prev_dy = dy;
        } else {
            for (int i = 0; i < w * cn; i++) {
                volatile float prod = beta * buf[i];
                sum[i] = sum[i] + prod;
            }
        }
    }
    uint8_t* D = dst + (size_t)prev_dy * w * cn;
    for (int i = 0; i < w * cn; i++) D[i] = sat_u8(rne_f(sum[i]));
    free(xt); free(yt); free(buf); free(sum);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* BGR2GRAY u8 (A3): (1868 B + 9617 G + 4899 R + 8192) >> 14                   */
void fmo_bgr2gray(const uint8_t* bgr, size_t n, uint8_t* gray)
{
    for (size_t i = 0; i < n; i++) {
        int b = bgr[3 * i], g = bgr[3 * i + 1], r = bgr[3 * i + 2];
        gray[i] = (uint8_t)((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14);
    }
}

/* ------------------------------------------------------------------------- */
/* GaussianBlur bit-exact fixed-point kernel (A4).                             */
/* Writes n coefficients (sum 256) into out.  Returns 0, or -1 if k even/<1.  */
int fmo_gauss_coeffs(int n, int32_t* out)
{
    if (n < 1 || (n & 1) == 0) return -1;
    double kd[512];
    if (n > 511) return -1;
    if (n == 1) { out[0] = 256; return 0; }
    static const double t3[] = {0.25, 0.5, 0.25};
    static const double t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
    static const double t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
    static const double t9[] = {4 / 256., 13 / 256., 30 / 256., 51 / 256., 60 / 256., 51 / 256., 30 / 256., 13 / 256., 4 / 256.};
    if (n == 3) memcpy(kd, t3, sizeof t3);
    else if (n == 5) memcpy(kd, t5, sizeof t5);
    else if (n == 7) memcpy(kd, t7, sizeof t7);
    else if (n == 9) memcpy(kd, t9, sizeof t9);
    else {
        double sigma = fma((double)n, 0.15, 0.35);          /* mulAdd(n, 0.15, 0.35) */
        double scale2X = -0.125 / (sigma * sigma);
        int n2 = (n - 1) / 2;
        double vals[256], sum = 0.0;
        for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
            double t = exp((double)(x * x) * scale2X);
            vals[i] = t;
            sum += t;
        }
        sum *= 2.0;
        sum += 1.0;
        for (int i = 0; i < n2; i++) {
            double t = vals[i] / sum;
            kd[i] = t; kd[n - 1 - i] = t;
        }
        kd[n2] = 1.0 / sum;
    }
    /* error-diffusion rounding to 8 fraction bits, outside in */
    int n2 = n / 2;
    double err = 0.0;
    int64_t s = 0;
    for (int i = 0; i < n2; i++) {
        double adj = kd[i] * 256.0 + err;
        int64_t v0 = (int64_t)nearbyint(adj);
        err = adj - (double)v0;
        out[i] = (int32_t)v0; out[n - 1 - i] = (int32_t)v0;
        s += v0;
    }
    s *= 2;
    out[n2] = (int32_t)(256 - s);
    return 0;
}

/* Separable fixed-point blur: out = (sum_y ky * (sum_x kx * p) + 2^15) >> 16, REFLECT_101. */
int fmo_gauss_blur(const uint8_t* src, int h, int w, int k, uint8_t* dst)
{
    int kx = k, ky = k;
    if (h == 1) ky = 1;
    if (w == 1) kx = 1;
    if (kx == 1 && ky == 1) { memcpy(dst, src, (size_t)h * w); return 0; }
    int32_t cx[512], cy[512];
    if (fmo_gauss_coeffs(kx, cx) || fmo_gauss_coeffs(ky, cy)) return -1;
    int rx = kx / 2, ry = ky / 2;
    uint32_t* H = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)h * w);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t acc = 0;
            for (int i = 0; i < kx; i++) acc += (uint32_t)cx[i] * src[(size_t)y * w + fmo_reflect101(x + i - rx, w)];
            H[(size_t)y * w + x] = acc;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t acc = 0;
            for (int i = 0; i < ky; i++) acc += (uint32_t)cy[i] * H[(size_t)fmo_reflect101(y + i - ry, h) * w + x];
            dst[(size_t)y * w + x] = (uint8_t)((acc + 32768u) >> 16);
        }
    free(H);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* convertScaleAbs(f64) + absdiff + threshold (A5, A10).                       */
/* AVX2 dispatch: continuous Mats are flattened; when the element count is    */
/* >= 16 every element takes the SIMD path (f64 -> f32 -> rne); a Mat with    */
/* fewer than 16 elements takes the scalar path (rne of the double).          */
void fmo_diff_thresh(const uint8_t* blur, const double* bg, size_t n, int thresh,
                     uint8_t* delta, uint8_t* th)
{
    int simd = n >= 16;
    for (size_t i = 0; i < n; i++) {
        int q = simd ? rne_f(fabsf((float)bg[i])) : rne_d(fabs(bg[i]));
        int d = abs((int)blur[i] - (int)sat_u8(q));
        if (delta) delta[i] = (uint8_t)d;
        th[i] = (d > thresh) ? 255 : 0;
    }
}

/* accumulateWeighted(u8 src, f64 dst, alpha) (A6): AVX2 vector body          */
/* dst = fma(dst, 1-a, src*a) over 16-element chunks, scalar tail             */
/* dst = src*a + dst*(1-a) (two roundings + add).                             */
void fmo_accumulate(const uint8_t* src, double* dst, size_t n, double alpha)
{
    double a = alpha, b = 1.0 - alpha;
    size_t vec_end = n - (n % 16);
    for (size_t i = 0; i < vec_end; i++) dst[i] = fma(dst[i], b, (double)src[i] * a);
    for (size_t i = vec_end; i < n; i++) {
        volatile double p1 = (double)src[i] * a;
        volatile double p2 = dst[i] * b;
        dst[i] = p1 + p2;
    }
}

/* ------------------------------------------------------------------------- */
/* dilate(None, iterations=2) == 5x5 rect max, out-of-image ignored (A7).      */
void fmo_dilate5(const uint8_t* src, int h, int w, uint8_t* dst)
{
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint8_t m = 0;
            for (int dy = -2; dy <= 2; dy++) {
                int yy = y + dy;
                if (yy < 0 || yy >= h) continue;
                for (int dx = -2; dx <= 2; dx++) {
                    int xx = x + dx;
                    if (xx < 0 || xx >= w) continue;
                    uint8_t v = src[(size_t)yy * w + xx];
                    if (v > m) m = v;
                }
            }
            dst[(size_t)y * w + x] = m;
        }
}

/* ------------------------------------------------------------------------- */
/* findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) (A8): literal restatement  */
/* of the legacy Suzuki-Abe scanner (cvFindNextContour, mode 0) and border    */
/* follower (icvFetchContour) on the 1-px zero-padded 0/1 image.              */
/* Per contour returns boundingRect (x,y,w,h), contourArea (|shoelace|), the  */
/* origin (start pixel) and the number of SIMPLE points.  Contours come out   */
/* in scan order of their start pixels.  Returns the count (may exceed cap:   */
/* only the first cap records are written).                                   */
static const int code_dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int code_dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

typedef struct {
    int minx, miny, maxx, maxy, npts;
    double a00;
    int fx, fy, px, py; /* first and previous point for shoelace */
} trace_acc_t;

static inline void acc_point(trace_acc_t* t, int x, int y)
{
    if (t->npts == 0) {
        t->fx = x; t->fy = y;
        t->minx = t->maxx = x; t->miny = t->maxy = y;
    } else {
        t->a00 += (double)t->px * y - (double)t->py * x;
        if (x < t->minx) t->minx = x;
        if (x > t->maxx) t->maxx = x;
        if (y < t->miny) t->miny = y;
        if (y > t->maxy) t->maxy = y;
    }
    t->px = x; t->py = y;
    t->npts++;
}

static void fetch_contour(int8_t* ptr, long step, int ox, int oy, trace_acc_t* acc,
                          int32_t* pts, int pts_cap)
{
    const int8_t nbd = 2;
    long deltas[16];
    deltas[0] = 1; deltas[1] = -step + 1; deltas[2] = -step; deltas[3] = -step - 1;
    deltas[4] = -1; deltas[5] = step - 1; deltas[6] = step; deltas[7] = step + 1;
    for (int i = 0; i < 8; i++) deltas[i + 8] = deltas[i];
    int8_t *i0 = ptr, *i1, *i3, *i4 = 0;
    int s, s_end, prev_s;
    int px = ox, py = oy;
    s_end = s = 4; /* outer border */
    do {
        s = (s - 1) & 7;
        i1 = i0 + deltas[s];
    } while (*i1 == 0 && s != s_end);
    if (s == s_end) { /* single pixel domain */
        *i0 = (int8_t)(nbd | -128);
        if (pts && acc->npts < pts_cap) { pts[2 * acc->npts] = px; pts[2 * acc->npts + 1] = py; }
        acc_point(acc, px, py);
        return;
    }
    i3 = i0;
    prev_s = s ^ 4;
    for (;;) {
        s_end = s;
        if (s > 15) s = 15; /* min(s, MAX_SIZE-1) */
        while (s < 15) {
            i4 = i3 + deltas[++s];
            if (*i4 != 0) break;
        }
        s &= 7;
        if ((unsigned)(s - 1) < (unsigned)s_end) *i3 = (int8_t)(nbd | -128);
        else if (*i3 == 1) *i3 = nbd;
        if (s != prev_s) { /* CHAIN_APPROX_SIMPLE: keep direction changes */
            if (pts && acc->npts < pts_cap) { pts[2 * acc->npts] = px; pts[2 * acc->npts + 1] = py; }
            acc_point(acc, px, py);
            prev_s = s;
        }
        px += code_dx[s];
        py += code_dy[s];
        if (i4 == i0 && i3 == i1) break;
        i3 = i4;
        s = (s + 4) & 7;
    }
}

/* out layout per contour (ints): x, y, w, h, origin_x, origin_y, npts.       */
int fmo_find_contours_ext(const uint8_t* img, int h, int w, int32_t* rec, double* areas,
                          int cap, int32_t* pts, int pts_cap_per_contour)
{
    int W = w + 2, H = h + 2;
    long step = W;
    int8_t* im = (int8_t*)calloc((size_t)W * H, 1);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) im[(size_t)(y + 1) * step + x + 1] = img[(size_t)y * w + x] ? 1 : 0;
    int width = W - 1, height = H - 1;
    int count = 0;
    int lnbd_x = 0, lnbd_y = 1;
    for (int y = 1; y < height; y++) {
        int8_t* row = im + (size_t)y * step;
        int prev = 0;
        lnbd_x = 0; lnbd_y = y;
        for (int x = 1; x < width; x++) {
            int p = row[x];
            if (p == prev) continue;
            int is_hole = 0;
            if (!(prev == 0 && p == 1)) {
                /* not an outer-border start: hole start needs p==0 && prev>=1 */
                if (p != 0 || prev < 1) goto resume;
                if (prev & -2) lnbd_x = x - 1;
                is_hole = 1;
            }
            /* RETR_EXTERNAL: skip holes and outer borders whose last-crossed
               border pixel is positive (an untraced/inner region) */
            if (is_hole || im[(size_t)lnbd_y * step + lnbd_x] > 0) goto resume;
            lnbd_x = x;
            {
                trace_acc_t acc;
                memset(&acc, 0, sizeof acc);
                int32_t* cp = (pts && count < cap) ? pts + (size_t)count * 2 * pts_cap_per_contour : 0;
                fetch_contour(row + x, step, x - 1, y - 1, &acc, cp, pts_cap_per_contour);
                /* close the shoelace polygon: last -> first */
                if (acc.npts > 0) acc.a00 += (double)acc.px * acc.fy - (double)acc.py * acc.fx;
                if (count < cap) {
                    int32_t* r = rec + (size_t)count * 7;
                    r[0] = acc.minx; r[1] = acc.miny;
                    r[2] = acc.maxx - acc.minx + 1; r[3] = acc.maxy - acc.miny + 1;
                    r[4] = x - 1; r[5] = y - 1; r[6] = acc.npts;
                    if (areas) areas[count] = fabs(acc.a00 * 0.5);
                }
                count++;
            }
            /* after a found contour the scan resumes at x+1 with prev = marked start pixel */
            prev = row[x];
            continue;
        resume:
            prev = p;
            if (prev & -2) lnbd_x = x;
        }
    }
    free(im);
    return count;
}

/* ------------------------------------------------------------------------- */
/* One find_motion frame step for one stream (fm.py:487-494, 619-636, 638-662)*/
typedef struct {
    int H, W;          /* source frame */
    int h, w;          /* work image (imutils rule) */
    int ksize;         /* odd Gaussian size (fm.py:478-484) */
    int thresh;        /* integer threshold (-t) */
    double alpha;      /* -a */
} fmo_cfg;

/* Any of gray/blur/delta/mask_out may be NULL.  bg must hold h*w doubles;    */
/* *bg_init is 0 before the first frame.  Returns contour count, <0 on error. */
int fmo_process_frame(const fmo_cfg* c, const uint8_t* bgr, const uint8_t* keep,
                      double* bg, int* bg_init,
                      uint8_t* gray_o, uint8_t* blur_o, uint8_t* delta_o, uint8_t* mask_o,
                      int32_t* rec, double* areas, int cap)
{
    size_t n = (size_t)c->h * c->w;
    uint8_t* small = (uint8_t*)malloc(n * 3);
    uint8_t* gray = gray_o ? gray_o : (uint8_t*)malloc(n);
    uint8_t* blur = blur_o ? blur_o : (uint8_t*)malloc(n);
    uint8_t* th = (uint8_t*)malloc(n);
    uint8_t* mask = mask_o ? mask_o : (uint8_t*)malloc(n);
    int rc = fmo_resize_area_bgr(bgr, c->H, c->W, small, c->h, c->w);
    if (rc == 0) {
        fmo_bgr2gray(small, n, gray);
        rc = fmo_gauss_blur(gray, c->h, c->w, c->ksize, blur);
    }
    if (rc == 0) {
        if (keep)
            for (size_t i = 0; i < n; i++) if (!keep[i]) blur[i] = 0;
        if (!*bg_init) { for (size_t i = 0; i < n; i++) bg[i] = (double)blur[i]; *bg_init = 1; }
        fmo_diff_thresh(blur, bg, n, c->thresh, delta_o, th);
        fmo_accumulate(blur, bg, n, c->alpha);
        fmo_dilate5(th, c->h, c->w, mask);
        rc = fmo_find_contours_ext(mask, c->h, c->w, rec, areas, cap, 0, 0);
    }
    free(small); free(th);
    if (!gray_o) free(gray);
    if (!blur_o) free(blur);
    if (!mask_o) free(mask);
    return rc;
}

/* CPU baseline: S independent streams x F frames, one OpenMP thread per      */
/* stream (mirrors run_pool's one-video-per-worker, fm.py:1071-1075).          */
/* frames layout [S][F][H][W][3], or [F][H][W][3] shared by every stream when  */
/* shared != 0; counts [S][F].  Returns threads used.                         */
int fmo_run_streams(const fmo_cfg* c, const uint8_t* frames, int S, int F, int nthreads,
                    int32_t* counts, int shared)
{
    int used = 1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
    }
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int s = 0; s < S; s++) {
        size_t n = (size_t)c->h * c->w;
        double* bg = (double*)malloc(n * sizeof(double));
        int init = 0;
        int32_t rec[7 * 64];
        for (int f = 0; f < F; f++) {
            const uint8_t* fr = frames + ((size_t)(shared ? 0 : s) * F + f) * (size_t)c->H * c->W * 3;
            counts[(size_t)s * F + f] = fmo_process_frame(c, fr, 0, bg, &init, 0, 0, 0, 0, rec, 0, 64);
        }
        free(bg);
    }
    return used;
}

/* ------------------------------------------------------------------------- */
/* fmo_process_sequence: fmo_process_frame over F consecutive frames of one   */
/* stream, scheduled in parallel where find_diff's data flow allows it, with  */
/* the identical arithmetic per pixel (so it is checked against              */
/* fmo_process_frame by tests/test_oracle_kat.py):                            */
/*   blur_frame + mask (fm.py:487-494, 619-636): frames are independent;      */
/*   diff / threshold / accumulateWeighted (fm.py:246-257, 651-659): a        */
/*     recurrence over frames but independent per pixel (each pixel keeps     */
/*     fmo_diff_thresh's SIMD rule and fmo_accumulate's frame-global vector-  */
/*     body / scalar-tail split);                                            */
/*   dilate + findContours (fm.py:260-276): frames are independent.           */
/* masks: NULL or [F] pointers (NULL entries: mask not kept).                 */
/* rec: [F][cap][7] as fmo_find_contours_ext, areas [F][cap] or NULL.         */
/* Returns 0, or -1 when a frame's resize/blur is unsupported.                */
int fmo_process_sequence(const fmo_cfg* c, const uint8_t* frames, int F, const uint8_t* keep,
                         double* bg, int* bg_init, uint8_t* const* masks, int32_t* counts,
                         int32_t* rec, double* areas, int cap, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const size_t n = (size_t)c->h * c->w, fb = (size_t)c->H * c->W * 3;
    const int CH = 32;
    const int simd = n >= 16;
    const size_t vec_end = n - (n % 16);
    const double a = c->alpha, b = 1.0 - c->alpha;
    uint8_t* blur = (uint8_t*)malloc(n * CH);
    uint8_t* th = (uint8_t*)malloc(n * CH);
    int bad = 0;
    for (int f0 = 0; f0 < F; f0 += CH) {
        const int nf = F - f0 < CH ? F - f0 : CH;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(| : bad)
#endif
        for (int j = 0; j < nf; j++) {
            uint8_t* small = (uint8_t*)malloc(n * 3);
            uint8_t* gray = (uint8_t*)malloc(n);
            uint8_t* bl = blur + (size_t)j * n;
            int rc = fmo_resize_area_bgr(frames + (size_t)(f0 + j) * fb, c->H, c->W, small, c->h, c->w);
            if (rc == 0) {
                fmo_bgr2gray(small, n, gray);
                rc = fmo_gauss_blur(gray, c->h, c->w, c->ksize, bl);
            }
            if (rc) bad |= 1;
            if (keep)
                for (size_t i = 0; i < n; i++) if (!keep[i]) bl[i] = 0;
            free(small); free(gray);
        }
        if (bad) break;
        const int init0 = *bg_init;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (long blk = 0; blk < (long)((n + 4095) / 4096); blk++) {
            const size_t i0 = (size_t)blk * 4096, i1 = i0 + 4096 < n ? i0 + 4096 : n;
            for (size_t i = i0; i < i1; i++) {
                double v = bg[i];
                for (int j = 0; j < nf; j++) {
                    const uint8_t s = blur[(size_t)j * n + i];
                    if (!init0 && j == 0) v = (double)s;
                    const int q = simd ? rne_f(fabsf((float)v)) : rne_d(fabs(v));
                    const int d = abs((int)s - (int)sat_u8(q));
                    th[(size_t)j * n + i] = (d > c->thresh) ? 255 : 0;
                    if (i < vec_end) {
                        v = fma(v, b, (double)s * a);
                    } else {
                        volatile double p1 = (double)s * a;
                        volatile double p2 = v * b;
                        v = p1 + p2;
                    }
                }
                bg[i] = v;
            }
        }
        *bg_init = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
        for (int j = 0; j < nf; j++) {
            const int f = f0 + j;
            uint8_t* m = (masks && masks[f]) ? masks[f] : (uint8_t*)malloc(n);
            fmo_dilate5(th + (size_t)j * n, c->h, c->w, m);
            counts[f] = fmo_find_contours_ext(m, c->h, c->w, rec + (size_t)f * cap * 7, areas ? areas + (size_t)f * cap : 0,
                                              cap, 0, 0);
            if (!(masks && masks[f])) free(m);
        }
    }
    free(blur); free(th);
    return bad ? -1 : 0;
}
