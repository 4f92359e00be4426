// fm_jpeg.hip — the decode side of the path: MJPEG frames decoded on the GPU.
//
// The reference reads frames with cv2.VideoCapture.read (fm.py:413, 497-506).  For MJPEG video each
// frame is a baseline JPEG; this decoder reproduces libjpeg-turbo's default decode (what OpenCV and
// Pillow call) bit for bit -- pinned against Pillow's libjpeg-turbo by tests/test_jpeg_host.py (CPU
// restatement oracle/jpeg.py) and tests/test_gpu_jpeg.py (this code):
//   host    marker segments (DQT, DHT, SOF0/1, DRI, SOS) parsed per frame; the entropy-coded bytes
//           copied into one pinned buffer with byte stuffing and RSTn markers removed, one segment
//           per restart interval (the whole scan without DRI);
//   k_jpeg_huff   one lane per segment: Huffman decode (9-bit lookahead tables in LDS, canonical slow
//           path past 9 bits), DC prediction, zigzag -> natural order; quantized coefficients scattered
//           (non-zeros only) into a zeroed int16 coefficient buffer [frame][component][block][64];
//   k_jpeg_idct   8 lanes per block: dequantize + jpeg_idct_islow (jidctint.c: CONST_BITS 13,
//           PASS1_BITS 2, zero-column / zero-row shortcuts, IDCT range-limit table) into component
//           planes; the block's coefficients are zeroed again for the next call;
//   k_jpeg_color  one thread per 4 output pixels: fancy upsampling (jdsample.c h2v1/h2v2 with the
//           edge-replicated context rows of jdmainct.c) and ycc_rgb_convert (jdcolor.c tables) ->
//           BGR u8 HWC, the cv2.VideoCapture layout, straight into the caller's frame buffer.
// Supported: 8-bit baseline / extended-sequential Huffman, grayscale or 3-component YCbCr with
// Cb, Cr at 1x1 and Y at 1x1, 2x1 or 2x2; restart intervals optional.  Anything else: FM_ENOTSUP.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fm_internal.h"

namespace fm {
namespace jp {

constexpr int kMaxComp = 3;

struct HuffDev {              // one table as the decoder reads it (LDS image)
    uint16_t lut[512];        // 9-bit lookahead: (length << 8) | symbol, 0 = longer code
    int32_t maxcode[18];      // largest code of each length (-1: none), [17] sentinel
    int32_t valoff[18];       // index into vals of code c of length l: valoff[l] + c
    uint8_t vals[256];
};

struct CompDev {
    int dc, ac;               // Huffman table slots (0..3) of this component
    int h, v;                 // sampling factors
    int bw, bh;               // coefficient grid of one frame (blocks, MCU-padded)
    long long coef0;          // block offset of frame 0's plane in the coefficient buffer
    long long plane0;         // byte offset of frame 0's sample plane
};

struct JpegGeom {
    int W, H, nc, hmax, vmax, mcux, mcuy, interleaved;
    long long frame_blocks;   // coefficient blocks per frame (all components)
    long long frame_plane;    // sample-plane bytes per frame (all components)
    CompDev comp[kMaxComp];
};

struct Seg {
    uint32_t off;             // byte offset of the segment's unstuffed data in the stream buffer
    uint32_t len;
    int32_t frame;            // frame of the call (0..n-1)
    int32_t mcu0, nmcu;       // MCUs the segment holds
};

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

__constant__ uint8_t c_zigzag[80] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                     12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                     35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                     58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                                     // k past 63 (corrupt runs): a harmless slot, as libjpeg's
                                     // jpeg_natural_order extra entries
                                     63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct BitReader {
    const uint32_t* w;
    const uint32_t* lim;
    uint64_t acc;
    int nb;
    __device__ __forceinline__ void init(const uint8_t* base, uint32_t off, const uint8_t* end) {
        w = reinterpret_cast<const uint32_t*>(base + (off & ~3u));
        lim = reinterpret_cast<const uint32_t*>(end);
        acc = 0;
        nb = 0;
        refill();
        const int skip = (int)(off & 3u) * 8;
        acc <<= skip;
        nb -= skip;
        refill();
    }
    __device__ __forceinline__ void refill() {
        while (nb <= 32) {
            const uint32_t v = w < lim ? bswap32(*w) : 0u;
            w++;
            acc |= (uint64_t)v << (32 - nb);
            nb += 32;
        }
    }
    __device__ __forceinline__ uint32_t peek(int n) const { return (uint32_t)(acc >> (64 - n)); }
    __device__ __forceinline__ void skip(int n) {
        acc <<= n;
        nb -= n;
    }
    __device__ __forceinline__ int get(int n) {  // n in [0, 16]
        if (n == 0) return 0;
        const int v = (int)peek(n);
        skip(n);
        return v;
    }
};

__device__ __forceinline__ int huff_decode(BitReader& br, const HuffDev& t) {
    br.refill();
    const uint32_t e = t.lut[br.peek(9)];
    if (e) {
        br.skip((int)(e >> 8));
        return (int)(e & 0xFF);
    }
    const uint32_t c16 = br.peek(16);
    for (int l = 10; l <= 16; l++) {
        const int code = (int)(c16 >> (16 - l));
        if (code <= t.maxcode[l]) {
            br.skip(l);
            return t.vals[(t.valoff[l] + code) & 0xFF];
        }
    }
    br.skip(16);  // not a code: corrupt data (libjpeg warns and returns 0)
    return 0;
}

__device__ __forceinline__ int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

// one lane per segment; one wave per workgroup (the Huffman tables of this call in LDS)
__global__ __launch_bounds__(64) void k_jpeg_huff(const uint8_t* __restrict__ stream, uint32_t stream_len,
                                                   const Seg* __restrict__ segs, int nseg, const HuffDev* __restrict__ tabs,
                                                   JpegGeom g, int16_t* __restrict__ coef) {
    __shared__ HuffDev T[4];
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(tabs);
        uint32_t* dst = reinterpret_cast<uint32_t*>(T);
        for (int i = threadIdx.x; i < (int)(sizeof(T) / 4); i += 64) dst[i] = src[i];
    }
    __syncthreads();
    const int si = blockIdx.x * 64 + threadIdx.x;
    if (si >= nseg) return;
    const Seg sg = segs[si];
    BitReader br;
    br.init(stream, sg.off, stream + stream_len);
    int pred[kMaxComp] = {0, 0, 0};
    int16_t* cf = coef + (size_t)sg.frame * g.frame_blocks * 64;
    for (int m = sg.mcu0; m < sg.mcu0 + sg.nmcu; m++) {
        const int my = m / g.mcux, mx = m - my * g.mcux;
        for (int ci = 0; ci < g.nc; ci++) {
            const CompDev& c = g.comp[ci];
            const int nv = g.interleaved ? c.v : 1, nh = g.interleaved ? c.h : 1;
            for (int v = 0; v < nv; v++) {
                for (int h = 0; h < nh; h++) {
                    const int by = g.interleaved ? my * c.v + v : my, bx = g.interleaved ? mx * c.h + h : mx;
                    int16_t* blk = cf + (size_t)(c.coef0 + (long long)by * c.bw + bx) * 64;
                    // DC (jdhuff.c decode_mcu: s = HUFF_DECODE; r = GET_BITS(s); s = HUFF_EXTEND(r, s))
                    const int s0 = huff_decode(br, T[c.dc]);
                    br.refill();
                    pred[ci] += extend(br.get(s0), s0);
                    blk[0] = (int16_t)pred[ci];
                    const HuffDev& at = T[c.ac];
                    for (int k = 1; k < 64; k++) {
                        const int rs = huff_decode(br, at);
                        const int r = rs >> 4, s = rs & 15;
                        if (s) {
                            k += r;
                            br.refill();
                            blk[c_zigzag[min(k, 79)]] = (int16_t)extend(br.get(s), s);
                        } else {
                            if (r != 15) break;
                            k += 15;
                        }
                    }
                }
            }
        }
    }
}

// jidctint.c constants (CONST_BITS 13)
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

__device__ __forceinline__ void idct1d(int v0, int v1, int v2, int v3, int v4, int v5, int v6, int v7, int (&o)[8]) {
    int z1 = (v2 + v6) * F0_541;
    const int tmp2 = z1 - v6 * F1_847, tmp3 = z1 + v2 * F0_765;
    const int tmp0 = (v0 + v4) * 8192, tmp1 = (v0 - v4) * 8192;
    const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    int a0 = v7, a1 = v5, a2 = v3, a3 = v1;
    z1 = a0 + a3;
    int z2 = a1 + a2, z3 = a0 + a2, z4 = a1 + a3;
    const int z5 = (z3 + z4) * F1_175;
    a0 *= F0_298;
    a1 *= F2_053;
    a2 *= F3_072;
    a3 *= F1_501;
    z1 *= -F0_899;
    z2 *= -F2_562;
    z3 = z3 * -F1_961 + z5;
    z4 = z4 * -F0_390 + z5;
    a0 += z1 + z3;
    a1 += z2 + z4;
    a2 += z2 + z3;
    a3 += z1 + z4;
    o[0] = t10 + a3;
    o[7] = t10 - a3;
    o[1] = t11 + a2;
    o[6] = t11 - a2;
    o[2] = t12 + a1;
    o[5] = t12 - a1;
    o[3] = t13 + a0;
    o[4] = t13 - a0;
}

// IDCT_range_limit(cinfo)[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)
__device__ __forceinline__ uint32_t range_idct(int x) {
    const int v = x & 1023;
    return (uint32_t)(v < 128 ? v + 128 : v < 512 ? 255 : v < 896 ? 0 : v - 896);
}

// 8 lanes per block: lane r runs column r of pass 1, then row r of pass 2
__global__ __launch_bounds__(256) void k_jpeg_idct(int16_t* __restrict__ coef, const uint16_t* __restrict__ qt, JpegGeom g,
                                                    long long nblocks, uint8_t* __restrict__ planes) {
    __shared__ int ws[32][64];
    const long long b = (long long)blockIdx.x * 32 + (threadIdx.x >> 3);
    const int r = threadIdx.x & 7, lb = threadIdx.x >> 3;
    const bool live = b < nblocks;
    const long long fb = live ? b : 0;
    const long long frame = fb / g.frame_blocks;
    const long long rem = fb - frame * g.frame_blocks;
    int ci = 0;
    while (ci + 1 < g.nc && rem >= g.comp[ci + 1].coef0) ci++;
    const CompDev& c = g.comp[ci];
    const long long ib = rem - c.coef0;
    const int by = (int)(ib / c.bw), bx = (int)(ib - (long long)by * c.bw);
    int16_t* blk = coef + (size_t)fb * 64;
    const uint16_t* q = qt + ((size_t)frame * kMaxComp + ci) * 64;
    // pass 1: column r (jpeg_idct_islow, with the all-zero-AC column shortcut)
    int v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = live ? (int)blk[8 * k + r] * (int)q[8 * k + r] : 0;
    if (v[1] == 0 && v[2] == 0 && v[3] == 0 && v[4] == 0 && v[5] == 0 && v[6] == 0 && v[7] == 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) ws[lb][8 * k + r] = v[0] * 4;
    } else {
        int o[8];
        idct1d(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o);
#pragma unroll
        for (int k = 0; k < 8; k++) ws[lb][8 * k + r] = (o[k] + (1 << 10)) >> 11;
    }
    __syncthreads();
    // pass 2: row r (zero-row shortcut), range-limited samples
    int w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = ws[lb][8 * r + k];
    uint32_t px[8];
    if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
        const uint32_t d = range_idct((w[0] + 16) >> 5);
#pragma unroll
        for (int k = 0; k < 8; k++) px[k] = d;
    } else {
        int o[8];
        idct1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
#pragma unroll
        for (int k = 0; k < 8; k++) px[k] = range_idct((o[k] + (1 << 17)) >> 18);
    }
    if (!live) return;
    const int pw = c.bw * 8;
    uint8_t* row = planes + (size_t)frame * g.frame_plane + c.plane0 + ((size_t)by * 8 + r) * pw + (size_t)bx * 8;
    reinterpret_cast<uint2*>(row)[0] = make_uint2(px[0] | px[1] << 8 | px[2] << 16 | px[3] << 24,
                                                  px[4] | px[5] << 8 | px[6] << 16 | px[7] << 24);
    // leave the coefficient buffer zeroed for the next call (this block's 64 values were read by
    // the column pass above: their values fed pass 1, so the loads have returned)
    reinterpret_cast<uint4*>(blk)[r] = make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ int clamp255(int x) { return x < 0 ? 0 : x > 255 ? 255 : x; }

// chroma sample (cb or cr) at output pixel (y, x) after fancy upsampling (jdsample.c), from a
// plane downsampled by (hf, vf) in {1, 2}, real size dw x dh, row pitch pw.  jinit_upsampler uses
// the fancy filters only when downsampled_width > 2; narrower planes are replicated (h2v1_upsample,
// h2v2_upsample).
__device__ __forceinline__ int chroma_at(const uint8_t* p, int pw, int dw, int dh, int hf, int vf, int y, int x) {
    if (hf == 2 && dw <= 2) return p[(size_t)(y / vf) * pw + (x >> 1)];
    if (vf == 2) {  // h2v2_fancy_upsample (hf == 2)
        const int cy = y >> 1;
        const int fy = (y & 1) ? min(cy + 1, dh - 1) : max(cy - 1, 0);  // the farther context row
        const uint8_t* n = p + (size_t)cy * pw;
        const uint8_t* f = p + (size_t)fy * pw;
        const int cx = x >> 1;
        const int cs = n[cx] * 3 + f[cx];
        if ((x & 1) == 0) return cx == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + n[cx - 1] * 3 + f[cx - 1] + 8) >> 4;
        return cx == dw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + n[cx + 1] * 3 + f[cx + 1] + 7) >> 4;
    }
    const uint8_t* n = p + (size_t)y * pw;
    if (hf == 1) return n[x];
    const int cx = x >> 1;  // h2v1_fancy_upsample
    if ((x & 1) == 0) return cx == 0 ? n[0] : (n[cx] * 3 + n[cx - 1] + 1) >> 2;
    return cx == dw - 1 ? n[cx] : (n[cx] * 3 + n[cx + 1] + 2) >> 2;
}

// one thread per 4 output pixels of a row; ycc_rgb_convert (jdcolor.c build_ycc_rgb_table) -> BGR
template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_jpeg_color(const uint8_t* __restrict__ planes, JpegGeom g, int n,
                                                     uint8_t* __restrict__ out) {
    const int qpr = (g.W + 3) / 4;  // quads per row
    const long long id = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long total = (long long)n * g.H * qpr;
    if (id >= total) return;
    const int frame = (int)(id / ((long long)g.H * qpr));
    const long long rem = id - (long long)frame * g.H * qpr;
    const int y = (int)(rem / qpr), x0 = (int)(rem - (long long)y * qpr) * 4;
    const uint8_t* fp = planes + (size_t)frame * g.frame_plane;
    const CompDev& cy = g.comp[0];
    const uint8_t* yrow = fp + cy.plane0 + (size_t)y * (cy.bw * 8);
    uint8_t* o = out + ((size_t)frame * g.H + y) * g.W * 3;
    uint32_t bgr[4];
    const int nx = min(4, g.W - x0);
    for (int k = 0; k < 4; k++) {
        const int x = min(x0 + k, g.W - 1);
        const int Y = yrow[x];
        if (g.nc == 1) {
            bgr[k] = (uint32_t)Y | (uint32_t)Y << 8 | (uint32_t)Y << 16;
            continue;
        }
        const CompDev& ccb = g.comp[1];
        const CompDev& ccr = g.comp[2];
        const int hf = g.hmax / ccb.h, vf = g.vmax / ccb.v;
        const int dw = (g.W * ccb.h + g.hmax - 1) / g.hmax, dh = (g.H * ccb.v + g.vmax - 1) / g.vmax;
        const int cb = chroma_at(fp + ccb.plane0, ccb.bw * 8, dw, dh, hf, vf, y, x) - 128;
        const int cr = chroma_at(fp + ccr.plane0, ccr.bw * 8, dw, dh, hf, vf, y, x) - 128;
        const int R = clamp255(Y + ((91881 * cr + 32768) >> 16));
        const int G = clamp255(Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16));
        const int B = clamp255(Y + ((116130 * cb + 32768) >> 16));
        bgr[k] = (uint32_t)B | (uint32_t)G << 8 | (uint32_t)R << 16;
    }
    uint8_t* dst = o + (size_t)x0 * 3;
    if (ALIGNED && nx == 4) {  // 12 B at a 4-B aligned address: three dwords
        uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
        d32[0] = bgr[0] | bgr[1] << 24;
        d32[1] = bgr[1] >> 8 | bgr[2] << 16;
        d32[2] = bgr[2] >> 16 | bgr[3] << 8;
    } else {
        for (int k = 0; k < nx; k++) {
            dst[3 * k] = (uint8_t)bgr[k];
            dst[3 * k + 1] = (uint8_t)(bgr[k] >> 8);
            dst[3 * k + 2] = (uint8_t)(bgr[k] >> 16);
        }
    }
}

}  // namespace jp
}  // namespace fm

using namespace fm::jp;

// ---------------------------------------------------------------------------------------------
// host side

struct fm_mjpeg {
    int device = 0, W = 0, H = 0, max_frames = 0;
    std::string err;
    bool have_geom = false;
    JpegGeom g{};
    int tsel[kMaxComp][2] = {};      // (td, ta) of each component in the scan
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    // device buffers
    uint8_t* d_stream = nullptr;
    size_t stream_cap = 0;
    Seg* d_segs = nullptr;
    size_t segs_cap = 0;
    HuffDev* d_tabs = nullptr;         // [n_sets][4]
    int tabs_cap = 0;
    uint16_t* d_qt = nullptr;          // [max_frames][3][64] natural order
    int16_t* d_coef = nullptr;         // [max_frames][frame_blocks][64]
    uint8_t* d_planes = nullptr;       // [max_frames][frame_plane]
    uint8_t* d_out = nullptr;          // device BGR when the caller wants host output
    // pinned host staging (reused; the previous call's transfers are finished before refilling)
    uint8_t* h_stream = nullptr;
    size_t h_stream_cap = 0;
    Seg* h_segs = nullptr;
    size_t h_segs_cap = 0;
    HuffDev* h_tabs = nullptr;
    uint16_t* h_qt = nullptr;
    float last_ms = 0.f;
    bool timing = false;
};

namespace {

int jfail(fm_mjpeg* d, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (d) d->err = buf;
    return code;
}

#define JHIP(d, expr)                                                                               \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) return jfail(d, FM_EHIP, "%s: %s", #expr, hipGetErrorString(_e));     \
    } while (0)

struct HuffHost {
    uint8_t bits[17] = {};
    uint8_t vals[256] = {};
    int n = 0;
    bool present = false;
};

struct ParsedJpeg {
    uint16_t qt[4][64] = {};  // natural order
    bool qt_present[4] = {};
    HuffHost ht[2][4];        // [class][id]
    int W = 0, H = 0, nc = 0;
    int cid[kMaxComp] = {}, ch[kMaxComp] = {}, cv[kMaxComp] = {}, ctq[kMaxComp] = {};
    int ns = 0, sid[kMaxComp] = {}, std_[kMaxComp] = {}, sta[kMaxComp] = {};
    int dri = 0;
    size_t scan_begin = 0, scan_end = 0;  // entropy-coded bytes [begin, end) of the data
    size_t nrst = 0;                      // RSTn markers in the scan
};

const int kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                      41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                      30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int parse_jpeg(fm_mjpeg* d, int idx, const uint8_t* p, size_t n, ParsedJpeg& J) {
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return jfail(d, FM_EINVAL, "frame %d: no SOI", idx);
    size_t i = 2;
    bool sof = false;
    while (i + 4 <= n) {
        if (p[i] != 0xFF) return jfail(d, FM_EINVAL, "frame %d: marker expected at byte %zu", idx, i);
        while (i < n && p[i] == 0xFF) i++;
        if (i >= n) break;
        const int m = p[i++];
        if (m == 0xD9) break;
        if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
        if (i + 2 > n) return jfail(d, FM_EINVAL, "frame %d: truncated marker", idx);
        const size_t len = ((size_t)p[i] << 8) | p[i + 1];
        if (len < 2 || i + len > n) return jfail(d, FM_EINVAL, "frame %d: bad segment length", idx);
        const uint8_t* s = p + i + 2;
        const size_t sl = len - 2;
        if (m == 0xDB) {
            size_t q = 0;
            while (q < sl) {
                const int pq = s[q] >> 4, tq = s[q] & 15;
                q++;
                if (tq > 3 || q + (pq ? 128 : 64) > sl) return jfail(d, FM_EINVAL, "frame %d: bad DQT", idx);
                for (int k = 0; k < 64; k++) J.qt[tq][kZig[k]] = pq ? (uint16_t)((s[q + 2 * k] << 8) | s[q + 2 * k + 1]) : s[q + k];
                J.qt_present[tq] = true;
                q += pq ? 128 : 64;
            }
        } else if (m == 0xC4) {
            size_t q = 0;
            while (q < sl) {
                const int tc = s[q] >> 4, th = s[q] & 15;
                if (tc > 1 || th > 3 || q + 17 > sl) return jfail(d, FM_EINVAL, "frame %d: bad DHT", idx);
                HuffHost& t = J.ht[tc][th];
                int cnt = 0;
                for (int l = 1; l <= 16; l++) {
                    t.bits[l] = s[q + l];
                    cnt += s[q + l];
                }
                if (cnt > 256 || q + 17 + cnt > sl) return jfail(d, FM_EINVAL, "frame %d: bad DHT counts", idx);
                memcpy(t.vals, s + q + 17, cnt);
                t.n = cnt;
                t.present = true;
                q += 17 + cnt;
            }
        } else if (m == 0xC0 || m == 0xC1) {
            if (sl < 6 || s[0] != 8) return jfail(d, FM_ENOTSUP, "frame %d: only 8-bit samples", idx);
            J.H = (s[1] << 8) | s[2];
            J.W = (s[3] << 8) | s[4];
            J.nc = s[5];
            if ((J.nc != 1 && J.nc != 3) || sl < 6 + 3 * (size_t)J.nc)
                return jfail(d, FM_ENOTSUP, "frame %d: %d components (1 or 3 supported)", idx, J.nc);
            for (int c = 0; c < J.nc; c++) {
                J.cid[c] = s[6 + 3 * c];
                J.ch[c] = s[7 + 3 * c] >> 4;
                J.cv[c] = s[7 + 3 * c] & 15;
                J.ctq[c] = s[8 + 3 * c] & 3;
            }
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return jfail(d, FM_ENOTSUP, "frame %d: SOF%d (progressive / lossless / arithmetic) not supported", idx,
                         m - 0xC0);
        } else if (m == 0xDD) {
            if (sl < 2) return jfail(d, FM_EINVAL, "frame %d: bad DRI", idx);
            J.dri = (s[0] << 8) | s[1];
        } else if (m == 0xDA) {
            if (!sof) return jfail(d, FM_EINVAL, "frame %d: SOS before SOF", idx);
            J.ns = s[0];
            if (J.ns != J.nc || sl < 1 + 2 * (size_t)J.ns + 3)
                return jfail(d, FM_ENOTSUP, "frame %d: non-interleaved multi-scan JPEG not supported", idx);
            for (int k = 0; k < J.ns; k++) {
                J.sid[k] = s[1 + 2 * k];
                J.std_[k] = s[2 + 2 * k] >> 4;
                J.sta[k] = s[2 + 2 * k] & 15;
            }
            J.scan_begin = i + len;
            // the scan ends at the first marker that is neither stuffing nor RSTn
            size_t k = J.scan_begin;
            while (k + 1 < n && !(p[k] == 0xFF && p[k + 1] != 0 && !(p[k + 1] >= 0xD0 && p[k + 1] <= 0xD7))) k++;
            J.scan_end = k + 1 < n ? k : n;
            for (size_t q = J.scan_begin; q + 1 < J.scan_end;) {
                const uint8_t* ff = (const uint8_t*)memchr(p + q, 0xFF, J.scan_end - 1 - q);
                if (!ff) break;
                q = (size_t)(ff - p);
                if (p[q + 1] >= 0xD0 && p[q + 1] <= 0xD7) J.nrst++;
                q += 2;
            }
            return FM_OK;
        }
        i += len;
    }
    return jfail(d, FM_EINVAL, "frame %d: no scan", idx);
}

void build_table(const HuffHost& h, HuffDev& t) {
    memset(&t, 0, sizeof t);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        t.valoff[l] = k - code;
        for (int j = 0; j < h.bits[l]; j++) {
            if (l <= 9) {
                const int lo = code << (9 - l), hi = (code + 1) << (9 - l);
                for (int x = lo; x < hi && x < 512; x++) t.lut[x] = (uint16_t)((l << 8) | h.vals[k]);
            }
            code++;
            k++;
        }
        t.maxcode[l] = h.bits[l] ? code - 1 : -1;
        code <<= 1;
    }
    t.maxcode[17] = 0x7FFFFFFF;
    memcpy(t.vals, h.vals, sizeof t.vals);
}

template <typename T>
int grow_dev(fm_mjpeg* d, T** p, size_t& cap, size_t need) {
    if (need <= cap) return FM_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const size_t nc = std::max(need, cap * 3 / 2 + 1);
    JHIP(d, hipMalloc((void**)p, nc * sizeof(T)));
    cap = nc;
    return FM_OK;
}

template <typename T>
int grow_host(fm_mjpeg* d, T** p, size_t& cap, size_t need) {
    if (need <= cap) return FM_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    const size_t nc = std::max(need, cap * 3 / 2 + 1);
    JHIP(d, hipHostMalloc((void**)p, nc * sizeof(T), hipHostMallocDefault));
    cap = nc;
    return FM_OK;
}

// frame geometry from the first frame: component grids, planes, buffers
int setup_geometry(fm_mjpeg* d, const ParsedJpeg& J) {
    if (J.W != d->W || J.H != d->H)
        return jfail(d, FM_EINVAL, "JPEG is %dx%d, the decoder was created for %dx%d", J.W, J.H, d->W, d->H);
    JpegGeom& g = d->g;
    g = JpegGeom{};
    g.W = J.W;
    g.H = J.H;
    g.nc = J.nc;
    g.hmax = 1;
    g.vmax = 1;
    for (int c = 0; c < J.nc; c++) {
        g.hmax = std::max(g.hmax, J.ch[c]);
        g.vmax = std::max(g.vmax, J.cv[c]);
    }
    if (J.nc == 3) {
        const bool ok = J.ch[1] == 1 && J.cv[1] == 1 && J.ch[2] == 1 && J.cv[2] == 1 &&
                        ((J.ch[0] == 1 && J.cv[0] == 1) || (J.ch[0] == 2 && J.cv[0] == 1) || (J.ch[0] == 2 && J.cv[0] == 2));
        if (!ok)
            return jfail(d, FM_ENOTSUP, "sampling Y %dx%d Cb %dx%d Cr %dx%d not supported", J.ch[0], J.cv[0], J.ch[1],
                         J.cv[1], J.ch[2], J.cv[2]);
    } else if (J.ch[0] < 1 || J.cv[0] < 1 || J.ch[0] > 4 || J.cv[0] > 4) {
        return jfail(d, FM_EINVAL, "bad sampling factors");
    }
    g.interleaved = J.nc > 1;
    if (g.interleaved) {
        g.mcux = (g.W + 8 * g.hmax - 1) / (8 * g.hmax);
        g.mcuy = (g.H + 8 * g.vmax - 1) / (8 * g.vmax);
    } else {  // one component: one block per MCU over its own grid
        g.mcux = (g.W * J.ch[0] + 8 * g.hmax - 1) / (8 * g.hmax);
        g.mcuy = (g.H * J.cv[0] + 8 * g.vmax - 1) / (8 * g.vmax);
    }
    long long blocks = 0, plane = 0;
    for (int c = 0; c < J.nc; c++) {
        CompDev& cd = g.comp[c];
        cd.h = J.ch[c];
        cd.v = J.cv[c];
        cd.bw = g.interleaved ? g.mcux * cd.h : g.mcux;
        cd.bh = g.interleaved ? g.mcuy * cd.v : g.mcuy;
        cd.coef0 = blocks;
        cd.plane0 = plane;
        blocks += (long long)cd.bw * cd.bh;
        plane += (long long)cd.bw * cd.bh * 64;
    }
    g.frame_blocks = blocks;
    g.frame_plane = (plane + 15) & ~15ll;
    const size_t nb = (size_t)d->max_frames * blocks * 64;
    JHIP(d, hipMalloc((void**)&d->d_coef, nb * sizeof(int16_t)));
    JHIP(d, hipMemsetAsync(d->d_coef, 0, nb * sizeof(int16_t), d->st));
    JHIP(d, hipMalloc((void**)&d->d_planes, (size_t)d->max_frames * g.frame_plane));
    JHIP(d, hipMalloc((void**)&d->d_qt, (size_t)d->max_frames * kMaxComp * 64 * sizeof(uint16_t)));
    JHIP(d, hipHostMalloc((void**)&d->h_qt, (size_t)d->max_frames * kMaxComp * 64 * sizeof(uint16_t), hipHostMallocDefault));
    JHIP(d, hipStreamSynchronize(d->st));
    d->have_geom = true;
    return FM_OK;
}

}  // namespace

extern "C" {

int fm_mjpeg_create(int device, int width, int height, int max_frames, fm_mjpeg** out) {
    if (!out) return FM_EINVAL;
    fm_mjpeg* d = new fm_mjpeg();
    *out = d;
    if (width < 1 || height < 1 || max_frames < 1)
        return jfail(d, FM_EINVAL, "bad geometry %dx%d, max_frames %d", width, height, max_frames);
    d->device = device;
    d->W = width;
    d->H = height;
    d->max_frames = max_frames;
    JHIP(d, hipSetDevice(device));
    JHIP(d, hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking));
    JHIP(d, hipEventCreate(&d->e0));
    JHIP(d, hipEventCreate(&d->e1));
    JHIP(d, hipHostMalloc((void**)&d->h_tabs, 4 * sizeof(HuffDev), hipHostMallocDefault));
    return FM_OK;
}

void fm_mjpeg_destroy(fm_mjpeg* d) {
    if (!d) return;
    if (d->st) (void)hipStreamSynchronize(d->st);
    for (void* p : {(void*)d->d_stream, (void*)d->d_segs, (void*)d->d_tabs, (void*)d->d_qt, (void*)d->d_coef,
                    (void*)d->d_planes, (void*)d->d_out})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)d->h_stream, (void*)d->h_segs, (void*)d->h_tabs, (void*)d->h_qt})
        if (p) (void)hipHostFree(p);
    if (d->e0) (void)hipEventDestroy(d->e0);
    if (d->e1) (void)hipEventDestroy(d->e1);
    if (d->st) (void)hipStreamDestroy(d->st);
    delete d;
}

const char* fm_mjpeg_last_error(const fm_mjpeg* d) { return d ? d->err.c_str() : "null decoder"; }

double fm_mjpeg_last_ms(const fm_mjpeg* d) { return d ? (double)d->last_ms : 0.0; }

}  // extern "C"

// Queue the decode of n JPEGs into n BGR frames at device address out (pitch W*3, frames
// contiguous) on stream st (the decoder's own when null).  Host work: parse, unstuff, upload.
int fm_mjpeg_enqueue(fm_mjpeg* d, const uint8_t* const* jpegs, const size_t* sizes, int n, uint8_t* out, hipStream_t st) {
    if (!d) return FM_EINVAL;
    if (!jpegs || !sizes || !out || n < 1 || n > d->max_frames)
        return jfail(d, FM_EINVAL, "n %d outside [1, max_frames=%d] or null buffers", n, d->max_frames);
    JHIP(d, hipSetDevice(d->device));
    if (!st) st = d->st;
    // the previous call's uploads must be done before the pinned staging is refilled
    JHIP(d, hipStreamSynchronize(st));
    if (st != d->st) JHIP(d, hipStreamSynchronize(d->st));
    std::vector<ParsedJpeg> P(n);
    size_t total = 0;
    for (int i = 0; i < n; i++) {
        if (!jpegs[i]) return jfail(d, FM_EINVAL, "frame %d: null", i);
        if (int rc = parse_jpeg(d, i, jpegs[i], sizes[i], P[i])) return rc;
        total += P[i].scan_end - P[i].scan_begin + 8 * (P[i].nrst + 1);  // + zero padding after each segment
    }
    if (!d->have_geom)
        if (int rc = setup_geometry(d, P[0])) return rc;
    const JpegGeom& g = d->g;
    // tables: every frame must use the first frame's Huffman tables (MJPEG streams repeat one set);
    // quantization tables may differ per frame
    int sel[kMaxComp][2];
    for (int c = 0; c < g.nc; c++) {
        int k = 0;
        while (k < P[0].ns && P[0].sid[k] != P[0].cid[c]) k++;
        if (k == P[0].ns) return jfail(d, FM_EINVAL, "frame 0: component %d not in the scan", P[0].cid[c]);
        sel[c][0] = P[0].std_[k] & 3;
        sel[c][1] = P[0].sta[k] & 3;
    }
    for (int i = 0; i < n; i++) {
        const ParsedJpeg& J = P[i];
        if (J.W != g.W || J.H != g.H || J.nc != g.nc) return jfail(d, FM_EINVAL, "frame %d: geometry differs", i);
        for (int c = 0; c < g.nc; c++) {
            if (J.ch[c] != g.comp[c].h || J.cv[c] != g.comp[c].v) return jfail(d, FM_EINVAL, "frame %d: sampling differs", i);
            if (!J.qt_present[J.ctq[c]]) return jfail(d, FM_EINVAL, "frame %d: missing DQT %d", i, J.ctq[c]);
            for (int t = 0; t < 2; t++) {
                const HuffHost& a = J.ht[t][sel[c][t]];
                const HuffHost& b = P[0].ht[t][sel[c][t]];
                if (!a.present) return jfail(d, FM_EINVAL, "frame %d: missing DHT", i);
                if (i && (a.n != b.n || memcmp(a.bits, b.bits, sizeof a.bits) || memcmp(a.vals, b.vals, a.n)))
                    return jfail(d, FM_ENOTSUP, "frame %d: Huffman tables differ from frame 0's", i);
            }
        }
    }
    // slots 0..3 = (dc, ac) x 2 distinct ids at most
    for (int c = 0; c < g.nc; c++) {
        d->g.comp[c].dc = sel[c][0] & 1;
        d->g.comp[c].ac = 2 + (sel[c][1] & 1);
    }
    for (int t = 0; t < 2; t++) {
        build_table(P[0].ht[0][t], d->h_tabs[t]);
        build_table(P[0].ht[1][t], d->h_tabs[2 + t]);
    }
    // entropy-coded bytes: stuffing and RSTn removed, one segment per restart interval
    if (int rc = grow_host(d, &d->h_stream, d->h_stream_cap, total + 16)) return rc;
    const long long nmcu = (long long)g.mcux * g.mcuy;
    std::vector<Seg> segs;
    segs.reserve(n);
    size_t w = 0;
    for (int i = 0; i < n; i++) {
        const ParsedJpeg& J = P[i];
        const uint8_t* s = jpegs[i];
        const long long per = J.dri > 0 ? J.dri : nmcu;
        Seg cur{(uint32_t)w, 0, i, 0, (int32_t)std::min<long long>(per, nmcu)};
        size_t k = J.scan_begin;
        while (k < J.scan_end) {
            const uint8_t* ff = (const uint8_t*)memchr(s + k, 0xFF, J.scan_end - k);
            const size_t run = ff ? (size_t)(ff - (s + k)) : J.scan_end - k;
            memcpy(d->h_stream + w, s + k, run);
            w += run;
            k += run;
            if (!ff) break;
            const uint8_t nx = k + 1 < J.scan_end ? s[k + 1] : 0;
            if (nx == 0x00) {
                d->h_stream[w++] = 0xFF;
                k += 2;
            } else if (nx >= 0xD0 && nx <= 0xD7) {  // restart marker: the next interval starts here
                cur.len = (uint32_t)(w - cur.off);
                segs.push_back(cur);
                memset(d->h_stream + w, 0, 8);
                w += 8;
                const long long m0 = (long long)cur.mcu0 + cur.nmcu;
                cur = Seg{(uint32_t)w, 0, i, (int32_t)m0, (int32_t)std::min<long long>(per, nmcu - m0)};
                k += 2;
                if (cur.nmcu <= 0) break;
            } else {
                k += 1;  // fill byte
            }
        }
        cur.len = (uint32_t)(w - cur.off);
        if (cur.nmcu > 0) segs.push_back(cur);
        memset(d->h_stream + w, 0, 8);
        w += 8;
        if (J.dri > 0 && (long long)(segs.back().mcu0 + segs.back().nmcu) != nmcu)
            return jfail(d, FM_EINVAL, "frame %d: restart markers do not cover the %lld MCUs", i, nmcu);
        for (int c = 0; c < g.nc; c++) memcpy(d->h_qt + ((size_t)i * kMaxComp + c) * 64, J.qt[J.ctq[c]], 128);
    }
    memset(d->h_stream + w, 0, 16);
    w += 16;
    if (w >= (size_t)UINT32_MAX) return jfail(d, FM_ENOTSUP, "compressed batch too large");
    if (int rc = grow_host(d, &d->h_segs, d->h_segs_cap, segs.size())) return rc;
    memcpy(d->h_segs, segs.data(), segs.size() * sizeof(Seg));
    if (int rc = grow_dev(d, &d->d_stream, d->stream_cap, w + 8)) return rc;  // word reads may pass w by 3 B
    if (int rc = grow_dev(d, &d->d_segs, d->segs_cap, segs.size())) return rc;
    size_t tcap = d->tabs_cap;
    if (int rc = grow_dev(d, &d->d_tabs, tcap, 4)) return rc;
    d->tabs_cap = (int)tcap;
    JHIP(d, hipMemcpyAsync(d->d_stream, d->h_stream, w, hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(d->d_segs, d->h_segs, segs.size() * sizeof(Seg), hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(d->d_tabs, d->h_tabs, 4 * sizeof(HuffDev), hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(d->d_qt, d->h_qt, (size_t)n * kMaxComp * 64 * sizeof(uint16_t), hipMemcpyHostToDevice, st));
    if (d->timing) JHIP(d, hipEventRecord(d->e0, st));
    const int nseg = (int)segs.size();
    hipLaunchKernelGGL(k_jpeg_huff, dim3((nseg + 63) / 64), dim3(64), 0, st, d->d_stream, (uint32_t)w, d->d_segs, nseg,
                       d->d_tabs, d->g, d->d_coef);
    JHIP(d, hipGetLastError());
    const long long nb = (long long)n * g.frame_blocks;
    hipLaunchKernelGGL(k_jpeg_idct, dim3((unsigned)((nb + 31) / 32)), dim3(256), 0, st, d->d_coef, d->d_qt, d->g, nb,
                       d->d_planes);
    JHIP(d, hipGetLastError());
    const long long nq = (long long)n * g.H * ((g.W + 3) / 4);
    const bool aligned = ((uintptr_t)out & 3) == 0 && (g.W * 3) % 4 == 0;
    if (aligned)
        hipLaunchKernelGGL(k_jpeg_color<true>, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, d->d_planes, d->g, n, out);
    else
        hipLaunchKernelGGL(k_jpeg_color<false>, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, d->d_planes, d->g, n, out);
    JHIP(d, hipGetLastError());
    if (d->timing) JHIP(d, hipEventRecord(d->e1, st));
    return FM_OK;
}

extern "C" {

int fm_mjpeg_decode(fm_mjpeg* d, const uint8_t* const* jpegs, const size_t* sizes, int n, uint8_t* out, int out_on_device) {
    if (!d) return FM_EINVAL;
    d->timing = true;
    uint8_t* dst = out;
    const size_t fb = (size_t)d->W * d->H * 3;
    if (!out_on_device) {
        if (!d->d_out) JHIP(d, hipMalloc((void**)&d->d_out, (size_t)d->max_frames * fb));
        dst = d->d_out;
    }
    if (int rc = fm_mjpeg_enqueue(d, jpegs, sizes, n, dst, d->st)) return rc;
    if (!out_on_device) JHIP(d, hipMemcpyAsync(out, dst, (size_t)n * fb, hipMemcpyDeviceToHost, d->st));
    JHIP(d, hipStreamSynchronize(d->st));
    JHIP(d, hipEventElapsedTime(&d->last_ms, d->e0, d->e1));
    return FM_OK;
}

}  // extern "C"
