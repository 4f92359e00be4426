// fm_small.hip — the per-pixel motion chain for small work images (round 5): mode D, the reference
// CLI's default -B 100 (find_motion.py:1474, resize fm.py:492: 1080p -> 100 x 56, two 64 x 64 tiles per
// stream).  Reference chain per frame (fm.py): cvtColor 493, GaussianBlur 494, mask_off_areas 619-636,
// absdiff(convertScaleAbs) 250, threshold 257, accumulateWeighted 659.
//
// On a two-tile image k_pix5 (16 waves per tile, two workgroups) runs a batch's 256 frames one after
// another: 224 us per 256 frames alone, 355 us beside the next batch's resize (round 4), a latency chain
// with one LDS barrier per frame on 2 CUs.  But only the f64 running average is sequential in time
// (SURVEY.md §5); gray and blur of a frame depend on that frame alone.  So:
//
//   k_small_blur  one workgroup per frame (all T x S frames of the batch at once, over every CU):
//                 gray (fm.py:493), the k x k fixed-point Gaussian (fm.py:494, REFLECT_101), the keep-mask
//                 (masked pixels blur to 0, fm.py:619-636) -> blur bytes [F][x][y] (column-major, column
//                 stride CS = nty * 64), and it clears the frame's tile flags and the bit words of the
//                 columns past the image;
//   k_small_scan  one wave per (stream, image column, 64-row tile row), lane = row: the frames in order
//                 with the f64 background in a register -- diff (convertScaleAbs + absdiff), threshold,
//                 accumulateWeighted -- and __ballot of `d > t` is the tile's column word of threshold
//                 bits directly (word c = column c, bit r = row r: the contour pass's layout).  A block of
//                 64 frames' words is held one frame per lane and stored at once, with the frames' flags
//                 ORed atomically into word 0 of each tile-frame's 8 (the reader ORs them) where a word has
//                 bits: no per-frame store, branch or address arithmetic (1,450 -> 1,002 instructions in the
//                 kernel, the scan 120 -> 65 us per 256 frames beside the resize, round 5).
//
// Same arithmetic as k_pix5 / the oracle: gray (1868 B + 9617 G + 4899 R + 8192) >> 14, blur
// (sum_y c_y sum_x c_x g + 2^15) >> 16 with OpenCV's 8-bit taps, q = sat_u8(rne(|(float)bg|)),
// d = |blur - q| > t, bg = fma(bg, 1 - a, blur * a) (scalar tail past acc_vec_end: blur * a + bg * (1 - a)),
// the stream's first frame bg := blur before the diff.
#include "fm_internal.h"

namespace fm {
namespace sm {

constexpr int BT = 256;  // k_small_blur threads
constexpr int ST = 256;  // k_small_scan threads (4 waves, each its own job)
constexpr int PFD = 8;  // k_small_scan: frames per group of blur-byte loads
constexpr int NG = 2;   // groups in flight (4 and 8: scans 5 % shorter, mode D unchanged, round 5)

__device__ __forceinline__ int refl(int p, int len) {  // BORDER_REFLECT_101 (any distance)
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = (p < 0) ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ uint32_t gray_px(uint32_t b, uint32_t g, uint32_t r) {
    return (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14;
}

// H's row stride in dwords: odd, so that the vertical pass's 64 lanes (consecutive rows of one column)
// read 64 distinct banks (at w = 100 the unpadded stride put them on 16 banks: 4-way conflicts)
__host__ __device__ constexpr int h_stride(int w) { return w | 1; }

// LDS of k_small_blur: gray u8 [h][w], H u32 [h][h_stride(w)], reflected column / row indices
__host__ __device__ constexpr size_t blur_lds_bytes(int h, int w, int R) {
    return ((size_t)h * w + 3) / 4 * 4 + (size_t)h * h_stride(w) * 4 + (size_t)(w + 2 * R) * 4 +
           (size_t)(h + 2 * R) * 4;
}

__global__ __launch_bounds__(BT) void k_small_blur(FusedArgs a, uint8_t* __restrict__ sblur, int CS) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int h = a.h, w = a.w, S = a.S, K = a.ksize, R = K >> 1;
    const int n = h * w, HS = h_stride(w);
    const size_t f = (size_t)a.t_begin * S + blockIdx.x;  // frame of this workgroup (t_begin * S + t * S + s)
    const int s = (int)(f % S);
    uint8_t* g = lds;
    uint32_t* H = reinterpret_cast<uint32_t*>(lds + (n + 3) / 4 * 4);
    int* xi = reinterpret_cast<int*>(H + (size_t)h * HS);  // [w + 2R]: reflected source column of x - R
    int* yi = xi + w + 2 * R;                 // [h + 2R]
    const int tid = threadIdx.x;
    kstamp_begin_grid(a.kstamp);
    for (int i = tid; i < w + 2 * R; i += BT) xi[i] = refl(i - R, w);
    for (int i = tid; i < h + 2 * R; i += BT) yi[i] = refl(i - R, h);
    // this frame's tile flags (k_small_scan ORs into word 0 of each) and the bit words of the columns
    // past the image in the last tile column (no scan wave writes them)
    for (int i = tid; i < a.ntiles * 8; i += BT) a.tflag[f * a.ntiles * 8 + i] = 0u;
    const int xpad = a.ntx * 64 - w;
    for (int i = tid; i < a.nty * xpad; i += BT) {
        const int ty = i / xpad, c = w - (a.ntx - 1) * 64 + (i - ty * xpad);
        a.bits[(f * a.ntiles + ty * a.ntx + a.ntx - 1) * 64 + c] = 0ull;
    }
    // gray: pixel quads as three dwords where the frame allows (4-B aligned), single pixels otherwise
    const uint8_t* src = a.src + f * (size_t)n * 3;
    const int nq = ((reinterpret_cast<uintptr_t>(src) & 3) == 0) ? n / 4 : 0;
    for (int q = tid; q < nq; q += BT) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(src) + 3 * q;
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
        const uint32_t v = gray_px(d0 & 0xFF, (d0 >> 8) & 0xFF, (d0 >> 16) & 0xFF) |
                           gray_px(d0 >> 24, d1 & 0xFF, (d1 >> 8) & 0xFF) << 8 |
                           gray_px((d1 >> 16) & 0xFF, d1 >> 24, d2 & 0xFF) << 16 |
                           gray_px((d2 >> 8) & 0xFF, (d2 >> 16) & 0xFF, d2 >> 24) << 24;
        reinterpret_cast<uint32_t*>(g)[q] = v;
    }
    for (int i = 4 * nq + tid; i < n; i += BT) g[i] = (uint8_t)gray_px(src[3 * i], src[3 * i + 1], src[3 * i + 2]);
    __syncthreads();
    // horizontal taps: H = sum_t c[t] * gray(y, x + t - R) (<= 255 * 256)
    for (int i = tid; i < n; i += BT) {
        const int y = i / w, x = i - y * w;
        const uint8_t* row = g + y * w;
        uint32_t acc = 0;
        for (int t = 0; t < K; t++) acc += (uint32_t)a.coef[t] * row[xi[x + t]];
        H[y * HS + x] = acc;
    }
    __syncthreads();
    // vertical taps, rounding, keep-mask; written column-major: thread i -> (x, y) with y fastest
    const bool hk = a.has_keep[s] != 0;
    const uint8_t* keep = a.keep + (size_t)s * n;
    uint8_t* out = sblur + f * (size_t)w * CS;
    for (int i = tid; i < n; i += BT) {
        const int x = i / h, y = i - x * h;
        uint32_t acc = 32768u;
        for (int t = 0; t < K; t++) acc += (uint32_t)a.coef[t] * H[yi[y + t] * HS + x];
        uint32_t blur = acc >> 16;
        if (hk && keep[y * w + x] == 0) blur = 0;
        out[x * CS + y] = (uint8_t)blur;
    }
    kstamp_end_wg(a.kstamp);
}

template <bool TAILK>
__global__ __launch_bounds__(ST) void k_small_scan(FusedArgs a, const uint8_t* __restrict__ sblur, int CS) {
    const int tid = threadIdx.x, ln = tid & 63;
    const int h = a.h, w = a.w, S = a.S;
    const double alpha = a.alpha;
    kstamp_begin_grid(a.kstamp);
    const int job = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (ST / 64) + (tid >> 6)));
    const int njobs = S * w * a.nty;
    if (job < njobs) {
        const int s = job / (w * a.nty);
        const int rem = job - s * w * a.nty;
        const int ty = rem / w, x = rem - ty * w;
        const int y = ty * 64 + ln;
        const bool valid = y < h;
        const uint64_t vmask = __builtin_amdgcn_ballot_w64(valid);
        const int tile = ty * a.ntx + x / 64, c = x & 63;
        const size_t plane = (size_t)h * w;
        const long long li = (long long)y * w + x;
        const bool tail = TAILK && li >= a.acc_vec_end;  // accumulateWeighted's scalar tail
        const double beta = a.beta;
        const int thr = a.thresh;
        const int t0 = a.t_begin, t1 = a.t_end;
        const bool init0 = a.init != nullptr && a.init[s] != 0;
        double bg = (valid && !init0) ? a.bg_in[(size_t)s * plane + li] : 0.0;
        const int yl = valid ? y : 0;
        // blur bytes of frame t of this pixel: sblur[((t * S + s) * w + x) * CS + y]
        const uint8_t* col = sblur + (size_t)x * CS + yl;
        const size_t fstride = (size_t)S * w * CS;
        const uint8_t* base = col + (size_t)s * w * CS;
        const uint32_t flagL = c < 2 ? (FLAG_L) : 0u, flagR = c >= 62 ? FLAG_R : 0u;
        // blur bytes of NG groups of PFD frames in flight (HBM latency is ~2 us beside the resize; one group
        // of 8 frames ahead left the scan waiting for every group)
        uint32_t rg[NG][PFD];
        // each frame's column word into lane (t - t0) % 64 of (wlo, whi); every 64 frames the
        // block's words are stored (one store, a frame per lane) and their flag words ORed into the tile-frame
        // flags (one atomic, lanes with bits): no per-frame store, branch or address arithmetic
        uint32_t wlo = 0, whi = 0;
        uint64_t* const bits0 = a.bits + ((size_t)s * a.ntiles + tile) * 64 + c;  // frame 0's word of (s, tile, c)
        uint32_t* const flag0 = a.tflag + ((size_t)s * a.ntiles + tile) * 8;
        const size_t bstride = (size_t)S * a.ntiles * 64, fstride8 = (size_t)S * a.ntiles * 8;
        auto flush = [&](int tb, int n) __attribute__((always_inline)) {  // frames tb .. tb + n - 1 in lanes 0 .. n - 1
            if (ln < n) {
                const size_t ft = (size_t)(tb + ln);
                const uint64_t word = ((uint64_t)whi << 32) | wlo;
                bits0[ft * bstride] = word;
                if (word) {
                    const uint32_t fl = FLAG_ANY | flagL | flagR |
                                        ((word & 3ull) ? (FLAG_T | (c < 2 ? FLAG_TL : 0u) | (c >= 62 ? FLAG_TR : 0u)) : 0u) |
                                        ((word >> 62) ? (FLAG_B | (c < 2 ? FLAG_BL : 0u) | (c >= 62 ? FLAG_BR : 0u)) : 0u);
                    atomicOr(&flag0[ft * fstride8], fl);
                }
            }
        };
        auto load_group = [&](uint32_t (&r)[PFD], int tg) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < PFD; k++) r[k] = base[(size_t)min(tg + k, t1 - 1) * fstride];  // clamped: unconditional
        };
        auto run_group = [&](const uint32_t (&r)[PFD], int tg) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < PFD; k++) {
                const int t = tg + k;
                if (t >= t1) break;  // wave-uniform
                const uint32_t blur = r[k];
                const double bv = (init0 && t == t0) ? (double)blur : bg;
                const int q = min(max(__float2int_rn(fabsf(__double2float_rn(bv))), 0), 255);
                const int d = abs((int)blur - q);
                const uint64_t word = __builtin_amdgcn_ballot_w64(d > thr) & vmask;
                // blur * alpha on the VALU (the pixel kernels' LDS table holds the same correctly rounded
                // product): a 256-entry f64 table read by 64 unrelated bytes averaged 1.95 bank-conflict
                // cycles per LDS cycle here, and the product is off the background's dependency chain
                const double bl = __dmul_rn((double)blur, alpha);
                bg = tail ? __dadd_rn(bl, __dmul_rn(bv, beta)) : __fma_rn(bv, beta, bl);
                const int kb = (t - t0) & 63;
                const bool mine = ln == kb;
                wlo = mine ? (uint32_t)word : wlo;
                whi = mine ? (uint32_t)(word >> 32) : whi;
                if (kb == 63) flush(t - 63, 64);
            }
        };
        static_for<NG>([&](auto g) { load_group(rg[decltype(g)::value], t0 + decltype(g)::value * PFD); });
        for (int tg = t0; tg < t1; tg += NG * PFD) {
            static_for<NG>([&](auto g) {
                constexpr int G = decltype(g)::value;
                run_group(rg[G], tg + G * PFD);
                load_group(rg[G], tg + (NG + G) * PFD);
            });
        }
        if (const int nrem = (t1 - t0) & 63) flush(t1 - nrem, nrem);  // the last, partial block
        if (valid) a.bg_out[(size_t)s * plane + li] = bg;
    }
    kstamp_end_wg(a.kstamp);
}

}  // namespace sm

bool small_supported(int h, int w, int ksize) {
    return (long long)h * w <= 16384 && ksize <= kMaxK && sm::blur_lds_bytes(h, w, ksize >> 1) <= 64 * 1024;
}

size_t small_scratch_bytes(int h, int w, int nty, size_t frames) { return frames * (size_t)w * nty * 64; }

// frames [a.t_begin, a.t_end) of the batch: blur of every frame in parallel, then the scan; a.init may mark
// first frames (bg := blur at t_begin).  ks1 / ks2: launch stamps of the two kernels (or nullptr)
hipError_t launch_small(hipStream_t st, const FusedArgs& a, uint8_t* sblur, uint64_t* ks1, uint64_t* ks2) {
    const int CS = a.nty * 64;
    const int nf = (a.t_end - a.t_begin) * a.S;
    const size_t lds = sm::blur_lds_bytes(a.h, a.w, a.ksize >> 1);
    FusedArgs b = a;
    b.kstamp = ks1;
    hipLaunchKernelGGL(sm::k_small_blur, dim3(nf), dim3(sm::BT), lds, st, b, sblur, CS);
    b.kstamp = ks2;
    const int njobs = a.S * a.w * a.nty;
    const dim3 grid((njobs + sm::ST / 64 - 1) / (sm::ST / 64));
    if (a.acc_vec_end < (long long)a.h * a.w) hipLaunchKernelGGL(sm::k_small_scan<true>, grid, dim3(sm::ST), 0, st, b, sblur, CS);
    else hipLaunchKernelGGL(sm::k_small_scan<false>, grid, dim3(sm::ST), 0, st, b, sblur, CS);
    return hipGetLastError();
}

}  // namespace fm
