// fm_pix.hip — the per-pixel motion chain, temporally blocked (gfx950).
//
// One workgroup (512 threads = 8 waves) owns a 64x64 tile of one stream for
// all T frames of a batch and computes, per frame (reference = fm.py):
//
//   gray    cvtColor(BGR2GRAY)                     fm.py:493   4 px/lane, v_perm + v_dot2
//   blur    GaussianBlur(k,k), fixed point,        fm.py:494   horizontal: v_dot4 over byte
//           REFLECT_101                                        windows; vertical: v_dot2 over
//                                                              transposed u16 pairs in LDS
//   mask    keep-mask (mask_off_areas)             fm.py:619-636
//   diff    absdiff(blur, convertScaleAbs(bg))     fm.py:250
//   thresh  delta > t                              fm.py:257   -> one bit per pixel (ballot)
//   accum   accumulateWeighted(blur, bg, a), f64   fm.py:659   bg lives in registers
//
// Every pixel's chain runs exactly once: the 5x5 dilation (fm.py:266) is NOT
// done here but on the threshold bit rows by k_dilate_ccl, which needs the
// 2-px halo of neighbouring tiles' bits, not their chains.  Outputs per
// frame: 64 threshold bit rows per tile (1/8 B per pixel), plus gray / blur /
// frame_delta planes when the caller keeps them (show / debug).
//
// HBM per launch (T frames, S streams): BGR 3 B/px/frame read once (the
// 2..12-px gray halo re-read comes from L2/MALL: tiles are swizzled so that
// horizontally adjacent tiles run on the same XCD), f64 background 16 B/px
// per batch, bits 1/8 B/px/frame.
#include "fm_internal.h"

namespace fm {
namespace px {

constexpr int TS = 64;          // tile edge
// minimum waves per SIMD the steady-state kernels are compiled for: 2 workgroups of 8 waves per CU =
// 4 per SIMD (<= 128 VGPRs).  (6 per SIMD, three k_pix5 workgroups per CU: 366 vs 401 k frames/s,
// round 4.)  k_pix<21> has no cap (178 VGPRs, one workgroup per CU).
constexpr int kPixWPE = 4;
constexpr int NT = 512;         // threads
constexpr int NW = NT / 64;     // waves; wave w owns tile rows [8w, 8w + 8)
constexpr int RPWV = TS / NW;   // rows per wave in the chain stage
static_assert(NW == 8, "tflag holds 8 words per tile (FusedArgs::tflag_waves)");

__host__ __device__ constexpr int a16(int v) { return (v + 15) & ~15; }

// Geometry of the gray (G) region for blur radius r: rows y0-r .. y0+63+r,
// columns x0-PC .. x0+63+PC with PC = 4*ceil(r/4) (quad aligned)
struct Geo {
    int r, PC, GW, NQ, GH, RS, CPR, nchunks, RSH;
    int o_raw, o_H, o_rowy, o_colx, o_atab, bytes;
    int raw_bytes, H_bytes;  // per buffer; raw and H are double buffered
    __host__ __device__ explicit Geo(int rr) {
        r = rr;
        PC = 4 * ((r + 3) / 4);
        GW = TS + 2 * PC;
        NQ = GW / 4;
        GH = TS + 2 * r;
        RS = a16(3 * GW + 15);  // aligned-down row start (<= 15 B early) + 3 B per gray column
        CPR = RS / 16;
        nchunks = GH * CPR;
        RSH = TS;  // H is row-major: u16 [GH (+1 pad row)][TS]
        // every thread's chunk slots (NT per 16-B column of chunks), so the staging stores
        // need no per-lane predicate: slots past the G region only take garbage
        raw_bytes = ((nchunks + NT - 1) / NT) * NT * 16;
        H_bytes = a16((GH + 1) * RSH * 2);
        o_raw = 0;
        o_H = o_raw + 2 * raw_bytes;
        o_rowy = o_H + 2 * H_bytes;
        o_colx = o_rowy + a16(GH * 4);
        o_atab = o_colx + a16(GW * 4);
        bytes = o_atab + 256 * 8;  // blur * alpha for blur = 0..255 (f64)
    }
};

__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = (p < 0) ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// LDS-only barrier: the next frame's raw prefetch (global loads) stays in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));


// BGR2GRAY of 4 consecutive pixels packed in 3 dwords (B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3):
// (1868 B + 9617 G + 4899 R + 8192) >> 14 computed with all constants x4, so that
// gray is byte 2 of the sum (< 2^24) and two v_perm gather the four results.
__device__ __forceinline__ uint32_t gray4(uint32_t d0, uint32_t d1, uint32_t d2) {
    const u16x2_t cbg = __builtin_bit_cast(u16x2_t, (4u * 1868u) | ((4u * 9617u) << 16));
    constexpr uint32_t CR = 4u * 4899u, RND = 4u * 8192u;
    const uint32_t p0 = __builtin_amdgcn_perm(d0, d0, 0x0C010C00u);
    const uint32_t p1 = __builtin_amdgcn_perm(d1, d0, 0x0C040C03u);
    const uint32_t p2 = __builtin_amdgcn_perm(d1, d1, 0x0C030C02u);
    const uint32_t p3 = __builtin_amdgcn_perm(d2, d2, 0x0C020C01u);
    const uint32_t g0 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p0), cbg, __umul24((d0 >> 16) & 0xFF, CR) + RND, false);
    const uint32_t g1 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p1), cbg, __umul24((d1 >> 8) & 0xFF, CR) + RND, false);
    const uint32_t g2 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p2), cbg, __umul24(d2 & 0xFF, CR) + RND, false);
    const uint32_t g3 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p3), cbg, __umul24(d2 >> 24, CR) + RND, false);
    return __builtin_amdgcn_perm(g1, g0, 0x0C0C0602u) | __builtin_amdgcn_perm(g3, g2, 0x06020C0Cu);
}

__device__ __forceinline__ uint32_t gray1(const uint8_t* p) {
    return ((uint32_t)p[0] * 1868u + (uint32_t)p[1] * 9617u + (uint32_t)p[2] * 4899u + 8192u) >> 14;
}

// window of 4 bytes starting at byte p of the little-endian concatenation q[0], q[1], ...
template <int P, int N>
__device__ __forceinline__ uint32_t win4(const uint32_t (&q)[N]) {
    if constexpr ((P & 3) == 0) return q[P >> 2];
    else return __builtin_amdgcn_alignbyte(q[(P >> 2) + 1], q[P >> 2], P & 3);
}

// horizontal taps of output I of a quad: sum_t c[t] * g[I + OFF + t]; NG dot4 groups
template <int I, int OFF, int NG, int G, int N>
__device__ __forceinline__ uint32_t htap(const uint32_t (&q)[N], const uint32_t (&cpk)[NG], uint32_t acc) {
    if constexpr (G == NG) return acc;
    else return htap<I, OFF, NG, G + 1, N>(q, cpk, __builtin_amdgcn_udot4(win4<I + OFF + 4 * G, N>(q), cpk[G], acc, false));
}

// 16-B raw chunks of the G region of one frame: chunk c -> row c / CPR, 16 B at
// the row's aligned start + 16 * (c % CPR); chunks past the row's last byte are skipped
template <int NCH>
struct Raw {
    uint4 v[NCH];
};

__device__ __attribute__((noinline)) uint4 load_partial(const uint8_t* ca, const uint8_t* fb, const uint8_t* fe) {
    uint32_t wds[4] = {0, 0, 0, 0};
    for (int b = 0; b < 16; b++)
        if (ca + b >= fb && ca + b < fe) wds[b >> 2] |= (uint32_t)ca[b] << (8 * (b & 3));
    return make_uint4(wds[0], wds[1], wds[2], wds[3]);
}

// Per-thread chunk plan, frame invariant: chunk i of this thread starts at byte
// rel0[i] - mis of its frame, where rel0 = (row offset + 3*cx0) + 16*k and
// mis = (frame address + rel0) & 15 aligns the row start down to 16 B.
template <int NCH>
struct ChunkPlan {
    uint32_t rel0[NCH];
    uint32_t k16[NCH];  // 16*k, or 0xFFFF for a slot past the last chunk
};

template <int NCH>
__device__ __forceinline__ void plan_chunks(ChunkPlan<NCH>& P, const int* rowy, const Geo& g, int cx0, int w, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        const int c = tid + NT * i;
        const int gy = c / g.CPR, k = c - gy * g.CPR;
        const bool live = c < g.nchunks;
        P.rel0[i] = live ? (uint32_t)(rowy[gy] * w + cx0) * 3u + 16u * k : 0u;
        P.k16[i] = live ? 16u * k : 0xFFFFu;
    }
}

template <int NCH>
__device__ __forceinline__ void load_raw(Raw<NCH>& R, const uint8_t* fsrc, uint32_t fbytes, const ChunkPlan<NCH>& P,
                                         uint32_t span) {
    const uint32_t flo = (uint32_t)(uintptr_t)fsrc;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        const uint32_t mis = (flo + P.rel0[i]) & 15u;
        const int rel = (int)P.rel0[i] - (int)mis;
        // one unconditional aligned 16-B load per slot from inside the frame: slots the gray
        // stage does not read (past the row segment's last byte, or past the G region) take
        // any in-frame window; a needed chunk hanging over either end of the frame (frame
        // not 16-B aligned) is gathered bytewise instead
        const bool full = rel >= 0 && (uint32_t)rel + 16u <= fbytes;
        const int relc = full ? rel : rel < 0 ? rel + 16 : rel - 16;
        uint4 val = *reinterpret_cast<const uint4*>(fsrc + relc);
        if (__builtin_expect(!full && P.k16[i] < span + mis, 0)) val = load_partial(fsrc + rel, fsrc, fsrc + fbytes);
        R.v[i] = val;
    }
}

template <int NCH>
__device__ __forceinline__ void store_raw(const Raw<NCH>& R, uint8_t* raw, const Geo& g, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        // chunk c = row c / CPR, 16 B at 16 * (c % CPR) of that row: byte 16 * c (RS = 16 * CPR)
        *reinterpret_cast<uint4*>(raw + 16 * (tid + NT * i)) = R.v[i];
    }
}

// XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8
// XCDs, so block b runs on XCD b % 8; give each XCD a contiguous run of tiles
// (row-major), so left/right neighbours share that XCD's L2 for the halo.
__device__ __forceinline__ int swizzle_tile(int b, int n) {
    const int full = n & ~7;
    if (b >= full) return b;
    return (b & 7) * (full >> 3) + (b >> 3);
}

// (A 2-D order -- each XCD's 64 resident workgroups as an 8 x 8 tile block, so that vertical halos
// also come through its L2 -- measured slower, round 4: config 5 3.33 vs 3.19 ms per launch.)

// OpenCV's 8-bit fixed-point Gaussian taps (getGaussianKernelBitExact +
// error-diffusion rounding, restated in fm_capi.cpp gaussian_taps); fixed at
// compile time so they are instruction literals.  launch_pix checks them
// against the context's taps.
template <int K> struct Taps;
template <> struct Taps<3> { static constexpr int c[3] = {64, 128, 64}; };
template <> struct Taps<5> { static constexpr int c[5] = {16, 64, 96, 64, 16}; };
template <> struct Taps<7> { static constexpr int c[7] = {8, 28, 56, 72, 56, 28, 8}; };
template <> struct Taps<21> {
    static constexpr int c[21] = {0, 2, 2, 4, 6, 11, 15, 20, 25, 28, 30, 28, 25, 20, 15, 11, 6, 4, 2, 2, 0};
};
template <int K> constexpr uint32_t tap4(int g) {
    uint32_t v = 0;
    for (int b = 0; b < 4; b++)
        if (4 * g + b < K) v |= (uint32_t)Taps<K>::c[4 * g + b] << (8 * b);
    return v;
}
template <int K> constexpr uint32_t tap2(int t) {
    return (uint32_t)Taps<K>::c[2 * t] | (2 * t + 1 < K ? (uint32_t)Taps<K>::c[2 * t + 1] << 16 : 0u);
}

// accumulateWeighted's bg = fma(bg, beta, blur * alpha) updating the background register in place.
// As __fma_rn the compiler picks v_fmac_f64 accumulating into the register of the table read, so
// every loop-carried background value went through a v_mov_b64 at the top of the frame loop
// (8 of the chain's ~95 VALU instructions per wave-frame).
__device__ __forceinline__ double bg_fma(double b, double beta, double bl) {
    asm("v_fma_f64 %0, %0, %1, %2" : "+v"(b) : "s"(beta), "v"(bl));
    return b;
}

// A frame's base address in SGPRs, so the quad loads take the saddr form (SGPR base + the lane's
// 32-bit offset) instead of a per-lane 64-bit multiply-add per load (LICM had hoisted
// src + offset out of the frame loop as a 64-bit VGPR pair).
typedef const __attribute__((address_space(1))) uint8_t* gbytes_t;  // global (not flat) addressing
typedef uint32_t u32x3_t __attribute__((ext_vector_type(3)));
// 12 bytes at a 4-B aligned global address (global_load_dwordx3)
// (the compiler keeps base + offset as one 64-bit add per load: passing the offset through an empty
// asm to get SGPR base + 32-bit VGPR offset cost a copy per load and a vmcnt wait at the back-edge)
// (non-temporal: 345 vs 412 k frames/s -- the halo lines are re-read from L2; round 6, r06i_nontemporal_ab.txt)
__device__ __forceinline__ void load12(u32x3_t& d, gbytes_t base, uint32_t off) {
    typedef uint32_t __attribute__((ext_vector_type(3), aligned(4))) u3a;
    d = *(const __attribute__((address_space(1))) u3a*)(base + off);
}
// k_pixw's quad loads are buffer loads through a per-frame descriptor built from wave-uniform values
// (frame base and size in SGPRs): the lane's 32-bit offset is the whole per-lane address, so the 64-bit
// add per load (v_lshl_add_u64) is gone; and its blur x alpha table is static LDS at address 0, its byte
// offset from the accumulator by ONE SDWA shift (byte 2 of acc times 8) instead of v_bfe_u32 +
// v_lshl_add_u32 (the dynamic LDS array's base is a link-time symbol the compiler adds to every index).
// Measured (round 4, 3 alternating rounds of the driver's command and 2 of config 5): both in k_pixw
// gain 1.9 % (80.9 vs 79.5 k frames/s, 3.07-3.12 vs 3.16-3.17 ms per launch); both in k_pix5 cost 3.4 %
// (396.0 vs 410.1 k frames/s), which keeps global loads.  (Round 5: the static table and SDWA offset alone in
// k_pix5, with its tap jobs' row pairs packed by v_perm: 430.3 vs 417.5 k, 4 alternating rounds; kept.  The
// buffer loads alone in k_pix5: 400-406 vs 414-428 k, 4 rounds; not kept.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint8_t* p, uint32_t bytes) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(p));
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uintptr_t>(p) >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)n, 0x00020000);
}
__device__ __forceinline__ void load12b(u32x3_t& d, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    d = __builtin_bit_cast(u32x3_t, __builtin_amdgcn_raw_buffer_load_b96(r, (int)off, 0, 0));
}
__device__ __forceinline__ gbytes_t frame_base(const uint8_t* p) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(p));
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uintptr_t>(p) >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (gbytes_t)(((uint64_t)hi << 32) | lo);
}

// Per-frame, per-wave constants of the chain stage (computed once per tile).
struct ChainCtx {
    uint64_t colmask;   // lanes whose column is inside the image
    uint32_t rowvalid;  // bit j: tile row 8*wv + j is inside the image
    uint32_t keep_lo, keep_hi;  // keep-mask bytes of the wave's 8 rows for this lane's column (1 = keep)
    uint32_t keep_2, keep_3;    // rows 8..15 of a 16-row wave (k_pix5<.., 4>)
    bool hk;            // stream has a keep-mask
    uint32_t vec;       // every pixel of the wave's rows lies in accumulateWeighted's vector body
    uint32_t tbmask;    // this lane's column inside the image ? rowvalid : 0
};

// One frame's vertical taps + per-pixel chain for the wave's 8 rows.
// INIT: the launch may hold a stream's first frame (bg := blur before the diff,
// fm.py:651-652); `init` says whether this frame is one.  KEEP: apply the
// keep-mask bytes (off when the stream has no mask).  TAIL: the wave's rows reach
// accumulateWeighted's scalar tail (per-pixel test of the product order).
template <int KC, bool PLANES, bool INIT, bool KEEP, bool TAIL>
__device__ __forceinline__ void chain_rows(const FusedArgs& a, const uint16_t* Hs, const double* atab, const Geo& g,
                                           double (&bg)[RPWV],
                                           int wv, int ln, int x0, int y0, size_t f, const ChainCtx& cc,
                                           bool init, uint32_t& colbits, uint32_t& flags) {
    constexpr int R = KC >> 1;
    constexpr int NV = RPWV + 2 * R;       // H rows feeding the wave's 8 outputs
    constexpr int NP = (NV + 1) / 2;       // u16 pairs
    const int w = a.w;
    // column ln of H, rows 8*wv .. 8*wv + NV - 1, as u16 pairs (ds_read_u16_d16 / _d16_hi)
    uint32_t P[NP + 1];
    {
        const uint16_t* col = Hs + (RPWV * wv) * g.RSH + ln;
#pragma unroll
        for (int i = 0; i < NP; i++) {
            u16x2_t v;
            v.x = col[(2 * i) * g.RSH];
            v.y = col[(2 * i + 1) * g.RSH];
            P[i] = __builtin_bit_cast(uint32_t, v);
        }
        P[NP] = 0;
    }
    const double beta = a.beta;
    // d in [0, 255]: with the threshold clamped to [-1, 255] (which keeps d > t), d + (255 - t)
    // is in [0, 511] and its bit 8 is d > t; v_sad_u8 adds the bias for free and one v_dot4 per
    // row moves that bit (byte 1 of the sum) to bit j of the lane's column byte
    const int thr = min(max(a.thresh, -1), 255);
    const uint32_t bias = (uint32_t)(255 - thr);
    uint32_t tb = 0;  // bit j: row 8*wv + j of this lane's column is over the threshold
    static_for<RPWV>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        // acc = sum_t c[t] * H[j + t] + 2^15 over u16 pairs (H[e], H[e+1]); blur = byte 2
        // (acc < 2^24), bytes 0-1 are the fraction
        uint32_t acc = 32768u;
#pragma unroll
        for (int t = 0; t < (KC + 1) / 2; t++) {
            const int e = j + 2 * t;
            const uint32_t pr = (e & 1) ? __builtin_amdgcn_alignbit(P[(e >> 1) + 1], P[e >> 1], 16) : P[e >> 1];
            acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, pr), __builtin_bit_cast(u16x2_t, tap2<KC>(t)), acc, false);
        }
        // keep bytes are 0xFF (keep) / 0x00 (masked off, fm.py:619-636): masked pixels blur to 0
        if (KEEP)
            acc &= (uint32_t)__builtin_amdgcn_sbfe(j < 4 ? (int)cc.keep_lo : (int)cc.keep_hi, 8 * (j & 3), 8);
        const uint32_t blur = acc >> 16;
        double b = bg[j];
        if (INIT && init) b = (double)blur;
        // convertScaleAbs: f64 -> f32 (rne), |.|, rne, saturate to u8 -- into byte 2 of a copy
        // of acc, so that the byte-wise absdiff of the two words is |blur - q|
        const uint32_t q = __builtin_amdgcn_cvt_pk_u8_f32(fabsf(__double2float_rn(b)), 2, acc);
        const uint32_t r = __builtin_amdgcn_sad_u8(acc, q, bias);  // absdiff + bias
        tb = __builtin_amdgcn_udot4(r, (1u << j) << 8, tb, false);
        // (double)blur * alpha from a 256-entry LDS table (the same correctly rounded product):
        // an LDS read instead of two f64-rate VALU ops per pixel
        const double bl = atab[blur];
        double nb = bg_fma(b, beta, bl);
        if (TAIL) {  // accumulateWeighted's scalar tail: two products, one add there
            const long long li = (long long)(y0 + RPWV * wv + j) * w + x0 + ln;
            if (li >= a.acc_vec_end) nb = __dadd_rn(bl, __dmul_rn(b, beta));
        }
        const bool rv = (cc.rowvalid >> j) & 1;
        bg[j] = nb;  // out-of-image pixels compute values that are never stored
        if (PLANES && rv && ((cc.colmask >> ln) & 1)) {
            const size_t plane = (size_t)a.h * w;
            const size_t li = (size_t)(y0 + RPWV * wv + j) * w + x0 + ln;
            a.planes[(size_t)a.T * a.S * plane + f * plane + li] = (uint8_t)blur;
            a.planes[2 * (size_t)a.T * a.S * plane + f * plane + li] = (uint8_t)(r - bias);
        }
    });
    // out-of-image pixels are background for the contour pass
    tb &= cc.tbmask;
    colbits = tb;
    // where the tile has threshold bits (decides the contour pass's candidate tiles):
    // any, within 2 px of the left / right edge, and for the tile's first / last two rows
    const uint64_t orr = __builtin_amdgcn_ballot_w64(tb != 0);
    const uint64_t top = wv == 0 ? __builtin_amdgcn_ballot_w64((tb & 3u) != 0) : 0ull;
    const uint64_t bot = wv == NW - 1 ? __builtin_amdgcn_ballot_w64((tb & (3u << (RPWV - 2))) != 0) : 0ull;
    uint32_t fl = 0;
    if (orr) fl = FLAG_ANY | ((orr & 3ull) ? FLAG_L : 0u) | ((orr >> 62) ? FLAG_R : 0u);
    if (wv == 0 && top) fl |= FLAG_T | ((top & 3ull) ? FLAG_TL : 0u) | ((top >> 62) ? FLAG_TR : 0u);
    if (wv == NW - 1 && bot) fl |= FLAG_B | ((bot & 3ull) ? FLAG_BL : 0u) | ((bot >> 62) ? FLAG_BR : 0u);
    flags = fl;
}

template <int KC, bool PLANES, bool INIT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu((!PLANES && !INIT && KC <= 7) ? kPixWPE : 1))) void k_pix(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int R = KC >> 1;
    const Geo g(R);
    uint8_t* raw = smem + g.o_raw;
    uint16_t* Hs = reinterpret_cast<uint16_t*>(smem + g.o_H);
    int* rowy = reinterpret_cast<int*>(smem + g.o_rowy);
    int* colx = reinterpret_cast<int*>(smem + g.o_colx);
    double* atab = reinterpret_cast<double*>(smem + g.o_atab);

    const int tid = threadIdx.x, ln = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = blockIdx.y;
    const int ti = swizzle_tile(blockIdx.x, a.ntiles);
    kstamp_begin(a.kstamp);
    // profiling only (FM_PTS): [hw_id | xcc_id << 32, realtime start, realtime end, memtime cycles]
    uint64_t* pts = (a.dbg_pts && tid == 0) ? a.dbg_pts + ((size_t)s * a.ntiles + ti) * 4 : nullptr;
    uint64_t rt0 = 0, mt0 = 0;
    if (pts) {
        pts[0] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
        rt0 = __builtin_amdgcn_s_memrealtime();
        mt0 = __builtin_amdgcn_s_memtime();
    }
    const int h = a.h, w = a.w, S = a.S;
    const int tx = ti % a.ntx, ty = ti / a.ntx;
    const int x0 = tx * TS, y0 = ty * TS;
    const size_t plane = (size_t)h * w;
    const size_t fbytes = plane * 3;
    const bool hk = a.has_keep[s] != 0;
    const uint8_t* keep = a.keep + (size_t)s * plane;
    const bool init0 = INIT && a.init != nullptr && a.init[s] != 0;
    // loaded source columns [cx0, cx1)
    const int gx0 = x0 - g.PC;
    const int cx0 = max(gx0, 0), cx1 = min(gx0 + g.GW, w);

    for (int i = tid; i < g.GH; i += NT) rowy[i] = reflect101(y0 - R + i, h);
    for (int i = tid; i < g.GW; i += NT) colx[i] = 3 * (min(max(reflect101(gx0 + i, w), cx0), cx1 - 1) - cx0);
    if (tid < 256) atab[tid] = __dmul_rn((double)tid, a.alpha);
    __syncthreads();

    // background of the wave's 8 rows x 64 columns -> registers; keep bytes likewise
    double bg[RPWV];
    ChainCtx cc;
    {
        const double* bgi = a.bg_in + (size_t)s * plane;
        const int x = x0 + ln;
        cc.colmask = __builtin_amdgcn_ballot_w64(x < w);
        cc.rowvalid = 0;
        cc.keep_lo = cc.keep_hi = 0;
        cc.hk = __builtin_amdgcn_readfirstlane(hk ? 1 : 0) != 0;  // wave-uniform (chooses the loop variant)
#pragma unroll
        for (int j = 0; j < RPWV; j++) {
            const int y = y0 + RPWV * wv + j;
            const bool in = x < w && y < h;
            if (y < h) cc.rowvalid |= 1u << j;
            bg[j] = (!init0 && in) ? bgi[(size_t)y * w + x] : 0.0;
            const uint32_t kb = (!hk || (in && keep[(size_t)y * w + x] != 0)) ? 0xFFu : 0u;
            if (j < 4) cc.keep_lo |= kb << (8 * j);
            else cc.keep_hi |= kb << (8 * (j - 4));
        }
        const long long last = (long long)(y0 + RPWV * wv + RPWV - 1) * w + x0 + TS - 1;
        cc.vec = (uint32_t)__builtin_amdgcn_readfirstlane(last < a.acc_vec_end ? 1 : 0);
        cc.tbmask = x < w ? cc.rowvalid : 0u;
    }
    // consume those loads here (the asm is a use, so the compiler waits before it):
    // inside the frame loop only the raw prefetch is then in flight and the chain
    // stage never waits for it
#pragma unroll
    for (int j = 0; j < RPWV; j++) asm volatile("" : "+v"(bg[j]));
    asm volatile("" : "+v"(cc.keep_lo), "+v"(cc.keep_hi));

    // horizontal stage geometry: lane -> (row group rg, gray quad q)
    constexpr int PCc = 4 * ((R + 3) / 4);
    constexpr int NQc = (TS + 2 * PCc) / 4;
    constexpr int GHc = TS + 2 * R;
    constexpr int RPW = 64 / NQc;
    constexpr int NIT = (GHc + RPW * NW - 1) / (RPW * NW);
    constexpr int OFF = PCc - R;
    constexpr int NQN = (3 + OFF + 2 * R) / 4 + 1;   // gray quads holding a quad's taps
    constexpr int NG = (KC + 3) / 4;                   // dot4 groups (last one zero padded)
    constexpr int NQW = (6 + OFF + 4 * (NG - 1)) / 4 + 1;  // quads the 4-byte windows touch
    const int rg = ln / NQc, q = ln - rg * NQc;
    // this lane's gray quad, columns [qc, qc + 4): the fast path needs it inside the
    // loaded columns (only the quads over a reflected image edge take the gather path)
    const int qc = gx0 + 4 * q;
    const bool qin = qc >= cx0 && qc + 4 <= cx1;
    // Quads over a reflected image edge (R <= 4, w % 4 == 0, w >= 8): the one quad just
    // outside the image on each side is rebuilt from the two mirrored inside quads by
    // lane shuffles (reflq 1 = left, 2 = right); quads further out feed only columns past
    // the image and keep whatever they read.  Those lanes read a clamped in-row quad.
    // Other geometries take the per-pixel gather below.
    const bool shfix = PCc == 4 && (w & 3) == 0 && w >= 8;
    const int reflq = !shfix ? 0 : qc == -4 ? 1 : qc == w ? 2 : 0;
    const bool qok = qin || (shfix && (reflq != 0 || qc >= w + 4));
    const int qoff = 3 * ((qin || !qok ? qc : qc < 0 ? cx0 : cx1 - 4) - cx0);
    const bool has_refl = shfix && (x0 == 0 || gx0 + g.GW > w);  // workgroup-uniform
    uint32_t cpk[NG];
#pragma unroll
    for (int gi = 0; gi < NG; gi++) cpk[gi] = tap4<KC>(gi);

    constexpr int NCH = (GHc * (a16(3 * (TS + 2 * PCc) + 15) / 16) + NT - 1) / NT;
    ChunkPlan<NCH> plan;
    plan_chunks(plan, rowy, g, cx0, w, tid);
    const uint32_t span = 3u * (uint32_t)(cx1 - cx0), fb32 = (uint32_t)fbytes;
    // ---- gray (4 px per lane) + horizontal taps of frame f -> transposed H (u16)
    // Lane (rg, q) of iteration it owns gray quad q of G row gy(it).  Frame-invariant
    // per-lane state: the row's byte offset in the frame (its 16-B aligned-down start
    // is where stage_raw put the row in LDS) and the G row index (clamped for idle lanes).
    uint32_t rowbyte[NIT], loff[NIT], hoff[NIT];
    int gyc[NIT];
    bool act[NIT];
#pragma unroll
    for (int it = 0; it < NIT; it++) {
        const int gy = (it * NW + wv) * RPW + rg;
        act[it] = rg < RPW && gy < GHc;
        gyc[it] = act[it] ? gy : 0;
        rowbyte[it] = (uint32_t)(rowy[gyc[it]] * w + cx0) * 3u;
        loff[it] = (uint32_t)(gyc[it] * g.RS + qoff);
        // H store target: lanes without an H quad (idle, or halo quads q >= 16) write the
        // pad row GH, which the vertical taps never read -- the store needs no predicate
        hoff[it] = (uint32_t)((act[it] && q < TS / 4 ? gyc[it] : GHc) * g.RSH + 4 * (q & (TS / 4 - 1)));
    }
    // rows of a 16-B multiple: every row starts at the same offset inside its first chunk
    const bool rows16 = (w * 3) % 16 == 0;
    auto gray_stage = [&](const uint8_t* rawb, uint16_t* Hb, size_t f) __attribute__((always_inline)) {
        const uint32_t flo = (uint32_t)(uintptr_t)(a.src + f * fbytes);
        uint32_t g4[NIT];
        bool slow = false;
        // straight-line over the iterations so their LDS round trips overlap
        if (rows16) {
            const uint32_t ro = (flo + 3u * (uint32_t)cx0) & 15u;  // uniform
            slow = act[0] && !(qok && ((ro + (uint32_t)qoff) & 3u) == 0);
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const uint32_t* p32 = reinterpret_cast<const uint32_t*>(rawb + ((loff[it] + ro) & ~3u));
                g4[it] = gray4(p32[0], p32[1], p32[2]);
            }
        } else {
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const uint32_t ro = (flo + rowbyte[it]) & 15u;  // row start inside its first 16-B chunk
                const uint32_t off = loff[it] + ro;
                slow |= act[it] && !(qok && (off & 3u) == 0);
                const uint32_t* p32 = reinterpret_cast<const uint32_t*>(rawb + (off & ~3u));
                g4[it] = gray4(p32[0], p32[1], p32[2]);
            }
        }
        if (__builtin_expect(slow, 0)) {  // reflected image edge or unaligned row: per-pixel gather
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const uint32_t ro = (flo + rowbyte[it]) & 15u;
                const uint32_t off = loff[it] + ro;
                if (act[it] && !(qok && (off & 3u) == 0)) {
                    const uint8_t* rowp = rawb + gyc[it] * g.RS + ro;
                    const int c0 = 4 * q;
                    g4[it] = gray1(rowp + colx[c0]) | (gray1(rowp + colx[c0 + 1]) << 8) |
                             (gray1(rowp + colx[c0 + 2]) << 16) | (gray1(rowp + colx[c0 + 3]) << 24);
                }
            }
        }
        if (has_refl) {  // reflected edge quads from the mirrored inside quads (see reflq)
            const int d = reflq == 1 ? 1 : reflq == 2 ? -1 : 0;
            const uint32_t sel = reflq == 1 ? 0x01020304u : 0x07000102u;
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const uint32_t A = (uint32_t)__builtin_amdgcn_ds_bpermute((ln + d) << 2, (int)g4[it]);
                const uint32_t B = (uint32_t)__builtin_amdgcn_ds_bpermute((ln + 2 * d) << 2, (int)g4[it]);
                if (reflq) g4[it] = __builtin_amdgcn_perm(B, A, sel);
            }
        }
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            if (PLANES && act[it]) {
                const int gy = gyc[it];
                const int y = y0 - R + gy, xq = gx0 + 4 * q;
                if (gy >= R && gy < R + TS && xq >= x0 && xq < x0 + TS && y < h) {
                    uint8_t* gp = a.planes + f * plane + (size_t)y * w;
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        if (xq + b < w) gp[xq + b] = (uint8_t)(g4[it] >> (8 * b));
                }
            }
            // neighbour quads q+1, q+2, ... by wavefront shifts (DPP wave_shl:1, lane i <- lane i+1);
            // across a row group's end they bring the next row's quads, which only feed halo lanes
            uint32_t qv[NQW];
            qv[0] = g4[it];
#pragma unroll
            for (int d = 1; d < NQW; d++)
                qv[d] = d < NQN ? (uint32_t)__builtin_amdgcn_mov_dpp((int)qv[d - 1], 0x130, 0xF, 0xF, true) : 0u;
            {
                const uint32_t h0 = htap<0, OFF, NG, 0, NQW>(qv, cpk, 0u);
                const uint32_t h1 = htap<1, OFF, NG, 0, NQW>(qv, cpk, 0u);
                const uint32_t h2 = htap<2, OFF, NG, 0, NQW>(qv, cpk, 0u);
                const uint32_t h3 = htap<3, OFF, NG, 0, NQW>(qv, cpk, 0u);
                // row-major: one conflict-free 8-B store of the quad's four taps
                *reinterpret_cast<uint2*>(Hb + hoff[it]) = make_uint2(h0 | (h1 << 16), h2 | (h3 << 16));
            }
        }
    };
    auto stage_raw = [&](const Raw<NCH>& Rr, int buf) __attribute__((always_inline)) { store_raw(Rr, raw + buf * g.raw_bytes, g, tid); };

    // Software pipeline, one barrier per frame: iteration t runs the chain of
    // frame t (H buffer t&1) and the gray/horizontal stage of frame t+1 (raw and
    // H buffers (t+1)&1), while frame t+2's raw tile is in flight into registers.
    const int t0 = a.t_begin, t1 = a.t_end;
    // profiling-only stage ablation (FM_DEBUG_SKIP bits; results invalid), 0 in normal use.
    // Kept as a runtime test on purpose: its branches bound the scheduler's live ranges
    // (117 VGPRs, measured 3 % faster than the branch-free build capped at 128)
    const int skip = __builtin_amdgcn_readfirstlane(a.dbg_skip);
    Raw<NCH> Rw;
    load_raw(Rw, a.src + ((size_t)t0 * S + s) * fbytes, fb32, plan, span);
    stage_raw(Rw, 0);
    if (t0 + 1 < t1) load_raw(Rw, a.src + ((size_t)(t0 + 1) * S + s) * fbytes, fb32, plan, span);
    lds_barrier();
    gray_stage(raw, Hs, (size_t)t0 * S + s);

    // the chain variant is fixed per wave for the whole launch: one loop instance each
    auto frame_loop = [&](auto keepc, auto tailc, const ChainCtx ccv) __attribute__((always_inline)) {
        constexpr bool KEEP = decltype(keepc)::value != 0, TAIL = decltype(tailc)::value != 0;
        for (int t = t0; t < t1; t++) {
            const int b = (t - t0) & 1;
            const size_t f = (size_t)t * S + s;
            if (t + 1 < t1) {
                if (!(skip & 8)) stage_raw(Rw, b ^ 1);
                if (t + 2 < t1 && !(skip & 4)) load_raw(Rw, a.src + (f + 2 * S) * fbytes, fb32, plan, span);
            }
            if (!(skip & 16)) lds_barrier();

            // ---- vertical taps + chain for the wave's 8 rows; threshold bits by ballot
            uint32_t colbits = 0;
            uint32_t fl = 0;
            // launder the per-tile uniforms each frame: otherwise LICM hoists dozens of
            // per-row exec masks out of the frame loop and they spill
            ChainCtx ccf = ccv;
            ccf.rowvalid = __builtin_amdgcn_readfirstlane(ccf.rowvalid);
            int x0f = __builtin_amdgcn_readfirstlane(x0), y0f = __builtin_amdgcn_readfirstlane(y0), wvf = wv;
            if constexpr (NT == 512) asm volatile("" : "+s"(ccf.colmask), "+s"(ccf.rowvalid), "+s"(x0f), "+s"(y0f), "+s"(wvf));
            asm volatile("" : "+v"(ccf.keep_lo), "+v"(ccf.keep_hi));
            if (!(skip & 2))
                chain_rows<KC, PLANES, INIT, KEEP, TAIL>(a, Hs + b * (g.H_bytes / 2), atab, g, bg, wvf, ln, x0f, y0f, f, ccf,
                                                         init0 && t == t0, colbits, fl);
            // column-major bit tile: word c of the tile = column c, bit r = row r; this wave
            // owns byte wv of every column word
            reinterpret_cast<uint8_t*>(a.bits)[((f * a.ntiles + ti) * TS + ln) * 8 + wv] = (uint8_t)colbits;
            // this wave's flag word, a plain store every frame (an atomic would sit in vmcnt
            // until the next frame's wait for the raw prefetch)
            if (ln == 0) a.tflag[(f * a.ntiles + ti) * NW + wv] = fl;

            if (t + 1 < t1 && !(skip & 1))
                gray_stage(raw + (b ^ 1) * g.raw_bytes, Hs + (b ^ 1) * (g.H_bytes / 2), f + S);
        }
    };
    if (!cc.vec) frame_loop(IntC<1>{}, IntC<1>{}, cc);
    else if (cc.hk) frame_loop(IntC<1>{}, IntC<0>{}, cc);
    else frame_loop(IntC<0>{}, IntC<0>{}, cc);

    // background out (ping-pong: neighbours never read this batch's update)
    double* bgo = a.bg_out + (size_t)s * plane;
    const int x = x0 + ln;
#pragma unroll
    for (int j = 0; j < RPWV; j++) {
        const int y = y0 + RPWV * wv + j;
        if (x < w && y < h) bgo[(size_t)y * w + x] = bg[j];
    }
    kstamp_end(a.kstamp);
    if (pts) {
        const uint64_t rt = __builtin_amdgcn_s_memrealtime(), mt = __builtin_amdgcn_s_memtime();
        pts[1] = rt0;
        pts[2] = rt;
        pts[3] = mt - mt0;
    }
}

// ---------------------------------------------------------------------------
// Geometry shared by k_pix5 and k_pixw (below): H as row pairs, the vertical taps over
// even-aligned pair windows (chain_rows_w), horizontal taps with shifted constants (HS).
template <int K> constexpr int tap_c(int t) { return t < 0 || t >= K ? 0 : Taps<K>::c[t]; }
template <int K> constexpr int tap_lo() {
    int i = 0;
    while (Taps<K>::c[i] == 0) i++;
    return i;
}
template <int K> constexpr int tap_hi() {
    int i = K - 1;
    while (Taps<K>::c[i] == 0) i--;
    return i;
}

// One 64-wide band of 8 waves per workgroup, each wave over RW rows: RW = 8, a 64 x 64 tile; RW = 16, a
// 64 x 128 band (two contour tiles), its 2R-row vertical halo loaded and filtered once per 128 rows.  (A
// 64 x 128 band of 16 waves of 8 rows: 3.61 vs 3.33 ms per config-5 launch, round 4.)
template <int KC, int RW_ = RPWV>
struct PW {
    static constexpr int NWB = 8;
    static constexpr int RW = RW_;                 // rows per wave
    static constexpr int R = KC / 2;
    static constexpr int PC = 4 * ((R + 3) / 4);   // gray columns each side of the tile (quad aligned)
    static constexpr int NTB = 64 * NWB;           // threads
    static constexpr int TH = RW * NWB;            // rows
    static constexpr int GH = TH + 2 * R;          // gray rows (even)
    static constexpr int GQ = (TS + 2 * PC) / 4;   // gray quads per row
    static constexpr int NG = GH * GQ;             // gray jobs per frame
    static constexpr int GSLOTS = (NG + 63) / 64;
    static constexpr int gcnt(int w) { return (GSLOTS - w + NWB - 1) / NWB; }  // gray slots of wave w: i * NWB + w
    static constexpr int GJ = gcnt(0);             // gray rounds per wave
    static constexpr int NHP = GH / 2;             // H row pairs
    static constexpr int NH = NHP * (TS / 4);      // tap jobs
    static constexpr int HJ = (NH + NTB - 1) / NTB;
    static constexpr int HLASTW = (NH - (HJ - 1) * NTB + 63) / 64;  // waves with a job in the last round
#ifndef FM_PIXW_GS
#define FM_PIXW_GS 24
#endif
    // gray row stride in LDS (dwords), 24 instead of GQ = 22: a tap job wave's four even gray rows start 48 dwords
    // apart, so their 16-quad windows fall in disjoint LDS banks (round 6, as in k_pix5)
    static constexpr int GS = FM_PIXW_GS > GQ ? FM_PIXW_GS : GQ;
    static constexpr int GBUF = GH * GS + 64;      // + a pad slot per lane (idle gray jobs)
    static constexpr int HBUF = (NHP + 1) * TS;    // u32 pairs + the pad pair row (idle tap jobs)
    static constexpr int LO = tap_lo<KC>(), HI = tap_hi<KC>();
    static constexpr int NGR = (HI - LO + 4) / 4;  // dot4 groups per output
    static constexpr int OFF = PC - R;             // byte of output k's tap 0 in its job's window: OFF + k
    static constexpr int WQ = (3 + OFF + LO + 4 * NGR - 1) / 4 + 1;  // gray dwords per row a tap job reads
    // chain: output row j of a wave takes pairs p0(j) .. p0(j) + np(j) - 1 (relative to the wave's first pair)
    static constexpr int p0(int j) { return (j + LO) >> 1; }
    static constexpr int np(int j) { return (j + HI + 2 - 2 * p0(j)) / 2; }
    static constexpr int np_max() {
        int m = 0;
        for (int j = 0; j < RW; j++) m = p0(j) + np(j) > m ? p0(j) + np(j) : m;
        return m;
    }
    static constexpr int NP = np_max();            // pairs a wave's chain reads
    static constexpr int bytes = 2 * GBUF * 4 + 2 * HBUF * 4 + 256 * 8;
    static constexpr int dyn_bytes = bytes - 256 * 8;  // (k_pixw: the table is static LDS)
};
template <int KC> constexpr uint32_t tapw4(int g) {  // dot4 group g of the non-zero taps
    uint32_t v = 0;
    for (int b = 0; b < 4; b++) {
        const int t = PW<KC>::LO + 4 * g + b;
        if (t <= PW<KC>::HI) v |= (uint32_t)Taps<KC>::c[t] << (8 * b);
    }
    return v;
}
template <int KC> constexpr uint32_t tapv2(int j, int i) {  // chain pair i of output row j: taps (ft, ft + 1)
    const int ft = 2 * (PW<KC>::p0(j) + i) - j;
    return (uint32_t)tap_c<KC>(ft) | (uint32_t)tap_c<KC>(ft + 1) << 16;
}

// chain_rows over H row pairs with even-aligned pair windows: output row j's window starts on an
// even H row, absorbing a zero tap (outside the kernel, or one of OpenCV's zero end taps) on the
// side the row parity needs, so no pair is rebuilt with v_alignbit
// wv: the wave within its workgroup = its 8-row slice of the 64-row tile (flag rows: FLAG_T* from slice 0,
// FLAG_B* from slice 7)
// pairs the chain of a RW-row wave reads
template <int KC, int RW> constexpr int np_rows() {
    int m = 0;
    for (int j = 0; j < RW; j++) m = PW<KC>::p0(j) + PW<KC>::np(j) > m ? PW<KC>::p0(j) + PW<KC>::np(j) : m;
    return m;
}

// RW: rows per wave (8, or 16 for k_pix5's 4-wave tiles and k_pixw's 128-row bands), NWT: waves per 64-row
// contour tile, BAND: waves of the workgroup (wv counts the band's waves; wv % NWT is the tile's slice)
template <int KC, bool KEEP, bool TAIL, bool SDWA, int RW = RPWV, int NWT = NW, int BAND = NWT>
__device__ __forceinline__ void chain_rows_w(const FusedArgs& a, const uint32_t* Hp, const double* atab, double (&bg)[RW],
                                             int wv, int ln, int x0, int y0, const ChainCtx& cc, uint32_t& colbits,
                                             uint32_t& flags) {
    using G = PW<KC>;
    static_assert(RW * NWT == TS && (RW == 8 || RW == 16), "rows per wave");
    constexpr int NPR = np_rows<KC, RW>();
    uint32_t P[NPR];
    const uint32_t* col = Hp + (RW / 2 * wv) * TS + ln;
#pragma unroll
    for (int i = 0; i < NPR; i++) P[i] = col[i * TS];
    const int w = a.w;
    const double beta = a.beta;
    const int thr = min(max(a.thresh, -1), 255);
    const uint32_t bias = (uint32_t)(255 - thr);
    uint32_t tb = 0, tb2 = 0;  // rows 0..7 / 8..15 (one dot4 moves a row's bit into byte 1 of the word)
    static_for<RW>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        uint32_t acc = 32768u;
        static_for<G::np(j)>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, P[G::p0(j) + i]),
                                         __builtin_bit_cast(u16x2_t, tapv2<KC>(j, i)), acc, false);
        });
        if (KEEP) {
            const uint32_t kw = j < 4 ? cc.keep_lo : j < 8 ? cc.keep_hi : j < 12 ? cc.keep_2 : cc.keep_3;
            acc &= (uint32_t)__builtin_amdgcn_sbfe((int)kw, 8 * (j & 3), 8);
        }
        // SDWA: the blur byte (byte 2: acc < 2^24) times 8, the table's byte offset, in ONE instruction
        // (the table must then be static LDS at address 0); else the blur value indexes the table
        uint32_t boff = 0, blur = 0;
        if constexpr (SDWA)
            asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
                : "=v"(boff) : "v"(acc));
        else
            blur = acc >> 16;
        const double b = bg[j];
        const uint32_t q = __builtin_amdgcn_cvt_pk_u8_f32(fabsf(__double2float_rn(b)), 2, acc);
        const uint32_t r = __builtin_amdgcn_sad_u8(acc, q, bias);
        if constexpr (j < 8) tb = __builtin_amdgcn_udot4(r, (1u << j) << 8, tb, false);
        else tb2 = __builtin_amdgcn_udot4(r, (1u << (j - 8)) << 8, tb2, false);
        const double bl = SDWA ? *reinterpret_cast<const double*>(reinterpret_cast<const char*>(atab) + boff)
                               : atab[blur];
        double nb = bg_fma(b, beta, bl);
        if (TAIL) {
            const long long li = (long long)(y0 + RW * wv + j) * w + x0 + ln;
            if (li >= a.acc_vec_end) nb = __dadd_rn(bl, __dmul_rn(b, beta));
        }
        bg[j] = nb;
    });
    if constexpr (RW > 8) tb |= tb2 << 8;
    tb &= cc.tbmask;
    colbits = tb;
    const int ws = BAND == NWT ? wv : wv % NWT;  // the wave's slice of its contour tile
    const uint64_t orr = __builtin_amdgcn_ballot_w64(tb != 0);
    const uint64_t top = ws == 0 ? __builtin_amdgcn_ballot_w64((tb & 3u) != 0) : 0ull;
    const uint64_t bot = ws == NWT - 1 ? __builtin_amdgcn_ballot_w64((tb & (3u << (RW - 2))) != 0) : 0ull;
    uint32_t fl = 0;
    if (orr) fl = FLAG_ANY | ((orr & 3ull) ? FLAG_L : 0u) | ((orr >> 62) ? FLAG_R : 0u);
    if (ws == 0 && top) fl |= FLAG_T | ((top & 3ull) ? FLAG_TL : 0u) | ((top >> 62) ? FLAG_TR : 0u);
    if (ws == NWT - 1 && bot) fl |= FLAG_B | ((bot & 3ull) ? FLAG_BL : 0u) | ((bot >> 62) ? FLAG_BR : 0u);
    flags = fl;
}

// Horizontal taps with the byte window folded into the constants: output k of a quad sums its
// taps over window bytes [B0 + k, B0 + k + NTAPS) of the row's gray dwords; instead of shifting
// the data (v_alignbyte per 4-byte group unless B0 + k is a multiple of 4), each aligned dword d
// of that range takes a dot4 with the taps shifted to where its bytes fall (zeros outside).
// k = 5: 8 dot4, no alignbyte per row of a quad (was 8 dot4 + 6 alignbyte).  The shifted tap words
// live in VGPRs (VOP3P takes no literal).  (k = 21 would need 22 such words instead of 20 dot4 + 15
// alignbyte: 128 VGPRs and spills in k_pixw, so it keeps the byte windows.)
template <int K>
struct HS {
    static constexpr int LO = tap_lo<K>(), NTAPS = tap_hi<K>() - LO + 1, B0 = PW<K>::OFF + LO;
    static constexpr int d0(int k) { return (B0 + k) / 4; }
    static constexpr int nd(int k) { return (B0 + k + NTAPS - 1) / 4 - d0(k) + 1; }
    static constexpr int base(int k) { return k == 0 ? 0 : base(k - 1) + nd(k - 1); }
    static constexpr int NC = base(4);
    static constexpr int NQ = (B0 + 3 + NTAPS - 1) / 4 + 1;  // dwords a row's 4 outputs read
    static constexpr uint32_t c(int k, int i) {
        uint32_t v = 0;
        const int d = d0(k) + i;
        for (int b = 0; b < 4; b++) {
            const int t = 4 * d + b - B0 - k;
            if (t >= 0 && t < NTAPS) v |= (uint32_t)Taps<K>::c[LO + t] << (8 * b);
        }
        return v;
    }
};
template <int K>
__device__ __forceinline__ void hs_consts(uint32_t (&cs)[HS<K>::NC]) {
    static_for<4>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        static_for<HS<K>::nd(k)>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            cs[HS<K>::base(k) + i] = HS<K>::c(k, i);
        });
    });
#pragma unroll
    for (int i = 0; i < HS<K>::NC; i++) asm volatile("" : "+v"(cs[i]));  // kept in VGPRs
}
template <int K, int k, int N>
__device__ __forceinline__ uint32_t hs_tap(const uint32_t (&q)[N], const uint32_t (&cs)[HS<K>::NC]) {
    static_assert(HS<K>::d0(k) + HS<K>::nd(k) <= N, "window dwords");
    uint32_t acc = 0;
    static_for<HS<K>::nd(k)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        acc = __builtin_amdgcn_udot4(q[HS<K>::d0(k) + i], cs[HS<K>::base(k) + i], acc, false);
    });
    return acc;
}

// ---------------------------------------------------------------------------
// k_pix5: the 5x5 steady-state chain (the bench configuration, and every k = 5
// run without planes) with gray computed where the frame is loaded.
//
// k_pix stages each frame's raw BGR tile in LDS and then converts it: every raw
// byte crosses LDS twice (a 16-B store, three 4-B reads per quad at a 12-B lane
// stride -- the gray stage's bank conflicts) and the 18 gray quads of a row are
// recomputed by the lanes that own the horizontal taps, so 24 wave-iterations of
// gray + taps cover 68 x 18 quad jobs.  Here:
//   gray  : a thread loads whole pixel quads (12 B, global_load_dwordx3) straight
//           into registers, two frames ahead, and turns them into one gray dword
//           (gray4) stored to LDS: 1224 quad jobs (68 rows x 18 quads) per frame;
//   taps  : 1088 jobs (68 rows x 16 quads) read three gray dwords each and store
//           the quad's four horizontal sums (u16) row-major, as k_pix does;
//   chain : k_pix's chain_rows on the 8 rows of each wave, unchanged.
// The image border: rows come from reflect101 source rows; a gray quad left of
// column 0 or right of the last column is never loaded, the taps rebuild the one
// quad just outside the image from the mirrored quad beside it (REFLECT_101).
// Needs w % 4 == 0 and w >= 8 (4-B aligned quads, one real quad each side);
// one barrier per frame as in k_pix.
// The chain runs on even-aligned pair windows (chain_rows_w); tap jobs cover 2 H rows x 4 columns and store
// them as row pairs (one ds_write_b128), which the chain reads back as six dwords instead of twelve u16
// reads and their merges; the horizontal taps take shifted constants (HS).
template <int NWB_ = 8>
struct P5G {
    static constexpr int NWB = NWB_;                     // waves of a tile (8 of 8 rows, or 4 of 16 rows)
    static constexpr int RW = TS / NWB;                  // rows per wave
    static constexpr int NTB = 64 * NWB;                 // threads
    static constexpr int TH = RW * NWB;                  // tile rows
    static constexpr int GH = TH + 4;                    // gray rows y0-2 .. y0+TH+1
    static constexpr int GQ = 18;                        // gray quads per row: columns x0-4 .. x0+67
#ifndef FM_P5_GS
#define FM_P5_GS 24
#endif
    // gray row stride in LDS (dwords): 24, not GQ = 18, so the four even gray rows a tap-job wave reads start 48
    // dwords apart and their windows fall in disjoint banks: LDS bank conflicts 176.3 M -> 68.2 M per 10-step run
    // (0.49 -> 0.19 per LDS-active cycle), throughput unchanged (round 6, profiles/r06/r06e_gray_stride_ab.txt)
    static constexpr int GS = FM_P5_GS > GQ ? FM_P5_GS : GQ;
    static constexpr int NG = GH * GQ;                   // gray jobs per frame
    // Gray jobs go to waves in whole wave-slots of 64 jobs.  Waves 4..7 lose issue arbitration to waves
    // 0..3 (age order) and set every frame's barrier (FM_PTS phase stamps: waves 0..3 spent ~30 % of
    // their cycles in the barrier), so waves 0..3 take GFAST slots each and waves 4..7 the rest; the
    // partial last slot goes to wave 3.  (GFAST A/B: 4 >= 3 > 5.)  Four waves: an even deal.
    static constexpr int GSLOTS = (NG + 63) / 64;
    static constexpr int GFAST = NWB == 8 ? 4 : (GSLOTS + NWB - 1) / NWB;
    static constexpr int GSLOW = NWB == 8 ? (GSLOTS - 4 * GFAST + 3) / 4 : 0;
    static constexpr int GJ = GFAST > GSLOW ? GFAST : GSLOW;  // load rounds per wave
    static constexpr int NH = (GH / 2) * (TS / 4);       // tap jobs per frame
    static constexpr int HJ = (NH + NTB - 1) / NTB;
    // the last job round is partial: only its first waves have jobs there (a wave-uniform branch)
    static constexpr int HLASTW = (NH - (HJ - 1) * NTB + 63) / 64;
    static constexpr int GBUF = GH * GS + 64;            // + a pad slot per lane for the idle jobs' stores (branch-free)
    static constexpr int HBUF = (GH + 2) * TS;           // u16; + the pad pair row idle tap jobs store to
    static constexpr int bytes = 2 * GBUF * 4 + 2 * HBUF * 2 + 256 * 8;
    static constexpr int dyn_bytes = bytes - 256 * 8;  // (the table is static LDS)
};
static_assert(P5G<8>::GSLOW >= 0 && 4 * (P5G<8>::GFAST + P5G<8>::GSLOW) >= P5G<8>::GSLOTS, "gray slots");
static_assert(4 * P5G<4>::GFAST >= P5G<4>::GSLOTS, "gray slots");

template <int GJ>
struct P5Raw {
    u32x3_t v[GJ];  // one 96-bit value per job: one register triple the allocator keeps whole
};

// KEEP: some stream has a keep-mask (streams without one get all-keep bytes); TAIL: the image has
// accumulateWeighted's scalar tail (h*w % 16 != 0), so some waves take the per-pixel test.  Fixed
// per launch, so the common kernel has a single chain path: a per-wave 3-way branch inside the
// frame loop made the background registers a phi and cost 8 v_mov_b64 per frame.
// Measured and withdrawn (round 4): 8- / 16-row bands for small images, two tiles per 1,024-thread
// workgroup sharing the frame barrier, issue priority falling with progress, chain and producer waves
// (DESIGN.md §3.1c); round 5: a wave-private variant without the frame barrier (k_pixq, each wave's own
// gray and taps over its 12 rows: 345-357 vs 383-418 k frames/s) -- small images now take fm_small.hip.
template <bool KEEP, bool TAIL, int NWB = 8>
__global__ __launch_bounds__(64 * NWB) __attribute__((amdgpu_waves_per_eu(kPixWPE))) void k_pix5(FusedArgs a) {
    using G = P5G<NWB>;
    constexpr int RW = G::RW;
    constexpr int GJX = G::GJ, HJX = G::HJ;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int KC = 5, R = 2;
    uint32_t* gray = reinterpret_cast<uint32_t*>(smem);                          // [2][G::GBUF]
    uint16_t* Hs = reinterpret_cast<uint16_t*>(smem + 2 * G::GBUF * 4);          // [2][G::HBUF]
    // blur x alpha (f64) as static LDS at address 0: the chain's table offset is ONE SDWA shift of the
    // accumulator (byte 2 times 8) instead of v_bfe_u32 + v_lshl_add_u32 with the dynamic array's base
    __shared__ double atab_s[256];
    double* atab = atab_s;
    const int tid = (int)threadIdx.x, ln = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = blockIdx.y;
    const int h = a.h, w = a.w, S = a.S;
    const int ti = swizzle_tile(blockIdx.x, a.ntiles);  // contour tile
    const int tx = ti % a.ntx;
    const int y0 = (ti / a.ntx) * TS;
    const int x0 = tx * TS;
    const size_t plane = (size_t)h * w;
    const size_t fbytes = plane * 3;
    const bool hk = a.has_keep[s] != 0;
    const uint8_t* keep = a.keep + (size_t)s * plane;
    if (tid < 256) atab[tid] = __dmul_rn((double)tid, a.alpha);
    kstamp_begin(a.kstamp);
#ifdef FM_DEV_SWITCHES
    // profiling only (FM_PTS, dev build): [hw_id | xcc_id << 32, realtime start, realtime end, memtime cycles]
    uint64_t* pts = (a.dbg_pts && tid == 0) ? a.dbg_pts + ((size_t)s * a.ntiles + ti) * 4 : nullptr;
    uint64_t rt0 = 0, mt0 = 0;
    if (pts) {
        pts[0] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
        rt0 = __builtin_amdgcn_s_memrealtime();
        mt0 = __builtin_amdgcn_s_memtime();
    }
#endif

    // ---- per-thread job plans (frame invariant)
    uint32_t goff[GJX];   // byte offset of the job's quad in a frame (0 for jobs that load nothing)
    uint32_t gdst[GJX];   // its gray dword in a buffer (the lane's pad slot for idle jobs)
    // this wave's gray slots (wave-uniform): the 4 / 4 deal
    const int gjobs = NWB == 8 ? (wv < 4 ? G::GFAST : G::GSLOW) : min(G::GFAST, G::GSLOTS - wv * G::GFAST);
#pragma unroll
    for (int i = 0; i < GJX; i++) {
        const int slot = NWB != 8 ? wv * G::GFAST + i : wv >= 4 ? (wv - 4) * G::GSLOW + i : 4 * G::GSLOW + wv * G::GFAST + i;
        const int j = i < gjobs ? slot * 64 + ln : G::NG;  // rounds past the wave's slots: idle (dummy load)
        const int gr = j / G::GQ, gq = j - gr * G::GQ;
        const int x = x0 - 4 + 4 * gq;
        const bool live = j < G::NG && x >= 0 && x + 4 <= w;
        const int y = reflect101(y0 - R + gr, h);
        goff[i] = live ? (uint32_t)(((size_t)y * w + x) * 3) : 0u;
        gdst[i] = j < G::NG ? (uint32_t)(G::GS == G::GQ ? j : gr * G::GS + gq) : (uint32_t)(G::GH * G::GS + ln);
    }
    uint32_t hsrc[HJX], hdst[HJX];
#pragma unroll
    for (int i = 0; i < HJX; i++) {
        const int j = tid + G::NTB * i;
        const bool live = j < G::NH;
        const int hr = live ? j / (TS / 4) : 0, hq = live ? j - hr * (TS / 4) : 0;
        hsrc[i] = (uint32_t)(2 * hr * G::GS + hq);
        hdst[i] = (uint32_t)((live ? hr : G::GH / 2) * TS + 4 * hq);  // u32 index of the pair's 4 columns
    }
    // REFLECT_101 quads: left of column 0 (tile x0 = 0, tap quad 0 reads gray quad 0 = columns -4..-1:
    // bytes 2, 3 = gray(2), gray(1) from quad 1) and the quad starting at column w (bytes 0, 1 =
    // gray(w-2), gray(w-3) from the quad before it); further quads feed only columns past the image
    const bool edge_tile = x0 == 0 || x0 + TS + 4 > w;  // workgroup-uniform
    const int vq = (w - x0 + 4) / 4;  // gray quad index of the quad starting at column w
    uint32_t hfix[HJX];  // bit0: q0 := mirror of q1 (left); bit1: q1 := mirror of q0; bit2: q2 := mirror of q1
#pragma unroll
    for (int i = 0; i < HJX; i++) {
        const int hq = (int)(hsrc[i] % G::GS);
        hfix[i] = (x0 == 0 && hq == 0 ? 1u : 0u) | (hq + 1 == vq ? 2u : 0u) | (hq + 2 == vq ? 4u : 0u);
    }

    // background of the wave's 8 rows x 64 columns -> registers (as k_pix)
    double bg[RW];
    ChainCtx cc;
    {
        const double* bgi = a.bg_in + (size_t)s * plane;
        const int x = x0 + ln;
        cc.colmask = __builtin_amdgcn_ballot_w64(x < w);
        cc.rowvalid = 0;
        cc.keep_lo = cc.keep_hi = cc.keep_2 = cc.keep_3 = 0;
        cc.hk = __builtin_amdgcn_readfirstlane(hk ? 1 : 0) != 0;
#pragma unroll
        for (int j = 0; j < RW; j++) {
            const int y = y0 + RW * wv + j;
            const bool in = x < w && y < h;
            if (y < h) cc.rowvalid |= 1u << j;
            bg[j] = in ? bgi[(size_t)y * w + x] : 0.0;
            const uint32_t kb = (!hk || (in && keep[(size_t)y * w + x] != 0)) ? 0xFFu : 0u;
            if (j < 4) cc.keep_lo |= kb << (8 * j);
            else if (j < 8) cc.keep_hi |= kb << (8 * (j - 4));
            else if (j < 12) cc.keep_2 |= kb << (8 * (j - 8));
            else cc.keep_3 |= kb << (8 * (j - 12));
        }
        const long long last = (long long)(y0 + RW * wv + RW - 1) * w + x0 + TS - 1;
        cc.vec = (uint32_t)__builtin_amdgcn_readfirstlane(last < a.acc_vec_end ? 1 : 0);
        cc.tbmask = x < w ? cc.rowvalid : 0u;
    }
#pragma unroll
    for (int j = 0; j < RW; j++) asm volatile("" : "+v"(bg[j]));
    asm volatile("" : "+v"(cc.keep_lo), "+v"(cc.keep_hi));
    if constexpr (RW > 8) asm volatile("" : "+v"(cc.keep_2), "+v"(cc.keep_3));

    uint32_t hcs[HS<KC>::NC];
    hs_consts<KC>(hcs);
    P5Raw<GJX> rw;
    // Every wave issues every job's load, idle jobs included (they read the frame's first
    // 12 B): a load under a branch makes its registers a phi of the loaded and the old
    // value, and the copies the compiler then inserts at the loop back-edge wait for the
    // load (vmcnt(0)), so the prefetch would not stay in flight across the frame barrier.
    auto load = [&](size_t f) __attribute__((always_inline)) {
        const gbytes_t src = frame_base(a.src + f * fbytes);
#pragma unroll
        for (int i = 0; i < GJX; i++) load12(rw.v[i], src, goff[i]);  // global_load_dwordx3 (4-B aligned)
    };
    auto gray_stage = [&](uint32_t* gb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < GJX; i++) {
            if (i >= gjobs) break;  // wave-uniform
            gb[gdst[i]] = gray4(rw.v[i].x, rw.v[i].y, rw.v[i].z);
        }
    };
    auto tap_stage = [&](const uint32_t* gb, uint16_t* Hb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < HJX; i++) {
            if (i == G::HJ - 1 && wv >= G::HLASTW) break;  // wave-uniform
            // (qv[3]: the last tap group's window reaches one byte into it, with zero taps there)
            uint32_t qv[4] = {gb[hsrc[i]], gb[hsrc[i] + 1], gb[hsrc[i] + 2], 0u};
            if (edge_tile) {
                if (hfix[i] & 1) qv[0] = __builtin_amdgcn_perm(qv[1], qv[1], 0x01020000u);
                if (hfix[i] & 2) qv[1] = __builtin_amdgcn_perm(qv[0], qv[0], 0x00000102u);
                if (hfix[i] & 4) qv[2] = __builtin_amdgcn_perm(qv[1], qv[1], 0x00000102u);
            }
            // outputs x0+4q+k, k = 0..3: taps over gray columns x0+4q+k-2 .. +2 = bytes k+2 .. k+6 of qv
            const uint32_t h0 = hs_tap<KC, 0>(qv, hcs);
            const uint32_t h1 = hs_tap<KC, 1>(qv, hcs);
            const uint32_t h2 = hs_tap<KC, 2>(qv, hcs);
            const uint32_t h3 = hs_tap<KC, 3>(qv, hcs);
            // the next gray row, then both rows' sums as row pairs
            uint32_t qw[4] = {gb[hsrc[i] + G::GS], gb[hsrc[i] + G::GS + 1], gb[hsrc[i] + G::GS + 2], 0u};
            if (edge_tile) {
                if (hfix[i] & 1) qw[0] = __builtin_amdgcn_perm(qw[1], qw[1], 0x01020000u);
                if (hfix[i] & 2) qw[1] = __builtin_amdgcn_perm(qw[0], qw[0], 0x00000102u);
                if (hfix[i] & 4) qw[2] = __builtin_amdgcn_perm(qw[1], qw[1], 0x00000102u);
            }
            const uint32_t k0 = hs_tap<KC, 0>(qw, hcs);
            const uint32_t k1 = hs_tap<KC, 1>(qw, hcs);
            const uint32_t k2 = hs_tap<KC, 2>(qw, hcs);
            const uint32_t k3 = hs_tap<KC, 3>(qw, hcs);
            // row pairs by one v_perm each (every sum < 2^16) instead of a shift and an or
            *reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(Hb) + hdst[i]) =
                make_uint4(__builtin_amdgcn_perm(k0, h0, 0x05040100u), __builtin_amdgcn_perm(k1, h1, 0x05040100u),
                           __builtin_amdgcn_perm(k2, h2, 0x05040100u), __builtin_amdgcn_perm(k3, h3, 0x05040100u));
        }
    };
    const int t0 = a.t_begin, t1 = a.t_end;
    // All work after the frame's barrier: chain(t), taps(t+1), gray(t+2), then the load of frame
    // t+3 into the registers gray(t+2) just consumed (one iteration in flight).  Loads are
    // unconditional, frame indices clamped to the batch (see load).
    load((size_t)t0 * S + s);
    gray_stage(gray);
    load((size_t)min(t0 + 1, t1 - 1) * S + s);
    __syncthreads();  // atab, gray(t0)
    tap_stage(gray, Hs);
    if (t0 + 1 < t1) gray_stage(gray + G::GBUF);
    load((size_t)min(t0 + 2, t1 - 1) * S + s);

    // ONE frame loop: the chain variant (keep-mask, accumulateWeighted's scalar tail) is a
    // wave-uniform branch inside it, re-read every frame so that the loop is not unswitched.
    // Three loop copies would give the in-flight loads different registers in each, and the
    // wait pass would then wait for them at the top of every frame.
    const int var0 = TAIL ? (int)(cc.vec == 0) : 0;  // (cc.vec is wave-uniform)
    auto frame = [&](int t, int b) __attribute__((always_inline)) {
            const size_t f = (size_t)t * S + s;
            lds_barrier();
            uint32_t colbits = 0, fl = 0;
            ChainCtx ccf = cc;
            ccf.rowvalid = __builtin_amdgcn_readfirstlane(ccf.rowvalid);
            int x0f = __builtin_amdgcn_readfirstlane(x0), y0f = __builtin_amdgcn_readfirstlane(y0), wvf = wv, var = var0;
            asm volatile("" : "+s"(ccf.colmask), "+s"(ccf.rowvalid), "+s"(x0f), "+s"(y0f), "+s"(wvf));
            var = __builtin_amdgcn_readfirstlane(var);
            if constexpr (KEEP) asm volatile("" : "+v"(ccf.keep_lo), "+v"(ccf.keep_hi));
            if constexpr (KEEP && RW > 8) asm volatile("" : "+v"(ccf.keep_2), "+v"(ccf.keep_3));
            const uint32_t* Hp = reinterpret_cast<const uint32_t*>(Hs + b * G::HBUF);
            if (!TAIL || var == 0)
                chain_rows_w<KC, KEEP, false, true, RW, NWB>(a, Hp, atab, bg, wvf, ln, x0f, y0f, ccf, colbits, fl);
            else
                chain_rows_w<KC, KEEP, true, true, RW, NWB>(a, Hp, atab, bg, wvf, ln, x0f, y0f, ccf, colbits, fl);
            if (t + 1 < t1) tap_stage(gray + (b ^ 1) * G::GBUF, Hs + (b ^ 1) * G::HBUF);
            // unconditional like the loads (past the batch's end it fills a buffer nothing reads):
            // a skipped gray stage leaves the loads unwaited on that path, and the wait pass then
            // makes every frame wait for the stores below before the next loads
            gray_stage(gray + b * G::GBUF);
            // the frame's bits and flag word, stored after gray(t+2) consumed the loads and before
            // the next ones: vmcnt counts stores and loads in issue order, so stores issued after
            // the prefetch would be waited for with it
            if constexpr (RW == 8) {
                reinterpret_cast<uint8_t*>(a.bits)[((f * a.ntiles + ti) * TS + ln) * 8 + wv] = (uint8_t)colbits;
                if (ln == 0) a.tflag[(f * a.ntiles + ti) * NW + wv] = fl;
            } else {  // bytes 2wv, 2wv + 1 of the column word; flag words 2wv (this wave's) and 2wv + 1 (none)
                reinterpret_cast<uint16_t*>(a.bits)[((f * a.ntiles + ti) * TS + ln) * 4 + wv] = (uint16_t)colbits;
                if (ln == 0) *reinterpret_cast<uint2*>(a.tflag + (f * a.ntiles + ti) * NW + 2 * wv) = make_uint2(fl, 0u);
            }
            // unconditional (see load): past the batch's last frame it re-reads that frame
            load((size_t)min(t + 3, t1 - 1) * S + s);
    };
    for (int t = t0; t < t1; t++) frame(t, (t - t0) & 1);

    double* bgo = a.bg_out + (size_t)s * plane;
    const int x = x0 + ln;
#pragma unroll
    for (int j = 0; j < RW; j++) {
        const int y = y0 + RW * wv + j;
        if (x < w && y < h) bgo[(size_t)y * w + x] = bg[j];
    }
    kstamp_end(a.kstamp);
#ifdef FM_DEV_SWITCHES
    if (pts) {
        const uint64_t rt = __builtin_amdgcn_s_memrealtime(), mt = __builtin_amdgcn_s_memtime();
        pts[1] = rt0;
        pts[2] = rt;
        pts[3] = mt - mt0;
    }
#endif
}

// ---------------------------------------------------------------------------
// k_pixw<KC>: k_pix5's decomposition for wide Gaussians (KC = 21: config 5's -B 3840 -b 183,
// fm.py:478-484).  k_pix<21> staged raw BGR in LDS, recomputed each gray quad in every lane
// that needed it and ran a 28-row u16 column per lane through alignbit + dot2 (168 VGPRs, 81
// SGPR spills, ~90 VALU lane-ops per pixel-frame, one workgroup per CU).  Here, as in k_pix5:
//   gray  : 12-B pixel quads loaded straight into registers one frame ahead, one gray dword per
//           job into LDS: (64 + 2R) rows x (16 + 2 PC / 4) quads per frame;
//   taps  : one job = 2 H rows x 4 columns; only the non-zero taps (OpenCV's k = 21 taps end in
//           zeros) as v_dot4 groups over byte windows; stored as row pairs (one ds_write_b128);
//   chain : per output row the pairs start on an even H row, choosing which zero tap of the
//           window the pair grid absorbs (row parity), so no alignbit; the rest is chain_rows.
// REFLECT_101 columns: quads left of column 0 / right of column w-1 are never loaded; on the
// two edge tiles of a tile row the tap jobs rebuild them from the mirrored inside quads (one
// v_perm of two gray dwords: quad at column c < 0 holds gray(-c .. -c-3), at c >= w gray(2w-2-c ..)).
// Rows: reflect101 source rows, as k_pix5.  Needs w % 4 == 0 and w >= 2 * PC + 8.
// 2 workgroups per CU (<= 128 VGPRs).  (8 chain + 4 producer waves per tile, as k_pix5's SPL: 57.8 vs
// 79.0 k frames/s at config 5, round 4.)
#ifndef FM_PIXW_WPE
#define FM_PIXW_WPE kPixWPE
#endif
template <int KC, bool KEEP, bool TAIL, int RW = RPWV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(RW == 16 ? FM_PIXW_WPE : kPixWPE))) void k_pixw(FusedArgs a) {
    using G = PW<KC, RW>;
    constexpr int TPB = RW / RPWV;  // contour tiles per band (stacked vertically)
    constexpr int GJX = G::GJ, HJX = G::HJ;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int R = G::R, PC = G::PC, GQ = G::GQ;
    uint32_t* gray = reinterpret_cast<uint32_t*>(smem);                          // [2][GBUF]
    uint32_t* Hs = reinterpret_cast<uint32_t*>(smem + 2 * G::GBUF * 4);          // [2][HBUF]
    __shared__ double atab_s[256];  // blur x alpha (f64), static LDS at address 0 (the SDWA table offset)
    double* atab = atab_s;
    const int tid = threadIdx.x, ln = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = blockIdx.y;
    const int h = a.h, w = a.w, S = a.S;
    // the band (TPB == 1: the contour tile); this wave's contour tile (TPB == 2: the upper one for waves 0..3),
    // past the grid in a last half band
    const int bi = swizzle_tile(blockIdx.x, TPB == 1 ? a.ntiles : a.ntx * ((a.nty + TPB - 1) / TPB));
    const int tx = bi % a.ntx;
    const int y0 = (bi / a.ntx) * G::TH;
    const int x0 = tx * TS;
    const int tyw = (bi / a.ntx) * TPB + (TPB == 1 ? 0 : (wv >> 2));
    const bool tile_ok = TPB == 1 || tyw < a.nty;
    const int ti = TPB == 1 ? bi : tyw * a.ntx + tx;
    const size_t plane = (size_t)h * w;
    const size_t fbytes = plane * 3;
    const bool hk = a.has_keep[s] != 0;
    const uint8_t* keep = a.keep + (size_t)s * plane;
    if (tid < 256) atab[tid] = __dmul_rn((double)tid, a.alpha);
    kstamp_begin(a.kstamp);

    // ---- per-thread job plans (frame invariant).  (Recomputed where used instead of held in 23 registers -- 99
    // instead of 119 VGPRs, so a detector or contour wave fits beside two band workgroups -- the launch took 25 %
    // longer: round 6, profiles/r06/r06j_replan_ab.txt.)
    const int gcnt_w = G::gcnt(wv);
    auto gplan = [&](int i, int lnv, uint32_t& go, uint32_t& gd) __attribute__((always_inline)) {
        const int slot = i * G::NWB + wv;
        const int j = (i < gcnt_w && slot < G::GSLOTS) ? slot * 64 + lnv : G::NG;  // idle: dummy load
        const int gr = j / GQ, gq = j - gr * GQ;
        const int x = x0 - PC + 4 * gq;
        const bool live = j < G::NG && x >= 0 && x + 4 <= w;
        const int y = reflect101(y0 - R + gr, h);
        go = live ? (uint32_t)(((size_t)y * w + x) * 3) : 0u;
        gd = j < G::NG ? (uint32_t)(gr * G::GS + gq) : (uint32_t)(G::GH * G::GS + lnv);
    };
    auto hplan = [&](int i, int tidv, uint32_t& hs, uint32_t& hd, int& hq_) __attribute__((always_inline)) {
        const int j = tidv + G::NTB * i;
        const bool live = j < G::NH;
        const int hp = live ? j / (TS / 4) : 0, hq = live ? j - hp * (TS / 4) : 0;
        hq_ = hq;
        hs = (uint32_t)(2 * hp * G::GS + hq);
        hd = (uint32_t)((live ? hp : G::NHP) * TS + 4 * hq);
    };
    uint32_t goff[GJX], gdst[GJX], hsrc[HJX], hdst[HJX];
    int hqv[HJX];
#pragma unroll
    for (int i = 0; i < GJX; i++) gplan(i, ln, goff[i], gdst[i]);
#pragma unroll
    for (int i = 0; i < HJX; i++) hplan(i, tid, hsrc[i], hdst[i], hqv[i]);
    const int gjobs = __builtin_amdgcn_readfirstlane(gcnt_w);  // this wave's gray rounds
    const bool edge_tile = x0 - PC < 0 || x0 + TS + PC > w;  // workgroup-uniform

    double bg[RW];
    ChainCtx cc;
    {
        const double* bgi = a.bg_in + (size_t)s * plane;
        const int x = x0 + ln;
        cc.colmask = __builtin_amdgcn_ballot_w64(x < w);
        cc.rowvalid = 0;
        cc.keep_lo = cc.keep_hi = cc.keep_2 = cc.keep_3 = 0;
        cc.hk = __builtin_amdgcn_readfirstlane(hk ? 1 : 0) != 0;
#pragma unroll
        for (int j = 0; j < RW; j++) {
            const int y = y0 + RW * wv + j;
            const bool in = x < w && y < h;
            if (y < h) cc.rowvalid |= 1u << j;
            bg[j] = in ? bgi[(size_t)y * w + x] : 0.0;
            const uint32_t kb = (!hk || (in && keep[(size_t)y * w + x] != 0)) ? 0xFFu : 0u;
            if (j < 4) cc.keep_lo |= kb << (8 * j);
            else if (j < 8) cc.keep_hi |= kb << (8 * (j - 4));
            else if (j < 12) cc.keep_2 |= kb << (8 * (j - 8));
            else cc.keep_3 |= kb << (8 * (j - 12));
        }
        const long long last = (long long)(y0 + RW * wv + RW - 1) * w + x0 + TS - 1;
        cc.vec = (uint32_t)__builtin_amdgcn_readfirstlane(last < a.acc_vec_end ? 1 : 0);
        cc.tbmask = x < w ? cc.rowvalid : 0u;
    }
#pragma unroll
    for (int j = 0; j < RW; j++) asm volatile("" : "+v"(bg[j]));
    asm volatile("" : "+v"(cc.keep_lo), "+v"(cc.keep_hi));
    if constexpr (RW > 8) asm volatile("" : "+v"(cc.keep_2), "+v"(cc.keep_3));

    uint32_t cpk[G::NGR];
#pragma unroll
    for (int gi = 0; gi < G::NGR; gi++) cpk[gi] = tapw4<KC>(gi);
    u32x3_t rw[GJX];
    // unconditional loads (idle jobs read the frame's first 12 B), as in k_pix5: a load under a
    // branch would make its registers a phi and the prefetch would be waited for at the back-edge
    auto load = [&](size_t f) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t rs = frame_rsrc(a.src + f * fbytes, (uint32_t)fbytes);
#pragma unroll
        for (int i = 0; i < GJX; i++) load12b(rw[i], rs, goff[i]);  // buffer_load_dwordx3, SGPR descriptor
    };
    auto gray_stage = [&](uint32_t* gb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < GJX; i++) {
            if (i >= gjobs) break;  // wave-uniform
            gb[gdst[i]] = gray4(rw[i].x, rw[i].y, rw[i].z);
        }
    };
    // (The horizontal taps as v_mfma_i32_16x16x64_i8 -- 5 blocks of 16 H rows x 16 columns per wave-frame instead of
    // the dot4 tap jobs, bit-exact on the GPU suite -- ran 6 % longer per configs[4] launch; round 6,
    // profiles/r06/r06g_mfma_taps_ab.txt.)
    // one row of a tap job: the quad's 4 horizontal sums from WQ gray dwords (edge tiles: the
    // mirrored quads rebuilt first)
    auto hrow = [&](const uint32_t* row, int hq, uint32_t (&o)[4]) __attribute__((always_inline)) {
        uint32_t qv[G::WQ];
#pragma unroll
        for (int d = 0; d < G::WQ; d++) qv[d] = row[hq + d];
        if (edge_tile) {
            // laundered so the mirror indices are computed here, on the edge tiles only, and not
            // hoisted out of the frame loop into ~30 registers every tile would carry
            int hqe = hq, xe = x0 - PC;
            asm volatile("" : "+v"(hqe), "+v"(xe));
#pragma unroll
            for (int d = 0; d < G::WQ; d++) {
                const int c = xe + 4 * (hqe + d);
                if (c < 0 || c >= w) {
                    const int sp = c < 0 ? -(c + 3) : 2 * w - 5 - c;  // first of the 4 mirrored source pixels
                    const int qa = min(max((sp - (x0 - PC)) >> 2, 0), GQ - 2);
                    qv[d] = __builtin_amdgcn_perm(row[qa + 1], row[qa], c < 0 ? 0x01020304u : 0x03040506u);
                }
            }
        }
        o[0] = htap<0, G::OFF + G::LO, G::NGR, 0, G::WQ>(qv, cpk, 0u);
        o[1] = htap<1, G::OFF + G::LO, G::NGR, 0, G::WQ>(qv, cpk, 0u);
        o[2] = htap<2, G::OFF + G::LO, G::NGR, 0, G::WQ>(qv, cpk, 0u);
        o[3] = htap<3, G::OFF + G::LO, G::NGR, 0, G::WQ>(qv, cpk, 0u);
    };
    auto tap_stage = [&](const uint32_t* gb, uint32_t* Hb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < HJX; i++) {
            if (i == G::HJ - 1 && wv >= G::HLASTW) break;  // wave-uniform
            const uint32_t hs = hsrc[i], hd = hdst[i];
            const int hq = hqv[i];
            const uint32_t* r0 = gb + (hs - hq);
            uint32_t u[4], v[4];
            hrow(r0, hq, u);
            hrow(r0 + G::GS, hq, v);
            *reinterpret_cast<uint4*>(Hb + hd) = make_uint4(u[0] | (v[0] << 16), u[1] | (v[1] << 16),
                                                             u[2] | (v[2] << 16), u[3] | (v[3] << 16));
        }
    };
    const int t0 = a.t_begin, t1 = a.t_end;
    load((size_t)t0 * S + s);
    gray_stage(gray);
    load((size_t)min(t0 + 1, t1 - 1) * S + s);
    __syncthreads();  // atab, gray(t0)
    tap_stage(gray, Hs);
    if (t0 + 1 < t1) gray_stage(gray + G::GBUF);
    load((size_t)min(t0 + 2, t1 - 1) * S + s);
    const int var0 = TAIL ? (int)(cc.vec == 0) : 0;
    for (int t = t0; t < t1; t++) {
        const int b = (t - t0) & 1;
        const size_t f = (size_t)t * S + s;
        lds_barrier();
        uint32_t colbits = 0, fl = 0;
        ChainCtx ccf = cc;
        ccf.rowvalid = __builtin_amdgcn_readfirstlane(ccf.rowvalid);
        int x0f = __builtin_amdgcn_readfirstlane(x0), y0f = __builtin_amdgcn_readfirstlane(y0), wvf = wv, var = var0;
        asm volatile("" : "+s"(ccf.colmask), "+s"(ccf.rowvalid), "+s"(x0f), "+s"(y0f), "+s"(wvf));
        var = __builtin_amdgcn_readfirstlane(var);
        asm volatile("" : "+v"(ccf.keep_lo), "+v"(ccf.keep_hi));
        if constexpr (RW > 8) asm volatile("" : "+v"(ccf.keep_2), "+v"(ccf.keep_3));
        const uint32_t* Hb = Hs + b * G::HBUF;
        constexpr int NWT = TS / RW;  // waves per contour tile
        if (!TAIL || var == 0)
            chain_rows_w<KC, KEEP, false, true, RW, NWT, 8>(a, Hb, atab, bg, wvf, ln, x0f, y0f, ccf, colbits, fl);
        else
            chain_rows_w<KC, KEEP, true, true, RW, NWT, 8>(a, Hb, atab, bg, wvf, ln, x0f, y0f, ccf, colbits, fl);
        if (t + 1 < t1) tap_stage(gray + (b ^ 1) * G::GBUF, Hs + (b ^ 1) * G::HBUF);
        gray_stage(gray + b * G::GBUF);
        if constexpr (RW == 8) {
            reinterpret_cast<uint8_t*>(a.bits)[((f * a.ntiles + ti) * TS + ln) * 8 + wv] = (uint8_t)colbits;
            if (ln == 0) a.tflag[(f * a.ntiles + ti) * NW + wv] = fl;
        } else if (tile_ok) {  // bytes 2 (wv & 3), +1 of the column word; flag words 2 (wv & 3) and the next (none)
            const int ws = wv & 3;
            reinterpret_cast<uint16_t*>(a.bits)[((f * a.ntiles + ti) * TS + ln) * 4 + ws] = (uint16_t)colbits;
            if (ln == 0) *reinterpret_cast<uint2*>(a.tflag + (f * a.ntiles + ti) * NW + 2 * ws) = make_uint2(fl, 0u);
        }
        load((size_t)min(t + 3, t1 - 1) * S + s);
    }
    double* bgo = a.bg_out + (size_t)s * plane;
    const int x = x0 + ln;
#pragma unroll
    for (int j = 0; j < RW; j++) {
        const int y = y0 + RW * wv + j;
        if (x < w && y < h) bgo[(size_t)y * w + x] = bg[j];
    }
    kstamp_end(a.kstamp);
}

}  // namespace px

int pix_lds_bytes(int ksize) { return px::Geo(ksize >> 1).bytes; }

bool pix_supported(int ksize) { return ksize == 5 || ksize == 3 || ksize == 7 || ksize == 21; }

template <int K>
static bool taps_match(const FusedArgs& a) {
    for (int i = 0; i < K; i++)
        if (a.coef[i] != px::Taps<K>::c[i]) return false;
    return true;
}

hipError_t launch_pix(hipStream_t st, const FusedArgs& a, bool planes, bool init) {
    const int bytes = px::Geo(a.ksize >> 1).bytes;
    const bool ok = a.ksize == 3 ? taps_match<3>(a) : a.ksize == 5 ? taps_match<5>(a) : a.ksize == 7 ? taps_match<7>(a)
                  : a.ksize == 21 ? taps_match<21>(a) : false;
    if (!ok) return hipErrorInvalidValue;
    dim3 grid(a.ntiles, a.S);
    // k = 5 steady state on k_pix5: 8 waves of 8 rows per 64 x 64 tile, or 4 waves of 16 rows once the grid
    // holds >= FM_P5_W4_MIN tile-streams (four 4-wave workgroups per CU still give 4 waves per SIMD, and each wave
    // has twice the independent rows per frame barrier).  Measured (round 6, tools/ab_bench.sh, 2 alternating
    // rounds): configs[2] (8 x 1080p, 4,080 tiles) 486 k vs 476 k frames/s, launch std 57-64 vs 50 us; configs[1]
    // (510 tiles, two 4-wave workgroups per CU = 2 waves per SIMD) 365 k vs 418 k over 4 rounds: not there.
#ifndef FM_P5_W4_MIN
#define FM_P5_W4_MIN 1024
#endif
    if (a.ksize == 5 && !planes && !init && (a.w & 3) == 0 && a.w >= 8 && ((uintptr_t)a.src & 3) == 0) {
        const bool keep = a.any_keep != 0, tail = a.acc_vec_end < (long long)a.h * a.w;
        static_assert(px::P5G<8>::bytes <= 64 * 1024 && px::P5G<4>::bytes <= 64 * 1024, "k_pix5 LDS");
        if ((long long)a.ntiles * a.S >= FM_P5_W4_MIN) {
            const size_t lds = px::P5G<4>::dyn_bytes;
            if (keep && tail) hipLaunchKernelGGL((px::k_pix5<true, true, 4>), grid, dim3(256), lds, st, a);
            else if (keep) hipLaunchKernelGGL((px::k_pix5<true, false, 4>), grid, dim3(256), lds, st, a);
            else if (tail) hipLaunchKernelGGL((px::k_pix5<false, true, 4>), grid, dim3(256), lds, st, a);
            else hipLaunchKernelGGL((px::k_pix5<false, false, 4>), grid, dim3(256), lds, st, a);
        } else {
            const size_t lds = px::P5G<8>::dyn_bytes;
            if (keep && tail) hipLaunchKernelGGL((px::k_pix5<true, true, 8>), grid, dim3(512), lds, st, a);
            else if (keep) hipLaunchKernelGGL((px::k_pix5<true, false, 8>), grid, dim3(512), lds, st, a);
            else if (tail) hipLaunchKernelGGL((px::k_pix5<false, true, 8>), grid, dim3(512), lds, st, a);
            else hipLaunchKernelGGL((px::k_pix5<false, false, 8>), grid, dim3(512), lds, st, a);
        }
        return hipGetLastError();
    }
    // k = 21 steady state (config 5) on k_pixw: 64 x 128 bands of 8 waves of 16 rows once the grid holds
    // >= FM_PIXW_BAND_MIN bands (two workgroups per CU), else 64 x 64 tiles of 8 waves of 8 rows.  Measured (round
    // 6, 3 alternating rounds of configs[4]'s geometry): 3.03-3.11 vs 3.13-3.17 ms per launch, 81.4-83.5 k vs
    // 79.7-80.9 k frames/s; with the Haar stage 66.3 k vs 63.4 k.
#ifndef FM_PIXW_BAND_MIN
#define FM_PIXW_BAND_MIN 512
#endif
    if (a.ksize == 21 && !planes && !init && (a.w & 3) == 0 && a.w >= 2 * px::PW<21>::PC + 8 && ((uintptr_t)a.src & 3) == 0) {
        const bool keep = a.any_keep != 0, tail = a.acc_vec_end < (long long)a.h * a.w;
        static_assert(2 * px::PW<21, 16>::bytes <= 160 * 1024, "k_pixw LDS: two workgroups per CU");
        const int nbands = (a.nty + 1) / 2;
        const bool band = (long long)a.ntx * nbands * a.S >= FM_PIXW_BAND_MIN;
#define FM_PIXW_LAUNCH(K, T, RW)                                                                                        \
    do {                                                                                                                \
        using G = px::PW<21, RW>;                                                                                       \
        const dim3 gw(a.ntx * (RW == 16 ? nbands : a.nty), a.S);                                                        \
        (void)hipFuncSetAttribute((const void*)px::k_pixw<21, K, T, RW>, hipFuncAttributeMaxDynamicSharedMemorySize, G::dyn_bytes); \
        hipLaunchKernelGGL((px::k_pixw<21, K, T, RW>), gw, dim3(512), G::dyn_bytes, st, a);                             \
    } while (0)
        if (band) {
            if (keep && tail) FM_PIXW_LAUNCH(true, true, 16);
            else if (keep) FM_PIXW_LAUNCH(true, false, 16);
            else if (tail) FM_PIXW_LAUNCH(false, true, 16);
            else FM_PIXW_LAUNCH(false, false, 16);
        } else {
            if (keep && tail) FM_PIXW_LAUNCH(true, true, 8);
            else if (keep) FM_PIXW_LAUNCH(true, false, 8);
            else if (tail) FM_PIXW_LAUNCH(false, true, 8);
            else FM_PIXW_LAUNCH(false, false, 8);
        }
#undef FM_PIXW_LAUNCH
        return hipGetLastError();
    }
#define FM_PIX_LAUNCH(K, P, I)                                                                                \
    do {                                                                                                        \
        (void)hipFuncSetAttribute((const void*)px::k_pix<K, P, I>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes); \
        hipLaunchKernelGGL((px::k_pix<K, P, I>), grid, dim3(px::NT), bytes, st, a);                             \
    } while (0)
#define FM_PIX_CASE(K)                                                    \
    case K:                                                               \
        if (planes) {                                                     \
            if (init) FM_PIX_LAUNCH(K, true, true); else FM_PIX_LAUNCH(K, true, false);   \
        } else {                                                          \
            if (init) FM_PIX_LAUNCH(K, false, true); else FM_PIX_LAUNCH(K, false, false); \
        }                                                                 \
        break;
    switch (a.ksize) {
        FM_PIX_CASE(3)
        FM_PIX_CASE(5)
        FM_PIX_CASE(7)
        FM_PIX_CASE(21)
        default:
            return hipErrorInvalidValue;
    }
#undef FM_PIX_LAUNCH
#undef FM_PIX_CASE
    return hipGetLastError();
}

}  // namespace fm
