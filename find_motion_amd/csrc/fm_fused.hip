// fm_fused.hip — temporally blocked fused kernel + tile-summary CCL (gfx950).
//
// One workgroup (512 threads) owns a 64x64 output tile of one stream for ALL
// frames of a batch:
//
//   per frame t:   raw BGR (tile + 2 + r halo) --16-B loads--> LDS      (prefetched one frame ahead)
//                  gray (BGR2GRAY)                        LDS u8        fm.py:493
//                  horizontal Gaussian taps               LDS u16       fm.py:494
//                  vertical taps, keep-mask, convertScaleAbs + absdiff,
//                  threshold, accumulateWeighted           registers    fm.py:619-662
//                    -> threshold rows as bits via __ballot (lane = column)
//                  dilate 5x5 on the bit rows (shift/or)   LDS u64/row  fm.py:266
//                  mask bytes out                                        VideoFrame.thresh
//                  run-length CCL of the tile (wave 0, lane = row)       fm.py:269-272
//                    -> tile record (edge labels, root list) + node records
//
// The f64 background of the tile + 2-px dilation halo lives in registers for
// the whole batch (the halo is updated redundantly, bit-identical to the
// neighbour's own update), so background HBM traffic is 16 B/px per BATCH,
// not per frame.  Reads come from bg_in and writes go to bg_out (ping-pong),
// so a neighbour's halo read never sees this batch's update.
//
// Global CCL over tile records (k_tile_merge / k_tile_resolve1 / _2): nodes
// are (tile, local component), unions only along tile edges.  The external
// test is the oracle-checked rule of the v1 CCL: a foreground component has
// an external contour iff the background component left of its raster-first
// pixel contains the 1-px zero pad, i.e. touches the image border.
#include "fm_internal.h"

namespace fm {
namespace fz {

constexpr int TS = 64;                   // output tile edge
constexpr int NT = 512;                  // threads per workgroup
constexpr int NW = NT / 64;              // waves
constexpr int EW = TS + 4;               // threshold region (tile + dilation halo)
constexpr int NCJ = (EW + NW - 1) / NW;  // center rows per thread (9)
constexpr int NHALO = EW * 4;            // 4 halo columns x 68 rows
constexpr int NCH = 6;                   // max 16-B raw chunks per thread for the generic-k kernel
constexpr int KMAX_FUSED = 49;

__host__ __device__ constexpr int a16(int v) { return (v + 15) & ~15; }
__host__ __device__ constexpr int gw_for(int r) { return TS + 4 + 2 * r; }
__host__ __device__ constexpr int rs_for(int r) { return a16(3 * gw_for(r) + 32); }
__host__ __device__ constexpr int nchunks_for(int r) { return gw_for(r) * (rs_for(r) / 16); }

struct Layout {
    int GW, RS, CPR, nchunks;
    int o_G, o_H, o_E, o_EH, o_O, o_roff, o_cf, o_rowy, o_colx, bytes;
    __host__ __device__ explicit Layout(int r) {
        GW = gw_for(r);
        RS = rs_for(r);
        CPR = RS / 16;
        nchunks = GW * CPR;
        o_G = GW * RS;
        o_H = o_G + a16(GW * GW);
        o_E = o_H + a16(GW * EW * 2);
        o_EH = o_E + EW * 8;
        o_O = o_EH + a16(NHALO);
        o_roff = o_O + TS * 8;
        o_cf = o_roff + a16(GW * 4);
        o_rowy = o_cf + 64 * 4;
        o_colx = o_rowy + a16(GW * 4);
        bytes = o_colx + a16(GW * 4);
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

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for
// vmcnt(0), which would drain the next frame's raw prefetch at every barrier;
// the stages below exchange data through LDS only.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int lload(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ int lfind(int* P, int x) {
    for (;;) {
        const int p = lload(&P[x]);
        if (p == x) return x;
        x = p;
    }
}
__device__ __forceinline__ void lunion(int* P, int a, int b) {
    for (;;) {
        a = lfind(P, a);
        b = lfind(P, b);
        if (a == b) return;
        if (a < b) {
            const int old = atomicMin(&P[b], a);
            if (old == b) return;
            b = old;
        } else {
            const int old = atomicMin(&P[a], b);
            if (old == a) return;
            a = old;
        }
    }
}

// global union-find over NodeRec::parent (relaxed agent-scope loads bypass the
// per-CU L1, so a find never follows a stale pointer written by another CU)
__device__ __forceinline__ int gpar(NodeRec* N, int x) {
    return __hip_atomic_load(&N[x].parent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// find with path halving done by atomicMin: a pointer only ever moves to a
// smaller member of the same set, so it cannot undo a concurrent link
__device__ __forceinline__ int gfind(NodeRec* N, int x) {
    for (;;) {
        const int p = gpar(N, x);
        if (p == x) return x;
        const int gp = gpar(N, p);
        if (gp == p) return p;
        atomicMin(&N[x].parent, gp);
        x = gp;
    }
}
__device__ __forceinline__ void gunion(NodeRec* N, int a, int b) {
    for (;;) {
        a = gfind(N, a);
        b = gfind(N, b);
        if (a == b) return;
        if (a < b) {
            const int old = atomicMin(&N[b].parent, a);
            if (old == b) return;
            b = old;
        } else {
            const int old = atomicMin(&N[a].parent, b);
            if (old == a) return;
            a = old;
        }
    }
}

__device__ __forceinline__ uint32_t nib2bytes(uint32_t n) { return ((n * 0x00204081u) & 0x01010101u) * 255u; }

// ---------------------------------------------------------------------------
// raw BGR halo region: chunk c = 16 aligned bytes of row gy
template <int N>
struct RawLoad {
    uint4 v[N];
};

// Bytes of a chunk that straddles the frame buffer's first/last byte (only
// possible when a frame does not start 16-B aligned): never read outside it.
__device__ __attribute__((noinline)) uint4 load_partial(const uint8_t* ca, const uint8_t* fb, const uint8_t* fe) {
    uint32_t wds[4] = {0, 0, 0, 0};
    for (int b = 0; b < 16; b++)
        if (ca + b >= fb && ca + b < fe) wds[b >> 2] |= (uint32_t)ca[b] << (8 * (b & 3));
    return make_uint4(wds[0], wds[1], wds[2], wds[3]);
}

// Pointer arithmetic stays on the kernel-argument pointer so the compiler
// emits global_load (a flat load would also count in lgkmcnt and every LDS
// wait would drain the next frame's prefetch).
template <int N>
__device__ __forceinline__ void load_raw(RawLoad<N>& R, const uint8_t* fsrc, size_t fbytes, const int* rowy, int nchunks,
                                         int cpr, int r, int x0, int w, int tid) {
    const uint8_t* fe = fsrc + fbytes;
    const int cx0 = max(x0 - 2 - r, 0), cx1 = min(x0 + TS + 2 + r, w);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const int c = tid + NT * i;
        uint4 val = make_uint4(0, 0, 0, 0);
        if (c < nchunks) {
            const int gy = c / cpr, k = c - gy * cpr;
            const size_t rowoff = (size_t)rowy[gy] * w;
            const uint8_t* sb = fsrc + (rowoff + cx0) * 3;
            const uint8_t* eb = fsrc + (rowoff + cx1) * 3;
            const uint8_t* ca = sb - ((uintptr_t)sb & 15) + 16 * k;
            if (ca < eb) {
                if (__builtin_expect(ca >= fsrc && ca + 16 <= fe, 1)) val = *reinterpret_cast<const uint4*>(ca);
                else val = load_partial(ca, fsrc, fe);
            }
        }
        R.v[i] = val;
    }
}

template <int N>
__device__ __forceinline__ void store_raw(const RawLoad<N>& R, uint8_t* smem, int* roff, const int* rowy,
                                          const uint8_t* fsrc, int nchunks, int cpr, int rs, int r, int x0, int w,
                                          int tid) {
    const int cx0 = max(x0 - 2 - r, 0);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const int c = tid + NT * i;
        if (c < nchunks) {
            const int gy = c / cpr, k = c - gy * cpr;
            *reinterpret_cast<uint4*>(smem + gy * rs + 16 * k) = R.v[i];
            if (k == 0) roff[gy] = (int)(((uintptr_t)fsrc + ((size_t)rowy[gy] * w + cx0) * 3) & 15);
        }
    }
}

// vertical taps at one E pixel: exact fixed point, round half up
template <int KC>
__device__ __forceinline__ int vblur(const uint16_t* hv, const int* cf, int k) {
    uint32_t acc = 0;  // taps < 256, horizontal sums <= 65280: 24-bit multiplies are exact
    if (KC) {
#pragma unroll
        for (int t = 0; t < KC; t++) acc += __umul24((uint32_t)cf[t], hv[t * EW]);
    } else {
        for (int t = 0; t < k; t++) acc += __umul24((uint32_t)cf[t], hv[t * EW]);
    }
    return (int)((acc + 32768u) >> 16);
}

typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

// BGR2GRAY of 4 consecutive pixels packed in 3 dwords (B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3):
// (B*1868 + G*9617 + R*4899 + 8192) >> 14 via v_perm (B,G as u16x2) + v_dot2_u32_u16.
__device__ __forceinline__ uint32_t gray4(uint32_t d0, uint32_t d1, uint32_t d2) {
    const u16x2_t cbg = __builtin_bit_cast(u16x2_t, 1868u | (9617u << 16));
    const uint32_t p0 = __builtin_amdgcn_perm(d0, d0, 0x0C010C00u);
    const uint32_t p1 = __builtin_amdgcn_perm(d1, d0, 0x0C040C03u);
    const uint32_t p2 = __builtin_amdgcn_perm(d1, d1, 0x0C030C02u);
    const uint32_t p3 = __builtin_amdgcn_perm(d2, d2, 0x0C020C01u);
    const uint32_t g0 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p0), cbg, __umul24((d0 >> 16) & 0xFF, 4899u) + 8192u, false) >> 14;
    const uint32_t g1 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p1), cbg, __umul24((d1 >> 8) & 0xFF, 4899u) + 8192u, false) >> 14;
    const uint32_t g2 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p2), cbg, __umul24(d2 & 0xFF, 4899u) + 8192u, false) >> 14;
    const uint32_t g3 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, p3), cbg, __umul24(d2 >> 24, 4899u) + 8192u, false) >> 14;
    return g0 | (g1 << 8) | (g2 << 16) | (g3 << 24);
}

// convertScaleAbs + absdiff + threshold + accumulateWeighted for one pixel.
// row_vec: the whole row lies in OpenCV's vector body (the usual case), so the
// per-pixel tail test is skipped.
__device__ __forceinline__ bool chain(int blur, long long li, double& bg, bool init, int thresh, double alpha,
                                      double beta, long long vec_end, int cvt_simd, int& d_out, bool row_vec = false) {
    const double bv = init ? (double)blur : bg;
    int q = cvt_simd ? __float2int_rn(fabsf(__double2float_rn(bv))) : __double2int_rn(fabs(bv));
    q = min(max(q, 0), 255);
    const int d = abs(blur - q);
    const double bl = (double)blur;
    if (row_vec || li < vec_end) bg = __fma_rn(bv, beta, __dmul_rn(bl, alpha));
    else bg = __dadd_rn(__dmul_rn(bl, alpha), __dmul_rn(bv, beta));
    d_out = d;
    return d > thresh;
}

template <int KC>
__global__ __launch_bounds__(NT) void k_fused(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int k = KC ? KC : a.ksize;
    const int r = k >> 1;
    const Layout L(r);
    uint8_t* G = smem + L.o_G;
    uint16_t* Hs = reinterpret_cast<uint16_t*>(smem + L.o_H);
    uint64_t* Eb = reinterpret_cast<uint64_t*>(smem + L.o_E);
    uint8_t* EH = smem + L.o_EH;
    uint64_t* Ob = reinterpret_cast<uint64_t*>(smem + L.o_O);
    int* roff = reinterpret_cast<int*>(smem + L.o_roff);
    int* cfl = reinterpret_cast<int*>(smem + L.o_cf);
    int* rowy = reinterpret_cast<int*>(smem + L.o_rowy);  // reflected source row of each halo-region row
    int* colx = reinterpret_cast<int*>(smem + L.o_colx);  // 3 * (reflected column - first loaded column)

    const int tid = threadIdx.x, ln = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ti = blockIdx.x, s = blockIdx.y;
    const int h = a.h, w = a.w, S = a.S;
    const int tx = ti % a.ntx, ty = ti / a.ntx;
    const int x0 = tx * TS, y0 = ty * TS;
    const size_t plane = (size_t)h * w;
    const size_t fbytes = plane * 3;
    const bool hk = a.has_keep[s] != 0;
    const uint8_t* keep = a.keep + (size_t)s * plane;
    const bool init0 = a.init != nullptr && a.init[s] != 0;
    const int thresh = a.thresh, cvt_simd = a.cvt_simd;
    const double alpha = a.alpha, beta = a.beta;
    const long long vec_end = a.acc_vec_end;

    int cfr[KC ? KC : 1];
    if (KC) {
#pragma unroll
        for (int t = 0; t < (KC ? KC : 1); t++) cfr[t] = a.coef[t];
    } else {
        if (tid < 64) cfl[tid] = tid < k ? a.coef[tid] : 0;
    }
    const int* cf = KC ? cfr : cfl;
    {
        const int cx0 = max(x0 - 2 - r, 0), cx1 = min(x0 + TS + 2 + r, w);
        for (int i = tid; i < L.GW; i += NT) {
            rowy[i] = reflect101(y0 - 2 - r + i, h);
            // out-of-range columns only feed pixels outside the image: clamp them
            colx[i] = 3 * (min(max(reflect101(x0 - 2 - r + i, w), cx0), cx1 - 1) - cx0);
        }
    }
    __syncthreads();

    // ---- background of the owned E pixels -> registers.  Wave w owns the
    //      contiguous E rows [rs, rs + cnt) (9 rows for waves 0-3, 8 for 4-7).
    const int rs = min(9 * wv, 8 * wv + 4), cnt = wv < 4 ? 9 : 8;
    double bgc[NCJ];
    double bgh = 0.0;
    const double* bgi = a.bg_in + (size_t)s * plane;
#pragma unroll
    for (int j = 0; j < NCJ; j++) {
        const int ey = rs + j, y = y0 - 2 + ey, x = x0 + ln;
        bgc[j] = (!init0 && j < cnt && y >= 0 && y < h && x < w) ? bgi[(size_t)y * w + x] : 0.0;
    }
    if (tid < NHALO && !init0) {
        const int ey = tid >> 2, c = tid & 3, ex = c < 2 ? c : 64 + c;
        const int y = y0 - 2 + ey, x = x0 - 2 + ex;
        if (y >= 0 && y < h && x >= 0 && x < w) bgh = bgi[(size_t)y * w + x];
    }

    // fast gray + horizontal path (k = 5, 13, 21, ...: (2 + r) % 4 == 0 keeps pixel
    // quads dword-aligned in the raw rows); lane -> (row group rg, pixel quad q)
    constexpr bool FAST = KC > 1 && ((2 + (KC >> 1)) % 4) == 0;
    constexpr int GWc = gw_for(KC >> 1);
    constexpr int NQG = GWc / 4;                     // gray quads per row
    constexpr int RPW = FAST ? 64 / NQG : 1;         // rows per wave instruction
    constexpr int NIT = FAST ? (GWc + RPW * NW - 1) / (RPW * NW) : 1;
    constexpr int NQN = (KC + 6) / 4;                // gray quads feeding one horizontal quad
    constexpr int NGRP = KC / 4;                     // 4-tap dot groups
    const int rg = ln / NQG, q = ln - rg * NQG;
    int colq[4] = {0, 0, 0, 0};
    bool qfast = false;
    uint32_t cpk[NGRP > 0 ? NGRP : 1];
    if (FAST) {
        if (rg < RPW) {
#pragma unroll
            for (int i = 0; i < 4; i++) colq[i] = colx[4 * q + i];
            qfast = colq[1] == colq[0] + 3 && colq[2] == colq[0] + 6 && colq[3] == colq[0] + 9 && (colq[0] & 3) == 0;
        }
#pragma unroll
        for (int g = 0; g < (NGRP > 0 ? NGRP : 1); g++)
            cpk[g] = NGRP > 0 ? ((uint32_t)cf[4 * g] | ((uint32_t)cf[4 * g + 1] << 8) | ((uint32_t)cf[4 * g + 2] << 16) |
                                 ((uint32_t)cf[4 * g + 3] << 24))
                              : 0u;
    }

    constexpr int NCHK = KC ? (nchunks_for(KC >> 1) + NT - 1) / NT : NCH;
    RawLoad<NCHK> R;
    load_raw(R, a.src + (size_t)s * fbytes, fbytes, rowy, L.nchunks, L.CPR, r, x0, w, tid);

    const size_t F = (size_t)a.T * S;
    for (int t = 0; t < a.T; t++) {
        const size_t f = (size_t)t * S + s;
        const uint8_t* fsrc = a.src + f * fbytes;
        const bool init = init0 && t == 0;
        // keep per-row scalar offsets from being hoisted out of the frame loop
        // (LICM of 9 rows x 64-bit offsets spills SGPRs)
        int y0v = y0, wvv = wv;
        asm volatile("" : "+s"(y0v), "+s"(wvv));
        const int dbg = a.dbg_skip;
        uint8_t* planes = a.planes;
        if (!(dbg & 16)) store_raw(R, smem, roff, rowy, fsrc, L.nchunks, L.CPR, L.RS, r, x0, w, tid);
        lds_barrier();
        if (t + 1 < a.T && !(dbg & 16)) load_raw(R, a.src + (f + S) * fbytes, fbytes, rowy, L.nchunks, L.CPR, r, x0, w, tid);

        if (FAST) {
            // ---- gray (4 px per lane) + horizontal taps in registers: no G in LDS
            if (!(dbg & 3)) {
#pragma unroll
                for (int it = 0; it < NIT; it++) {
                    const int gy = (it * NW + wvv) * RPW + rg;
                    const bool act = rg < RPW && gy < GWc;
                    uint32_t g4 = 0;
                    if (act) {
                        const int ro = roff[gy];
                        const uint8_t* rowp = smem + gy * L.RS + ro;
                        uint32_t d0, d1, d2;
                        if (qfast && (ro & 3) == 0) {
                            const uint32_t* p32 = reinterpret_cast<const uint32_t*>(rowp + colq[0]);
                            d0 = p32[0];
                            d1 = p32[1];
                            d2 = p32[2];
                        } else {  // reflected / unaligned columns (border tiles)
                            const uint8_t *p0 = rowp + colq[0], *p1 = rowp + colq[1], *p2 = rowp + colq[2], *p3 = rowp + colq[3];
                            d0 = p0[0] | (p0[1] << 8) | (p0[2] << 16) | ((uint32_t)p1[0] << 24);
                            d1 = p1[1] | (p1[2] << 8) | (p2[0] << 16) | ((uint32_t)p2[1] << 24);
                            d2 = p2[2] | (p3[0] << 8) | (p3[1] << 16) | ((uint32_t)p3[2] << 24);
                        }
                        g4 = gray4(d0, d1, d2);
                        if (planes) *reinterpret_cast<uint32_t*>(G + gy * GWc + 4 * q) = g4;
                    }
                    uint32_t qv[NQN];
                    qv[0] = g4;
#pragma unroll
                    for (int d = 1; d < NQN; d++) qv[d] = (uint32_t)__shfl_down((int)g4, d, 64);
                    if (act && q < EW / 4) {
                        uint32_t hq[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            uint32_t acc = 0;
#pragma unroll
                            for (int g = 0; g < NGRP; g++)
                                acc = __builtin_amdgcn_udot4(j ? __builtin_amdgcn_alignbyte(qv[g + 1], qv[g], j) : qv[g],
                                                             cpk[g], acc, false);
#pragma unroll
                            for (int tt = 4 * NGRP; tt < KC; tt++)
                                acc += __umul24((uint32_t)cf[tt], (qv[(j + tt) >> 2] >> (8 * ((j + tt) & 3))) & 0xFFu);
                            hq[j] = acc;
                        }
                        *reinterpret_cast<uint2*>(Hs + gy * EW + 4 * q) = make_uint2(hq[0] | (hq[1] << 16), hq[2] | (hq[3] << 16));
                    }
                }
            }
            lds_barrier();
        } else {
            // ---- gray over the G region (generic k)
            if (!(dbg & 1)) {
                for (int i = tid; i < L.GW * L.GW; i += NT) {
                    const int gy = i / L.GW, gx = i - gy * L.GW;
                    const uint8_t* p = smem + gy * L.RS + roff[gy] + colx[gx];
                    G[i] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14);
                }
            }
            lds_barrier();
            // ---- horizontal taps (exact, 8 fraction bits)
            if (!(dbg & 2)) {
                for (int i = tid; i < L.GW * EW; i += NT) {
                    const int gy = i / EW, c = i - gy * EW;
                    const uint8_t* g = G + gy * L.GW + c;
                    uint32_t acc = 0;
                    for (int tt = 0; tt < k; tt++) acc += __umul24((uint32_t)cf[tt], g[tt]);
                    Hs[i] = (uint16_t)acc;
                }
            }
            lds_barrier();
        }

        // ---- vertical taps (sliding window over the wave's rows) + per-pixel
        //      chain; threshold row bits by ballot
        {
            const int rsv = min(9 * wvv, 8 * wvv + 4), cntv = wvv < 4 ? 9 : 8;
            uint32_t win[KC ? KC : 1];
            if (KC) {
#pragma unroll
                for (int tt = 0; tt + 1 < (KC ? KC : 1); tt++) win[tt] = Hs[(rsv + tt) * EW + ln + 2];
            }
#pragma unroll
            for (int j = 0; j < NCJ; j++) {
                const int ey = rsv + j;
                if (j < cntv && !(dbg & 4)) {  // wave-uniform
                    if (KC) win[(KC ? KC : 1) - 1] = Hs[(ey + (KC ? KC : 1) - 1) * EW + ln + 2];
                    const int y = y0v - 2 + ey, x = x0 + ln;
                    bool th = false;
                    if (y >= 0 && y < h && x < w) {
                        int blur;
                        if (KC) {
                            uint32_t acc = 0;
#pragma unroll
                            for (int tt = 0; tt < (KC ? KC : 1); tt++) acc += __umul24((uint32_t)cf[tt], win[tt]);
                            blur = (int)((acc + 32768u) >> 16);
                        } else {
                            blur = vblur<0>(Hs + ey * EW + ln + 2, cf, k);
                        }
                        const long long li = (long long)y * w + x;
                        if (hk && keep[li] == 0) blur = 0;
                        int d;
                        const bool row_vec = (long long)y * w + x0 + 63 < vec_end;  // wave-uniform
                        th = chain(blur, li, bgc[j], init, thresh, alpha, beta, vec_end, cvt_simd, d, row_vec);
                        if (planes && ey >= 2 && ey < EW - 2) {
                            const size_t o = f * plane + li;
                            planes[o] = G[(ey + r) * L.GW + ln + 2 + r];
                            planes[F * plane + o] = (uint8_t)blur;
                            planes[2 * F * plane + o] = (uint8_t)d;
                        }
                    }
                    const uint64_t bits = __ballot(th);
                    if (ln == 0) Eb[ey] = bits;
                    if (KC) {
#pragma unroll
                        for (int tt = 0; tt + 1 < (KC ? KC : 1); tt++) win[tt] = win[tt + 1];
                    }
                }
            }
        }
        if (tid < NHALO) {
            const int ey = tid >> 2, c = tid & 3, ex = c < 2 ? c : 64 + c;
            const int y = y0 - 2 + ey, x = x0 - 2 + ex;
            bool th = false;
            if (y >= 0 && y < h && x >= 0 && x < w) {
                int blur = vblur<KC>(Hs + ey * EW + ex, cf, k);
                const long long li = (long long)y * w + x;
                if (hk && keep[li] == 0) blur = 0;
                int d;
                th = chain(blur, li, bgh, init, thresh, alpha, beta, vec_end, cvt_simd, d);
            }
            EH[tid] = th ? 1 : 0;
        }
        lds_barrier();

        // ---- dilate 5x5 on bit rows (wave 0, lane = output row)
        if (wv == 0 && !(dbg & 8)) {
            uint64_t C = 0, hl = 0, hr = 0;
#pragma unroll
            for (int d = 0; d < 5; d++) {
                const int ey = ln + d;
                C |= Eb[ey];
                hl |= (uint64_t)EH[ey * 4 + 0] | ((uint64_t)EH[ey * 4 + 1] << 1);
                hr |= (uint64_t)EH[ey * 4 + 2] | ((uint64_t)EH[ey * 4 + 3] << 1);
            }
            // 68-bit row V (bit ex), out bit x = OR of V bits x..x+4
            const uint64_t lo = hl | (C << 2), hi = (C >> 62) | (hr << 2);
            uint64_t o = lo | ((lo >> 1) | (hi << 63)) | ((lo >> 2) | (hi << 62)) | ((lo >> 3) | (hi << 61)) |
                         ((lo >> 4) | (hi << 60));
            const int vc = w - x0;
            if (vc < 64) o &= (1ull << vc) - 1;
            if (y0 + ln >= h) o = 0;
            Ob[ln] = o;
            a.dbits[(f * a.ntiles + ti) * 64 + ln] = o;
            if (__ballot(o != 0) != 0 && ln == 0) a.tflag[f * a.ntiles + ti] = FLAG_ANY;
        }
        lds_barrier();

    }

    // ---- interior background out: owned center pixels
    double* bgo = a.bg_out + (size_t)s * plane;
#pragma unroll
    for (int j = 0; j < NCJ; j++) {
        const int ey = rs + j, y = y0 - 2 + ey, x = x0 + ln;
        if (j < cnt && ey >= 2 && ey < EW - 2 && y < h && x < w) bgo[(size_t)y * w + x] = bgc[j];
    }
}


}  // namespace fz

int fused_lds_bytes(int ksize) { return fz::Layout(ksize >> 1).bytes; }
int fused_max_ksize() { return fz::KMAX_FUSED; }

hipError_t launch_fused(hipStream_t st, const FusedArgs& a, KernelTimer* tm) {
    const int bytes = fz::Layout(a.ksize >> 1).bytes;
    if (a.ksize > fz::KMAX_FUSED || bytes > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid(a.ntiles, a.S);
    int tok = tm ? tm->begin("fused", st) : -1;
    if (a.ksize == 5) {
        (void)hipFuncSetAttribute((const void*)fz::k_fused<5>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        hipLaunchKernelGGL(fz::k_fused<5>, grid, dim3(fz::NT), bytes, st, a);
    } else {
        (void)hipFuncSetAttribute((const void*)fz::k_fused<0>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        hipLaunchKernelGGL(fz::k_fused<0>, grid, dim3(fz::NT), bytes, st, a);
    }
    if (tm) tm->end(tok);
    return hipGetLastError();
}

}  // namespace fm
