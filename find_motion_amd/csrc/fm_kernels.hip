// fm_kernels.hip — gfx950 kernels of the motion-detection hot path.
//
// Stage map (reference = find_motion/find_motion.py, "fm.py"):
//   k_resize_area / k_resize_area_fast   imutils.resize(INTER_AREA)        fm.py:492
//   k_pixel                              cvtColor, GaussianBlur, mask,     fm.py:493-494, 619-662
//                                        convertScaleAbs+absdiff,
//                                        threshold, accumulateWeighted,
//                                        dilate(iterations=2)
//   k_ccl_*                              findContours(RETR_EXTERNAL) count fm.py:269-272
//                                        + boundingRect                    fm.py:792
//
// Bit-exactness notes: the file is compiled with -ffp-contract=off and every
// floating-point step that OpenCV performs with separate roundings is written
// with explicit __f*_rn / __d*_rn intrinsics; the fused accumulate step uses
// __fma_rn exactly where OpenCV's AVX2 body uses v_fma.
#include "fm_internal.h"

namespace fm {

// ---------------------------------------------------------------------------
// helpers
__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = (p < 0) ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int gray_of(int b, int g, int r) {
    return (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;  // COLOR_BGR2GRAY, u8
}

__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)min(max(v, 0), 255); }

// ---------------------------------------------------------------------------
// INTER_AREA, general (non-integer scale) path.  One workgroup per
// (destination row, frame); thread e owns destination element (dx, c) and
// runs OpenCV's sequential float chain: buf = sum_x S*alpha (in xtab order),
// sum = sum_y beta*buf (in ytab order), then saturate_cast (rne).
__global__ __launch_bounds__(256) void k_resize_area(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                      int H, int W, int h, int w, const int32_t* __restrict__ xofs,
                                                      const int32_t* __restrict__ xcnt, const float* __restrict__ xwt,
                                                      int xtaps, const int32_t* __restrict__ yofs,
                                                      const int32_t* __restrict__ ycnt, const float* __restrict__ ywt,
                                                      int ytaps, uint64_t* kstamp) {
    kstamp_begin_grid(kstamp);
    const int dy = blockIdx.x;
    const size_t f = blockIdx.y;
    const uint8_t* S0 = src + f * (size_t)H * W * 3;
    uint8_t* D = dst + (f * h + dy) * (size_t)w * 3;
    const int sy0 = yofs[dy], ny = ycnt[dy];
    const float* wy = ywt + (size_t)dy * ytaps;
    for (int e = threadIdx.x; e < w * 3; e += blockDim.x) {
        const int dx = e / 3, c = e - dx * 3;
        const int sx0 = xofs[dx], nx = xcnt[dx];
        const float* wx = xwt + (size_t)dx * xtaps;
        float sum = 0.f;
        for (int j = 0; j < ny; j++) {
            const uint8_t* S = S0 + (size_t)(sy0 + j) * W * 3 + (size_t)sx0 * 3 + c;
            float buf = 0.f;
            for (int t = 0; t < nx; t++) buf = __fadd_rn(buf, __fmul_rn((float)S[t * 3], wx[t]));
            const float term = __fmul_rn(wy[j], buf);
            sum = (j == 0) ? term : __fadd_rn(sum, term);
        }
        D[e] = sat_u8(__float2int_rn(sum));
    }
    kstamp_end_wg(kstamp);
}

// INTER_AREA, general path, staged: one workgroup per (destination row, frame) walks
// that row's source rows in ytab order.  Each source row (3*W bytes) is read once with
// coalesced 16-B loads into LDS (double buffered: row j+1 is in flight into registers
// while row j is summed), the x weights sit in LDS for the whole walk, and thread e keeps
// the running sums of its destination elements (dx, c) = (e / 3, e % 3) in registers.
// The float chain per element is k_resize_area's, in the same order, so the bytes are
// identical.  Limits (else k_resize_area): 3*W % 16 == 0, 16-B aligned frames,
// 3*W <= RS_MAXROW, w*3 <= 256 * RS_EPT, w * xtaps floats <= RS_MAXWT.
constexpr int RS_T = 256, RS_EPT = 8, RS_CPT = 4;
constexpr int RS_MAXROW = RS_T * RS_CPT * 16;
constexpr int RS_MAXWT = 8192;
__global__ __launch_bounds__(RS_T) void k_resize_area_rows(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           int H, int W, int h, int w, const int32_t* __restrict__ xofs,
                                                           const int32_t* __restrict__ xcnt, const float* __restrict__ xwt,
                                                           int xtaps, const int32_t* __restrict__ yofs,
                                                           const int32_t* __restrict__ ycnt, const float* __restrict__ ywt,
                                                           int ytaps, uint64_t* kstamp) {
    kstamp_begin_grid(kstamp);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int rowb = 3 * W;                        // multiple of 16
    uint8_t* rows = lds;                           // [2][rowb]
    float* wt = reinterpret_cast<float*>(lds + 2 * rowb);  // [w][xtaps]
    const int dy = blockIdx.x;
    const size_t f = blockIdx.y;
    const int tid = threadIdx.x;
    const uint8_t* S0 = src + f * (size_t)H * rowb;
    for (int i = tid; i < w * xtaps; i += RS_T) wt[i] = xwt[i];
    const int sy0 = yofs[dy], ny = ycnt[dy];
    const int nch = rowb / 16;
    uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, p2 = p0, p3 = p0;  // row prefetch (RS_CPT = 4 chunks)
    static_assert(RS_CPT == 4, "prefetch registers");
#define RS_LOAD_ROW(J)                                                                          \
    do {                                                                                        \
        const uint4* R_ = reinterpret_cast<const uint4*>(S0 + (size_t)(sy0 + (J)) * rowb);     \
        if (tid < nch) p0 = R_[tid];                                                            \
        if (tid + RS_T < nch) p1 = R_[tid + RS_T];                                              \
        if (tid + 2 * RS_T < nch) p2 = R_[tid + 2 * RS_T];                                      \
        if (tid + 3 * RS_T < nch) p3 = R_[tid + 3 * RS_T];                                      \
    } while (0)
#define RS_STORE_ROW(B)                                                                         \
    do {                                                                                        \
        uint4* L_ = reinterpret_cast<uint4*>(rows + (B) * rowb);                                \
        if (tid < nch) L_[tid] = p0;                                                            \
        if (tid + RS_T < nch) L_[tid + RS_T] = p1;                                              \
        if (tid + 2 * RS_T < nch) L_[tid + 2 * RS_T] = p2;                                      \
        if (tid + 3 * RS_T < nch) L_[tid + 3 * RS_T] = p3;                                      \
    } while (0)
    const int ne = w * 3;
    int sx0[RS_EPT], nx[RS_EPT], c3[RS_EPT];
    float sum[RS_EPT];
#pragma unroll
    for (int k = 0; k < RS_EPT; k++) {
        const int e = tid + RS_T * k;
        const int dx = e < ne ? e / 3 : 0;
        sx0[k] = xofs[dx];
        nx[k] = e < ne ? xcnt[dx] : 0;
        c3[k] = dx * xtaps;                   // weight row
        sum[k] = 0.f;
        sx0[k] = sx0[k] * 3 + (e < ne ? e - dx * 3 : 0);  // byte of tap 0 in the row
    }
    const float* wy = ywt + (size_t)dy * ytaps;
    RS_LOAD_ROW(0);
    for (int j = 0; j < ny; j++) {
        const int b = j & 1;
        __syncthreads();  // buffer b is free (row j-2 summed) and the weights are in
        RS_STORE_ROW(b);
        if (j + 1 < ny) RS_LOAD_ROW(j + 1);
        __syncthreads();
        const uint8_t* L = rows + b * rowb;
        const float wyj = wy[j];
#pragma unroll
        for (int k = 0; k < RS_EPT; k++) {
            if (RS_T * k < ne) {  // wave-uniform
                float buf = 0.f;
                const uint8_t* Lp = L + sx0[k];
                const float* wp = wt + c3[k];
                for (int t = 0; t < nx[k]; t++) buf = __fadd_rn(buf, __fmul_rn((float)Lp[3 * t], wp[t]));
                const float term = __fmul_rn(wyj, buf);
                sum[k] = (j == 0) ? term : __fadd_rn(sum[k], term);
            }
        }
    }
    uint8_t* D = dst + (f * h + dy) * (size_t)ne;
#pragma unroll
    for (int k = 0; k < RS_EPT; k++) {
        const int e = tid + RS_T * k;
        if (e < ne) D[e] = sat_u8(__float2int_rn(sum[k]));
    }
    kstamp_end_wg(kstamp);
#undef RS_LOAD_ROW
#undef RS_STORE_ROW
}

// INTER_AREA, general path, register-resident (round 4): one thread per destination pixel
// (dx, dy) of one frame, all three channels, no LDS and no barriers.  The thread walks its
// ycnt[dy] source rows two at a time; for each row pair it loads the 3*NT bytes of its x taps
// from both rows (per-frame buffer descriptor, 4-B aligned b128 loads, one v_alignbyte per
// dword to take out the 0..3-byte misalignment), and runs OpenCV's float chain on packed f32:
// lane (row j, row j+1) of one v_pk_mul_f32 / v_pk_add_f32 pair per (tap, channel), the tap
// weight broadcast.  The x weights (padded with zeros to NT: 0 * S = +0 and buf + 0 = buf, so
// the padding is exact) stay in registers for the whole walk.  The per-element order is
// k_resize_area's: buf = sum_x S*alpha in xtab order, sum = beta_0*buf_0 + beta_1*buf_1 + ...
// in ytab order, then saturate_cast (rne).
typedef float rs_f2 __attribute__((ext_vector_type(2)));
// (Non-temporal frame loads: mode D 492 vs 822 k frames/s -- neighbouring windows re-read a column; round 6,
// profiles/r06/r06i_nontemporal_ab.txt.)
constexpr int RN_T = 256;
template <int NT>
__global__ __launch_bounds__(RN_T) void k_resize_area_nt(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         int H, int W, int h, int w, const int32_t* __restrict__ xofs,
                                                         const int32_t* __restrict__ xcnt, const float* __restrict__ xwt,
                                                         int xtaps, const int32_t* __restrict__ yofs,
                                                         const int32_t* __restrict__ ycnt, const float* __restrict__ ywt,
                                                         int ytaps, const uint8_t* const* __restrict__ srcs,
                                                         uint64_t* kstamp) {
    kstamp_begin_grid(kstamp);
    constexpr int NB = 3 * NT;          // tap bytes of one row
    constexpr int NA = (NB + 3) / 4;    // aligned dwords holding them
    constexpr int ND = NA + 1;          // dwords loaded (a 0..3-byte misalignment)
    constexpr int NQ = ND / 4, NR = ND % 4;
    const int n = h * w;
    const int item = blockIdx.x * RN_T + threadIdx.x;
    const int it = item < n ? item : n - 1;
    const int dy = it / w, dx = it - dy * w;
    const uint32_t rowb = 3u * (uint32_t)W;
    const uint32_t fbytes = rowb * (uint32_t)H;
    const uint32_t lim = (fbytes + 3u) & ~3u;  // every dword holding a frame byte is in range
    // frame blockIdx.y: consecutive frames from src, or one address per frame (srcs: find_objects' ROI
    // frames, read where the engine left them)
    const uint8_t* F = srcs ? srcs[blockIdx.y] : src + (size_t)blockIdx.y * fbytes;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)F, 0, (int)lim, 0x00020000);
    const int nx = xcnt[dx];
    float wx[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) wx[t] = t < nx ? xwt[(size_t)dx * xtaps + t] : 0.f;
    const uint32_t b0 = 3u * (uint32_t)xofs[dx];
    const int sy0 = yofs[dy], ny = ycnt[dy];
    const float* wy = ywt + (size_t)dy * ytaps;
    float sum[3] = {0.f, 0.f, 0.f};
    for (int j = 0; j < ny; j += 2) {
        uint32_t o[2] = {(uint32_t)(sy0 + j) * rowb + b0, (uint32_t)(sy0 + j + 1) * rowb + b0};
        uint32_t al[2][NA];
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t a = o[r] & ~3u, sh = o[r] & 3u;
            uint32_t d[ND];
            if (a + 4u * ND <= lim) {
#pragma unroll
                for (int q = 0; q < NQ; q++) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(a + 16u * q), 0, 0);
                    d[4 * q] = v[0]; d[4 * q + 1] = v[1]; d[4 * q + 2] = v[2]; d[4 * q + 3] = v[3];
                }
                if constexpr (NR == 1) {
                    d[4 * NQ] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a + 16u * NQ), 0, 0);
                } else if constexpr (NR == 2) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(a + 16u * NQ), 0, 0);
                    d[4 * NQ] = v[0]; d[4 * NQ + 1] = v[1];
                } else if constexpr (NR == 3) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(a + 16u * NQ), 0, 0);
                    d[4 * NQ] = v[0]; d[4 * NQ + 1] = v[1]; d[4 * NQ + 2] = v[2];
                }
            } else {  // the window runs past the frame (its last columns / a row past the walk): dwords
                      // wholly out of range read as 0 and carry zero weights or are discarded.  One dword
                      // per load, the step in soffset, so that the loads are not merged into multi-dword
                      // ones (whose range check would not be per dword on every target)
#pragma unroll
                for (int q = 0; q < ND; q++) d[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)a, 4 * q, 0);
            }
#pragma unroll
            for (int q = 0; q < NA; q++) al[r][q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh);
        }
        rs_f2 acc[3];
#pragma unroll
        for (int t = 0; t < NT; t++) {
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const int k = 3 * t + c, q = k >> 2, s = 8 * (k & 3);
                const rs_f2 p = {(float)(uint8_t)(al[0][q] >> s), (float)(uint8_t)(al[1][q] >> s)};
                const rs_f2 m = p * wx[t];
                acc[c] = t == 0 ? m : acc[c] + m;  // 0 + m == m: OpenCV's zeroed buf
            }
        }
        const float by0 = wy[j];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float term = __fmul_rn(by0, acc[c].x);
            sum[c] = j == 0 ? term : __fadd_rn(sum[c], term);
        }
        if (j + 1 < ny) {
            const float by1 = wy[j + 1];
#pragma unroll
            for (int c = 0; c < 3; c++) sum[c] = __fadd_rn(sum[c], __fmul_rn(by1, acc[c].y));
        }
    }
    if (item < n) {
        uint8_t* D = dst + ((size_t)blockIdx.y * n + item) * 3;
#pragma unroll
        for (int c = 0; c < 3; c++) D[c] = sat_u8(__float2int_rn(sum[c]));
    }
    kstamp_end_wg(kstamp);
}

// INTER_AREA integer-scale path (resizeAreaFast): 2x2 => (sum+2)>>2,
// otherwise cvRound(sum * (1.f/area)).
__global__ __launch_bounds__(256) void k_resize_area_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           int H, int W, int h, int w, int sx, int sy, float inv_area,
                                                           uint64_t* kstamp) {
    kstamp_begin_grid(kstamp);
    const size_t f = blockIdx.y;
    const int n = h * w * 3;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) {
        const int c = e % 3, dx = (e / 3) % w, dy = e / (3 * w);
        const uint8_t* S = src + f * (size_t)H * W * 3;
        int sum = 0;
        for (int yy = 0; yy < sy; yy++)
            for (int xx = 0; xx < sx; xx++) sum += S[((size_t)(dy * sy + yy) * W + (dx * sx + xx)) * 3 + c];
        const int v = (sx == 2 && sy == 2) ? ((sum + 2) >> 2) : __float2int_rn(__fmul_rn((float)sum, inv_area));
        dst[f * (size_t)n + e] = sat_u8(v);
    }
    kstamp_end_wg(kstamp);
}

hipError_t launch_resize_area(hipStream_t st, const uint8_t* src, uint8_t* dst, int F, int H, int W, int h, int w,
                              const int32_t* xofs, const int32_t* xcnt, const float* xwt, int xtaps,
                              const int32_t* yofs, const int32_t* ycnt, const float* ywt, int ytaps,
                              const uint8_t* const* srcs, uint64_t* kstamp) {
    const int nt = (xtaps + 1) & ~1;
    if (nt <= 32 && (size_t)3 * W * H < (1u << 31)) {
        const dim3 g((h * w + RN_T - 1) / RN_T, F);
        switch (nt) {
#define RN_CASE(N)                                                                                                      \
    case N:                                                                                                            \
        hipLaunchKernelGGL(k_resize_area_nt<N>, g, dim3(RN_T), 0, st, src, dst, H, W, h, w, xofs, xcnt, xwt, xtaps, yofs, \
                           ycnt, ywt, ytaps, srcs, kstamp);                                                            \
        break;
            RN_CASE(2) RN_CASE(4) RN_CASE(6) RN_CASE(8) RN_CASE(10) RN_CASE(12) RN_CASE(14) RN_CASE(16)
            RN_CASE(18) RN_CASE(20) RN_CASE(22) RN_CASE(24) RN_CASE(26) RN_CASE(28) RN_CASE(30) RN_CASE(32)
#undef RN_CASE
        }
        return hipGetLastError();
    }
    if (srcs) return hipErrorInvalidValue;  // per-frame addresses: the register kernel only (callers gather)
    dim3 grid(h, F);
    const int rowb = 3 * W;
    if (rowb % 16 == 0 && ((uintptr_t)src & 15) == 0 && rowb <= RS_MAXROW && w * 3 <= RS_T * RS_EPT &&
        w * xtaps <= RS_MAXWT) {
        const int bytes = 2 * rowb + w * xtaps * 4;
        (void)hipFuncSetAttribute((const void*)k_resize_area_rows, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        hipLaunchKernelGGL(k_resize_area_rows, grid, dim3(RS_T), bytes, st, src, dst, H, W, h, w, xofs, xcnt, xwt, xtaps,
                           yofs, ycnt, ywt, ytaps, kstamp);
    } else {
        hipLaunchKernelGGL(k_resize_area, grid, dim3(256), 0, st, src, dst, H, W, h, w, xofs, xcnt, xwt, xtaps, yofs,
                           ycnt, ywt, ytaps, kstamp);
    }
    return hipGetLastError();
}

hipError_t launch_resize_area_fast(hipStream_t st, const uint8_t* src, uint8_t* dst, int F, int H, int W, int h,
                                   int w, int sx, int sy, uint64_t* kstamp) {
    const int n = h * w * 3;
    dim3 grid((n + 255) / 256, F);
    const float inv_area = 1.f / (float)(sx * sy);
    hipLaunchKernelGGL(k_resize_area_fast, grid, dim3(256), 0, st, src, dst, H, W, h, w, sx, sy, inv_area, kstamp);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused per-pixel chain for one frame of every stream.
//
// Tile = TW x TH output pixels of the dilated mask.  The dilation needs the
// threshold on the tile + 2 px halo (E region), the threshold needs the blur
// there, and the blur needs gray on E + r = ksize/2 (G region).  Stages:
//   G  : gray from BGR (REFLECT_101 indices)            LDS u8
//   Hs : horizontal taps  sum kx*g                      LDS u16 (<= 255*256)
//   E  : vertical taps, rounding, mask, diff, threshold LDS u8; background
//        updated for the tile interior only (bg_in -> bg_out ping-pong so a
//        neighbour's halo read never sees this frame's update)
//   dilate 5x5 as two separable max passes -> mask_out
constexpr int kTW = 64, kTH = 16, kPixThreads = 256;

__host__ __device__ constexpr int align16(int v) { return (v + 15) & ~15; }

struct PixelLayout {
    int GW, GH, EW, EH, offH, offE, offD, bytes;
    __host__ __device__ PixelLayout(int r) {
        GW = kTW + 4 + 2 * r;
        GH = kTH + 4 + 2 * r;
        EW = kTW + 4;
        EH = kTH + 4;
        offH = align16(GW * GH);
        offE = offH + align16(GH * EW * 2);
        offD = offE + align16(EH * EW);
        bytes = offD + align16(EH * kTW);
    }
};

struct PixelKArgs {
    PixelArgs a;
    const double* bg_in;
};

__global__ __launch_bounds__(kPixThreads) void k_pixel(PixelArgs a, const double* __restrict__ bg_in,
                                                        double* __restrict__ bg_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int r = a.ksize >> 1;
    const PixelLayout L(r);
    uint8_t* G = smem;
    uint16_t* Hs = reinterpret_cast<uint16_t*>(smem + L.offH);
    uint8_t* E = smem + L.offE;
    uint8_t* D = smem + L.offD;

    const int s = blockIdx.z;
    const int h = a.h, w = a.w;
    const int x0 = blockIdx.x * kTW, y0 = blockIdx.y * kTH;
    const size_t plane = (size_t)h * w;
    const uint8_t* src = a.src + (size_t)s * plane * 3;
    const size_t sbase = (size_t)s * plane;
    const bool has_keep = a.has_keep[s] != 0;
    const bool init = a.init != nullptr && a.init[s] != 0;
    const int k = a.ksize;

    // G: gray over the halo region
    for (int i = threadIdx.x; i < L.GW * L.GH; i += kPixThreads) {
        const int gy = i / L.GW, gx = i - gy * L.GW;
        const int y = reflect101(y0 - 2 - r + gy, h);
        const int x = reflect101(x0 - 2 - r + gx, w);
        const uint8_t* p = src + ((size_t)y * w + x) * 3;
        G[i] = (uint8_t)gray_of(p[0], p[1], p[2]);
    }
    __syncthreads();
    // Hs: horizontal pass (8 fraction bits, exact)
    for (int i = threadIdx.x; i < L.GH * L.EW; i += kPixThreads) {
        const int gy = i / L.EW, c = i - gy * L.EW;
        const uint8_t* g = G + gy * L.GW + c;
        uint32_t acc = 0;
        for (int t = 0; t < k; t++) acc += (uint32_t)a.coef[t] * g[t];
        Hs[i] = (uint16_t)acc;
    }
    __syncthreads();
    // E: vertical pass + mask + diff + threshold (+ background update inside)
    for (int i = threadIdx.x; i < L.EH * L.EW; i += kPixThreads) {
        const int ty = i / L.EW, tx = i - ty * L.EW;
        const int y = y0 - 2 + ty, x = x0 - 2 + tx;
        uint8_t th = 0;
        if (y >= 0 && y < h && x >= 0 && x < w) {
            uint32_t acc = 0;
            const uint16_t* hv = Hs + ty * L.EW + tx;
            for (int t = 0; t < k; t++) acc += (uint32_t)a.coef[t] * hv[t * L.EW];
            int blur = (int)((acc + 32768u) >> 16);
            const size_t li = (size_t)y * w + x;
            const size_t pix = sbase + li;
            if (has_keep && a.keep[pix] == 0) blur = 0;
            const double bgv = init ? (double)blur : bg_in[pix];
            int q = a.cvt_simd ? __float2int_rn(fabsf(__double2float_rn(bgv))) : __double2int_rn(fabs(bgv));
            q = min(max(q, 0), 255);
            const int d = abs(blur - q);
            th = d > a.thresh ? 255 : 0;
            if (ty >= 2 && ty < kTH + 2 && tx >= 2 && tx < kTW + 2) {
                const double bl = (double)blur;
                double nb;
                if ((long long)li < a.acc_vec_end)
                    nb = __fma_rn(bgv, a.beta, __dmul_rn(bl, a.alpha));
                else
                    nb = __dadd_rn(__dmul_rn(bl, a.alpha), __dmul_rn(bgv, a.beta));
                bg_out[pix] = nb;
                if (a.gray_out) {
                    a.gray_out[pix] = G[(ty + r) * L.GW + tx + r];
                    a.blur_out[pix] = (uint8_t)blur;
                    a.delta_out[pix] = (uint8_t)d;
                }
            }
        }
        E[i] = th;
    }
    __syncthreads();
    // dilate: horizontal 5-max over E rows
    for (int i = threadIdx.x; i < L.EH * kTW; i += kPixThreads) {
        const int ty = i / kTW, c = i - ty * kTW;
        const uint8_t* e = E + ty * L.EW + c;
        D[i] = max(max(max(e[0], e[1]), max(e[2], e[3])), e[4]);
    }
    __syncthreads();
    // dilate: vertical 5-max -> output
    for (int i = threadIdx.x; i < kTH * kTW; i += kPixThreads) {
        const int oy = i / kTW, ox = i - oy * kTW;
        const int y = y0 + oy, x = x0 + ox;
        if (y < h && x < w) {
            const uint8_t* d = D + oy * kTW + ox;
            const uint8_t m = max(max(max(d[0], d[kTW]), max(d[2 * kTW], d[3 * kTW])), d[4 * kTW]);
            a.mask_out[sbase + (size_t)y * w + x] = m;
        }
    }
}

int pixel_lds_bytes(int ksize) { return PixelLayout(ksize >> 1).bytes; }

hipError_t launch_pixel_pp(hipStream_t st, const PixelArgs& a, const double* bg_in, double* bg_out) {
    const int bytes = PixelLayout(a.ksize >> 1).bytes;
    if (bytes > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid((a.w + kTW - 1) / kTW, (a.h + kTH - 1) / kTH, a.S);
    hipLaunchKernelGGL(k_pixel, grid, dim3(kPixThreads), bytes, st, a, bg_in, bg_out);
    return hipGetLastError();
}

hipError_t launch_pixel(hipStream_t st, const PixelArgs& a) { return launch_pixel_pp(st, a, a.bg, a.bg); }

// ---------------------------------------------------------------------------
// Connected components for findContours(RETR_EXTERNAL).
//
// Every pixel is labelled: foreground 8-connected, background 4-connected
// (Suzuki-Abe's connectivity pair), label = raster index of the component's
// raster-first pixel (union-find that always links the larger root under the
// smaller).  A foreground component has an external contour iff the
// background component left of its first pixel is the outer one, i.e. the
// component of the 1-px zero pad = every background component touching the
// image border.  That equals OpenCV's EXTERNAL scan (checked against the
// literal Suzuki-Abe restatement in oracle/fm_oracle.c).

__device__ __forceinline__ int lds_load(int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int lfind(int* Lb, int x) {
    for (;;) {
        const int p = lds_load(&Lb[x]);
        if (p == x) return x;
        x = p;
    }
}
__device__ __forceinline__ void lunion(int* Lb, int a, int b) {
    for (;;) {
        a = lfind(Lb, a);
        b = lfind(Lb, b);
        if (a == b) return;
        if (a < b) {
            const int old = atomicMin(&Lb[b], a);
            if (old == b) return;
            b = old;
        } else {
            const int old = atomicMin(&Lb[a], b);
            if (old == a) return;
            a = old;
        }
    }
}

__device__ __forceinline__ int gload(int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int gfind(int* Lg, int x) {
    for (;;) {
        const int p = gload(&Lg[x]);
        if (p == x) return x;
        x = p;
    }
}
__device__ __forceinline__ void gunion(int* Lg, int a, int b) {
    for (;;) {
        a = gfind(Lg, a);
        b = gfind(Lg, b);
        if (a == b) return;
        if (a < b) {
            const int old = atomicMin(&Lg[b], a);
            if (old == b) return;
            b = old;
        } else {
            const int old = atomicMin(&Lg[a], b);
            if (old == a) return;
            a = old;
        }
    }
}

constexpr int CB = kCclBlock;

__global__ __launch_bounds__(256) void k_ccl_local(CclArgs a) {
    __shared__ int Lb[CB * CB];
    __shared__ uint8_t M[CB * CB];
    const size_t f = blockIdx.z;
    const int h = a.h, w = a.w;
    const int bx = blockIdx.x * CB, by = blockIdx.y * CB;
    const uint8_t* mask = a.mask + f * (size_t)h * w;
    int32_t* label = a.label + f * (size_t)h * w;
    for (int p = threadIdx.x; p < CB * CB; p += 256) {
        const int ly = p / CB, lx = p % CB, y = by + ly, x = bx + lx;
        M[p] = (y < h && x < w) ? (mask[(size_t)y * w + x] ? 1 : 0) : 2;
        Lb[p] = p;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < CB * CB; p += 256) {
        const int m = M[p];
        if (m == 2) continue;
        const int ly = p / CB, lx = p % CB;
        if (m == 1) {
            if (lx > 0 && M[p - 1] == 1) lunion(Lb, p, p - 1);
            if (ly > 0) {
                if (M[p - CB] == 1) lunion(Lb, p, p - CB);
                if (lx > 0 && M[p - CB - 1] == 1) lunion(Lb, p, p - CB - 1);
                if (lx < CB - 1 && M[p - CB + 1] == 1) lunion(Lb, p, p - CB + 1);
            }
        } else {
            if (lx > 0 && M[p - 1] == 0) lunion(Lb, p, p - 1);
            if (ly > 0 && M[p - CB] == 0) lunion(Lb, p, p - CB);
        }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < CB * CB; p += 256) {
        if (M[p] == 2) continue;
        const int ly = p / CB, lx = p % CB;
        const int root = lfind(Lb, p);
        const int ry = root / CB, rx = root % CB;
        label[(size_t)(by + ly) * w + bx + lx] = (by + ry) * w + bx + rx;
    }
}

// Union across block edges: right-column pixels with E/NE/SE, bottom-row
// pixels with S/SE/SW (foreground), E / S (background).
__global__ __launch_bounds__(64) void k_ccl_merge(CclArgs a) {
    const size_t f = blockIdx.z;
    const int h = a.h, w = a.w;
    const uint8_t* mask = a.mask + f * (size_t)h * w;
    int32_t* L = a.label + f * (size_t)h * w;
    const int bx = blockIdx.x * CB, by = blockIdx.y * CB;
    const int t = threadIdx.x;
    int x, y;
    if (t < CB) {
        x = bx + CB - 1;
        y = by + t;
        if (x + 1 >= w || y >= h) return;
    } else {
        x = bx + (t - CB);
        y = by + CB - 1;
        if (y + 1 >= h || x >= w) return;
    }
    const int p = y * w + x;
    const bool fg = mask[p] != 0;
    auto link = [&](int xx, int yy, bool diag) {
        if (xx < 0 || xx >= w || yy < 0 || yy >= h) return;
        const int q = yy * w + xx;
        const bool qfg = mask[q] != 0;
        if (qfg != fg) return;
        if (!fg && diag) return;
        gunion(L, L[p], L[q]);
    };
    if (t < CB) {
        link(x + 1, y, false);
        link(x + 1, y - 1, true);
        link(x + 1, y + 1, true);
    } else {
        link(x, y + 1, false);
        link(x + 1, y + 1, true);
        link(x - 1, y + 1, true);
    }
}

__global__ __launch_bounds__(256) void k_ccl_flatten(CclArgs a) {
    const size_t f = blockIdx.y;
    const int n = a.h * a.w;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int32_t* L = a.label + f * (size_t)n;
    const int l = L[i];
    if (l != i) L[i] = gfind(L, l);
}

// Mark background components that touch the image border (== the pad's).
__global__ __launch_bounds__(256) void k_ccl_outer(CclArgs a) {
    const size_t f = blockIdx.y;
    const int h = a.h, w = a.w;
    const int per = 2 * w + 2 * h;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= per) return;
    int x, y;
    if (i < w) { x = i; y = 0; }
    else if (i < 2 * w) { x = i - w; y = h - 1; }
    else if (i < 2 * w + h) { x = 0; y = i - 2 * w; }
    else { x = w - 1; y = i - 2 * w - h; }
    const size_t base = f * (size_t)h * w;
    const int p = y * w + x;
    if (a.mask[base + p] == 0) a.outer[base + a.label[base + p]] = 1;
}

// Foreground roots (raster-first pixels): external test + record allocation.
__global__ __launch_bounds__(256) void k_ccl_roots(CclArgs a) {
    const size_t f = blockIdx.y;
    const int h = a.h, w = a.w, n = h * w;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t base = f * (size_t)n;
    if (a.mask[base + i] == 0 || a.label[base + i] != i) return;
    const int y = i / w, x = i - y * w;
    const bool ext = (x == 0) || a.outer[base + a.label[base + i - 1]] != 0;
    int id = -1;
    if (ext) {
        id = atomicAdd(&a.count[f], 1);
        if (id < a.cap) {
            int32_t* r = a.rec + (f * a.cap + id) * 5;
            r[0] = i; r[1] = x; r[2] = y; r[3] = x; r[4] = y;
        }
    }
    a.cid[base + i] = id;
}

// Bounding boxes: only component-boundary pixels can hold an extreme.
__global__ __launch_bounds__(256) void k_ccl_bbox(CclArgs a) {
    const size_t f = blockIdx.y;
    const int h = a.h, w = a.w, n = h * w;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t base = f * (size_t)n;
    const uint8_t* m = a.mask + base;
    if (m[i] == 0) return;
    const int y = i / w, x = i - y * w;
    const bool left = (x == 0) || m[i - 1] == 0;
    const bool right = (x == w - 1) || m[i + 1] == 0;
    const bool down = (y == h - 1) || m[i + w] == 0;
    if (!(left || right || down)) return;
    const int id = a.cid[base + a.label[base + i]];
    if (id < 0 || id >= a.cap) return;
    int32_t* r = a.rec + (f * a.cap + id) * 5;
    if (left) atomicMin(&r[1], x);
    if (right) atomicMax(&r[3], x);
    if (down) atomicMax(&r[4], y);
}

hipError_t launch_ccl(hipStream_t st, const CclArgs& a, KernelTimer* tm) {
    const int F = a.F, h = a.h, w = a.w, n = h * w;
    dim3 gb((w + CB - 1) / CB, (h + CB - 1) / CB, F);
    hipError_t e;
    int tok = tm ? tm->begin("ccl_local", st) : -1;
    hipLaunchKernelGGL(k_ccl_local, gb, dim3(256), 0, st, a);
    if (tm) tm->end(tok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tok = tm ? tm->begin("ccl_merge", st) : -1;
    hipLaunchKernelGGL(k_ccl_merge, gb, dim3(64), 0, st, a);
    if (tm) tm->end(tok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    dim3 gp((n + 255) / 256, F);
    tok = tm ? tm->begin("ccl_flatten", st) : -1;
    hipLaunchKernelGGL(k_ccl_flatten, gp, dim3(256), 0, st, a);
    if (tm) tm->end(tok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    dim3 go((2 * w + 2 * h + 255) / 256, F);
    tok = tm ? tm->begin("ccl_outer", st) : -1;
    hipLaunchKernelGGL(k_ccl_outer, go, dim3(256), 0, st, a);
    if (tm) tm->end(tok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tok = tm ? tm->begin("ccl_roots", st) : -1;
    hipLaunchKernelGGL(k_ccl_roots, gp, dim3(256), 0, st, a);
    if (tm) tm->end(tok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tok = tm ? tm->begin("ccl_bbox", st) : -1;
    hipLaunchKernelGGL(k_ccl_bbox, gp, dim3(256), 0, st, a);
    if (tm) tm->end(tok);
    return hipGetLastError();
}

}  // namespace fm
