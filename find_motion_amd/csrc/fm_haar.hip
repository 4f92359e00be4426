// Object-ROI stage: cv::CascadeClassifier::detectMultiScale
// for HAAR cascades, as find_motion.py:722-731 calls it on the 300-px-wide
// resized frame every 15th frame.  Batched: n images of one size per call.
//
// Device side, per call (one HIP stream, all images and scales in each launch):
//   k_hgray    BGR -> gray (cvtColor fixed point, as the motion path)
//   k_hresize  every scale's INTER_LINEAR_EXACT image (resize.cpp
//              resize_bitExact: 8-bit taps, 16-bit horizontal values,
//              (v + 2^15) >> 16; borders = tap 0 on the clamped edge)
//   k_hrows    integral rows: sum and squared sum, int32 wrapping (CV_32S)
//   k_hcols    integral columns
//   k_htilt    tilted sum T(X,Y) = sum_{y<Y, |x-X+1| <= Y-y-1} I(x,y) (only for
//              cascades with tilted features)
//   k_heval    one thread per window of the ystep grid: HaarEvaluator::setWindow
//              variance normalisation, then the first stages (stumps or trees)
//              with float32 feature sums without FMA and double leaf sums;
//              survivors are compacted into a list
//   k_heval_tail  the remaining stages over the survivors (dense waves)
// Host side: the x-skip of rows whose window was rejected by stage 0 and
// groupRectangles (partition + class means + nested-rect filter), both
// sequential by definition and tiny next to the window sweep.
//
// Algorithmic bytes per image (bench): the BGR image once, plus each scale's
// resized image, integrals (8 or 12 B/px) and the window results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/find_motion_amd.h"
#include "fm_internal.h"

namespace fm {
namespace haar {

constexpr int kPostThreads = 16;  // host threads for a batch's per-image post-pass (the GPU box's CPU share)

constexpr int MAXSC = 64;  // scales per call (1.1^64 > 400: far beyond any frame)

struct Node { int left, right, feat; float thr; };
struct Feat { int r[3][4]; float w[3]; int tilted; };
// k_hdetect's stump record (FM_HAAR_REC): the feature's 12 rectangle corners as offsets from the
// window's corner in the LDS integral patch (row stride pw_max, a per-cascade constant), weights,
// threshold and the two leaf values; 80 B, read by 5 vector loads one stump ahead (vmcnt, not
// lgkmcnt: the prefetch does not hold up the corner reads from LDS)
struct alignas(16) StumpRec { int off[12]; float w[3]; float thr, leaf_lt, leaf_ge; int flags, pad; };
constexpr int kRecTilted = 1, kRecThree = 2;

struct Geo {  // per scale, copied to the device as kernel arguments
    int n;                    // scales
    int sw[MAXSC], sh[MAXSC];  // resized size
    int step[MAXSC];           // ystep
    int gw[MAXSC], gh[MAXSC];  // window grid (columns, rows) on the ystep grid
    int poff[MAXSC];           // resized-image offset (pixels) within one image
    int ioff[MAXSC];           // integral offset (elements) within one image
    int woff[MAXSC];           // window offset within one image
    int xtab[MAXSC], ytab[MAXSC];  // offsets into the tap table
    int toff[MAXSC], tnx[MAXSC];   // k_hdetect: first window tile of each scale, tiles per tile row
    int roff[MAXSC];           // k_hwalk: first window row of each scale
    int P, I, NW, NT, NR;      // per image totals (NT: window tiles, NR: window rows)
};

__device__ __forceinline__ int find_scale(const int* off, int n, int r) {
    int s = 0;
    while (s + 1 < n && off[s + 1] <= r) ++s;
    return s;
}

__global__ void k_hgray(const uint8_t* __restrict__ src, uint8_t* __restrict__ gray, long long npx, int channels) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npx) return;
    if (channels == 1) { gray[i] = src[i]; return; }
    const uint8_t* p = src + i * channels;
    gray[i] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14);
}

// taps: int2 (source offset, 8-bit weight of offset+1); borders carry weight 0
__global__ void k_hresize(const uint8_t* __restrict__ gray, uint8_t* __restrict__ rimg, const int2* __restrict__ taps,
                          Geo g, int W, int H, int nimg) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)nimg * g.P) return;
    const int img = (int)(i / g.P), r = (int)(i - (long long)img * g.P);
    const int s = find_scale(g.poff, g.n, r);
    const int q = r - g.poff[s], y = q / g.sw[s], x = q - y * g.sw[s];
    const int2 tx = taps[g.xtab[s] + x], ty = taps[g.ytab[s] + y];
    const uint8_t* src = gray + (size_t)img * W * H;
    const int x1 = min(tx.x + 1, W - 1), y1 = min(ty.x + 1, H - 1);
    const uint8_t* r0 = src + (size_t)ty.x * W;
    const uint8_t* r1 = src + (size_t)y1 * W;
    const uint32_t h0 = r0[tx.x] * (256 - tx.y) + r0[x1] * tx.y;
    const uint32_t h1 = r1[tx.x] * (256 - tx.y) + r1[x1] * tx.y;
    const uint32_t v = (h0 * (256 - ty.y) + h1 * ty.y + (1u << 15)) >> 16;
    rimg[(size_t)img * g.P + r] = (uint8_t)min(v, 255u);
}

// integral rows: S[y+1][x+1] = sum_{x'<=x} I(x', y) (row prefix; columns follow).
// One wave per row: 64 columns at a time, inclusive wave scan by shuffles, carry in lane 63.
__global__ __launch_bounds__(64) void k_hrows(const uint8_t* __restrict__ rimg, uint32_t* __restrict__ S,
                                              uint32_t* __restrict__ Q, Geo g, int nimg, int maxh) {
    const int row = blockIdx.x, lane = threadIdx.x;
    const int s = blockIdx.y, img = blockIdx.z;
    if (row >= g.sh[s]) return;
    const int sw = g.sw[s];
    const uint8_t* p = rimg + (size_t)img * g.P + g.poff[s] + (size_t)row * sw;
    uint32_t* ps = S + (size_t)img * g.I + g.ioff[s] + (size_t)(row + 1) * (sw + 1);
    uint32_t* pq = Q + (size_t)img * g.I + g.ioff[s] + (size_t)(row + 1) * (sw + 1);
    if (lane == 0) {
        ps[0] = 0;
        pq[0] = 0;
    }
    uint32_t ca = 0, cb = 0;
    for (int base = 0; base < sw; base += 64) {
        const int x = base + lane;
        const uint32_t v = x < sw ? p[x] : 0u;
        uint32_t a = v, b = v * v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t ua = __shfl_up(a, d), ub = __shfl_up(b, d);
            if (lane >= d) {
                a += ua;
                b += ub;
            }
        }
        a += ca;
        b += cb;
        if (x < sw) {
            ps[x + 1] = a;
            pq[x + 1] = b;
        }
        ca = __shfl(a, 63);
        cb = __shfl(b, 63);
    }
}

__global__ void k_hcols(uint32_t* __restrict__ S, uint32_t* __restrict__ Q, Geo g, int nimg) {
    const int col = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y, img = blockIdx.z;
    const int sw = g.sw[s], sh = g.sh[s];
    if (col > sw) return;
    uint32_t* ps = S + (size_t)img * g.I + g.ioff[s] + col;
    uint32_t* pq = Q + (size_t)img * g.I + g.ioff[s] + col;
    ps[0] = 0;
    pq[0] = 0;
    uint32_t a = 0, b = 0;
    const size_t st = (size_t)sw + 1;
    int y = 1;
    // eight rows' loads in flight before their sums are stored (one dependent load per row was a
    // global-memory round trip per row: 87 us per 64-frame call)
    constexpr int U = 8;
    for (; y + U - 1 <= sh; y += U) {
        uint32_t va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            va[u] = ps[(size_t)(y + u) * st];
            vb[u] = pq[(size_t)(y + u) * st];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a += va[u];
            b += vb[u];
            ps[(size_t)(y + u) * st] = a;
            pq[(size_t)(y + u) * st] = b;
        }
    }
    for (; y <= sh; ++y) {
        a += ps[(size_t)y * st];
        b += pq[(size_t)y * st];
        ps[(size_t)y * st] = a;
        pq[(size_t)y * st] = b;
    }
}

// tilted: T(X,Y) = sum_{y<Y} P(y, min(w, X+Y-1-y)) - P(y, max(0, X-Y+y)), P = row prefix
__global__ void k_htilt(const uint32_t* __restrict__ S, uint32_t* __restrict__ T, Geo g, int nimg) {
    const int s = blockIdx.y, img = blockIdx.z;
    const int sw = g.sw[s], sh = g.sh[s], st = sw + 1;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= st * (sh + 1)) return;
    const int Y = e / st, X = e - Y * st;
    const uint32_t* ps = S + (size_t)img * g.I + g.ioff[s];
    uint32_t acc = 0;
    for (int y = 0; y < Y; ++y) {
        const int hi = min(sw, max(0, X + Y - 1 - y)), lo = min(sw, max(0, X - Y + y));
        if (hi > lo) {
            const uint32_t* r1 = ps + (size_t)(y + 1) * st;
            const uint32_t* r0 = ps + (size_t)y * st;
            acc += (r1[hi] - r0[hi]) - (r1[lo] - r0[lo]);
        }
    }
    T[(size_t)img * g.I + g.ioff[s] + e] = acc;
}

struct CascadeDev {
    int win_w, win_h, n_stages, has_tilted;
    int stumps;                // every tree is one node (maxNodesPerTree == 1): scalar node/feature loads
    const int* stage_first;    // first tree of each stage
    const int* stage_ntrees;
    const float* stage_thr;
    const int* tree_node_ofs;  // first node of each tree
    const int* tree_leaf_ofs;  // first leaf of each tree
    const Node* nodes;
    const float* leaves;
    const Feat* feats;
    const StumpRec* recs;      // stumps only: one record per stump (k_hdetect), else nullptr
    int n_recs;
};

__device__ __forceinline__ int32_t rsum(const uint32_t* I, int st, int x, int y, const int* r, bool tilted) {
    uint32_t p0, p1, p2, p3;
    if (!tilted) {
        p0 = I[(y + r[1]) * st + x + r[0]];
        p1 = I[(y + r[1]) * st + x + r[0] + r[2]];
        p2 = I[(y + r[1] + r[3]) * st + x + r[0]];
        p3 = I[(y + r[1] + r[3]) * st + x + r[0] + r[2]];
    } else {
        p0 = I[(y + r[1]) * st + x + r[0]];
        p1 = I[(y + r[1] + r[3]) * st + x + r[0] - r[3]];
        p2 = I[(y + r[1] + r[2]) * st + x + r[0] + r[2]];
        p3 = I[(y + r[1] + r[2] + r[3]) * st + x + r[0] + r[2] - r[3]];
    }
    return (int32_t)(p0 - p1 - p2 + p3);
}

struct Win {  // one window: integral bases, stride, position, variance normaliser
    const uint32_t *S, *T;
    int st, x, y;
    float vnf;
};

// window index -> Win; false for a flat window (HaarEvaluator::setWindow returns false)
__device__ __forceinline__ bool set_window(const uint32_t* S, const uint32_t* Q, const uint32_t* T,
                                           const CascadeDev& c, const Geo& g, long long i, Win& w) {
    const int img = (int)(i / g.NW), r = (int)(i - (long long)img * g.NW);
    const int s = find_scale(g.woff, g.n, r);
    const int q = r - g.woff[s], gy = q / g.gw[s], gx = q - gy * g.gw[s];
    w.x = gx * g.step[s];
    w.y = gy * g.step[s];
    w.st = g.sw[s] + 1;
    const size_t base = (size_t)img * g.I + g.ioff[s];
    w.S = S + base;
    w.T = c.has_tilted ? T + base : nullptr;
    const int nr[4] = {1, 1, c.win_w - 2, c.win_h - 2};
    const int32_t valsum = rsum(w.S, w.st, w.x, w.y, nr, false);
    const uint32_t valsq = (uint32_t)rsum(Q + base, w.st, w.x, w.y, nr, false);
    const double area = (double)((c.win_w - 2) * (c.win_h - 2));
    double nf = area * (double)valsq - (double)valsum * (double)valsum;
    if (!(nf > 0.)) return false;
    nf = sqrt(nf);
    w.vnf = (float)(1. / nf);
    return area * (double)w.vnf < 1e-1;
}

__device__ __forceinline__ float feature(const Feat& f, const Win& w) {
    const uint32_t* I = f.tilted ? w.T : w.S;
    float v = __fmul_rn(f.w[0], (float)rsum(I, w.st, w.x, w.y, f.r[0], f.tilted));
    v = __fadd_rn(v, __fmul_rn(f.w[1], (float)rsum(I, w.st, w.x, w.y, f.r[1], f.tilted)));
    if (f.w[2] != 0.f) v = __fadd_rn(v, __fmul_rn(f.w[2], (float)rsum(I, w.st, w.x, w.y, f.r[2], f.tilted)));
    return __fmul_rn(v, w.vnf);
}

// stages [s0, s1): the first failing stage, or -1 if all pass
__device__ __forceinline__ int run_stages(const CascadeDev& c, const Win& w, int s0, int s1) {
    for (int si = s0; si < s1; ++si) {
        // stage, tree and node indices are the same in every lane: readfirstlane keeps them
        // in SGPRs so the node and feature records come in by scalar loads
        const int t0 = __builtin_amdgcn_readfirstlane(c.stage_first[si]);
        const int nt = __builtin_amdgcn_readfirstlane(c.stage_ntrees[si]);
        double sum = 0.;
#ifndef FM_HAAR_PF
#define FM_HAAR_PF 1
#endif
        if (c.stumps && FM_HAAR_PF) {
            // the next stump's node and feature records are loaded while this one is evaluated (scalar
            // loads: every lane evaluates the same stump); leaves are summed in stump order as OpenCV does
            // The two leaves of a stump are the same in every lane too: loaded by scalar loads with the
            // records, then selected per lane (a per-lane leaf gather stalled every stump on an L2 round trip)
            Node n = c.nodes[t0];
            Feat fe = c.feats[__builtin_amdgcn_readfirstlane(n.feat)];
            float lf = c.leaves[__builtin_amdgcn_readfirstlane(2 * t0 - n.left)];
            float rt = c.leaves[__builtin_amdgcn_readfirstlane(2 * t0 - n.right)];
            for (int t = t0; t < t0 + nt; ++t) {
                const int tn = t + 1 < t0 + nt ? t + 1 : t;
                const Node nn = c.nodes[tn];
                const Feat fn = c.feats[__builtin_amdgcn_readfirstlane(nn.feat)];
                const float nlf = c.leaves[__builtin_amdgcn_readfirstlane(2 * tn - nn.left)];
                const float nrt = c.leaves[__builtin_amdgcn_readfirstlane(2 * tn - nn.right)];
                const float v = feature(fe, w);
                sum += (double)(v < n.thr ? lf : rt);
                n = nn;
                fe = fn;
                lf = nlf;
                rt = nrt;
            }
        } else if (c.stumps) {
            for (int t = t0; t < t0 + nt; ++t) {
                const Node n = c.nodes[t];  // stump t = node t, leaves 2t, 2t + 1
                const float v = feature(c.feats[__builtin_amdgcn_readfirstlane(n.feat)], w);
                const int idx = v < n.thr ? n.left : n.right;
                sum += (double)c.leaves[2 * t - idx];
            }
        } else {
            for (int t = t0; t < t0 + nt; ++t) {
                const Node* nd = c.nodes + c.tree_node_ofs[t];
                int idx = 0;
                do {
                    const Node n = nd[idx];
                    idx = feature(c.feats[n.feat], w) < n.thr ? n.left : n.right;
                } while (idx > 0);
                sum += (double)c.leaves[c.tree_leaf_ofs[t] - idx];
            }
        }
        if (sum < (double)c.stage_thr[si]) return si;
    }
    return -1;
}

#ifndef FM_HAAR_REC
#define FM_HAAR_REC 1  // k_hdetect on stump records (StumpRec) when the cascade is all stumps
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
struct RecV { u32x4_t o0, o1, o2, wt, lf; };  // corners 0-3, 4-7, 8-11; w0 w1 w2 thr; leaf_lt leaf_ge flags pad

__device__ __forceinline__ RecV load_rec(__amdgpu_buffer_rsrc_t rs, int t) {
    // buffer loads (vector memory): past the last record they read zeros
    const int b = t * (int)sizeof(StumpRec);
    return RecV{__builtin_amdgcn_raw_buffer_load_b128(rs, 0, b, 0), __builtin_amdgcn_raw_buffer_load_b128(rs, 0, b + 16, 0),
                __builtin_amdgcn_raw_buffer_load_b128(rs, 0, b + 32, 0), __builtin_amdgcn_raw_buffer_load_b128(rs, 0, b + 48, 0),
                __builtin_amdgcn_raw_buffer_load_b128(rs, 0, b + 64, 0)};
}

__device__ __forceinline__ int32_t rsum4(const uint32_t* P, u32x4_t o) {
    return (int32_t)(P[(int)o.x] - P[(int)o.y] - P[(int)o.z] + P[(int)o.w]);
}

// one stump on the window whose patch corners start at PS / PT: feature (as feature()) -> leaf value
__device__ __forceinline__ float stump_rec(const RecV& R, const uint32_t* PS, const uint32_t* PT, float vnf) {
    const int fl = __builtin_amdgcn_readfirstlane((int)R.lf.z);
    const uint32_t* P = (fl & kRecTilted) ? PT : PS;
    float v = __fmul_rn(__uint_as_float(R.wt.x), (float)rsum4(P, R.o0));
    v = __fadd_rn(v, __fmul_rn(__uint_as_float(R.wt.y), (float)rsum4(P, R.o1)));
    if (fl & kRecThree) v = __fadd_rn(v, __fmul_rn(__uint_as_float(R.wt.z), (float)rsum4(P, R.o2)));
    v = __fmul_rn(v, vnf);
    return v < __uint_as_float(R.wt.w) ? __uint_as_float(R.lf.x) : __uint_as_float(R.lf.y);
}

// run_stages on stump records: stages [s0, s1) of the window whose corner is PS / PT in the LDS patch.
// Stumps are visited in cascade order, so the next one's record is loaded while this one is evaluated
// (two records in flight, renamed by a 2-way unrolled loop); leaves are summed in stump order.
__device__ __forceinline__ int run_stages_rec(const CascadeDev& c, const uint32_t* PS, const uint32_t* PT, float vnf,
                                              int s0, int s1) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)c.recs, 0, c.n_recs * (int)sizeof(StumpRec),
                                                                        0x00020000);
#ifndef FM_HAAR_PFD
#define FM_HAAR_PFD 2  // records in flight ahead of the stump being evaluated (1 or 2; 2: 1.23 -> 1.11 ms per 64-frame call)
#endif
    int t = __builtin_amdgcn_readfirstlane(c.stage_first[s0]);
    if constexpr (FM_HAAR_PFD >= 2) {
        // R0 = record t, R1 = record t + 1 at the top of every stump; a 3-way unrolled loop renames them
        RecV R0 = load_rec(rs, t), R1 = load_rec(rs, t + 1);
        for (int si = s0; si < s1; ++si) {
            const int t1 = t + __builtin_amdgcn_readfirstlane(c.stage_ntrees[si]);
            double sum = 0.;
            for (; t + 2 < t1; t += 3) {
                const RecV R2 = load_rec(rs, t + 2);
                sum += (double)stump_rec(R0, PS, PT, vnf);
                R0 = load_rec(rs, t + 3);
                sum += (double)stump_rec(R1, PS, PT, vnf);
                R1 = load_rec(rs, t + 4);
                sum += (double)stump_rec(R2, PS, PT, vnf);
            }
            for (; t < t1; ++t) {
                const RecV R2 = load_rec(rs, t + 2);
                sum += (double)stump_rec(R0, PS, PT, vnf);
                R0 = R1;
                R1 = R2;
            }
            if (sum < (double)c.stage_thr[si]) return si;
        }
        return -1;
    }
    RecV A = load_rec(rs, t);
    for (int si = s0; si < s1; ++si) {
        const int t1 = t + __builtin_amdgcn_readfirstlane(c.stage_ntrees[si]);
        double sum = 0.;
        for (; t + 1 < t1; t += 2) {
            const RecV B = load_rec(rs, t + 1);
            sum += (double)stump_rec(A, PS, PT, vnf);
            A = load_rec(rs, t + 2);
            sum += (double)stump_rec(B, PS, PT, vnf);
        }
        if (t < t1) {
            const RecV B = load_rec(rs, t + 1);
            sum += (double)stump_rec(A, PS, PT, vnf);
            A = B;
            ++t;
        }
        if (sum < (double)c.stage_thr[si]) return si;
    }
    return -1;
}

// head: one thread per window of the ystep grid, stages [0, split); survivors are appended
// to `live` so the later stages run dense waves.  res: 1 accepted, 0 rejected by stage 0,
// -1 rejected later or flat (the tail overwrites survivors' entries)
__global__ __launch_bounds__(256) void k_heval(const uint32_t* __restrict__ S, const uint32_t* __restrict__ Q,
                                               const uint32_t* __restrict__ T, int8_t* __restrict__ res,
                                               int* __restrict__ live, int* __restrict__ nlive, int split,
                                               CascadeDev c, Geo g, int nimg) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)nimg * g.NW) return;
    Win w;
    int8_t out = -1;
    if (set_window(S, Q, T, c, g, i, w)) {
        const int f = run_stages(c, w, 0, split);
        if (f >= 0) {
            out = f == 0 ? 0 : -1;
        } else if (split < c.n_stages) {
            live[atomicAdd(nlive, 1)] = (int)i;
        } else {
            out = 1;
        }
    }
    res[i] = out;
}

// tail: survivors of the head, grid-stride over the list, stages [split, n_stages)
__global__ __launch_bounds__(256) void k_heval_tail(const uint32_t* __restrict__ S, const uint32_t* __restrict__ Q,
                                                    const uint32_t* __restrict__ T, int8_t* __restrict__ res,
                                                    const int* __restrict__ live, const int* __restrict__ nlive,
                                                    int split, CascadeDev c, Geo g, int nimg) {
    const int n = *nlive;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const long long i = live[k];
        Win w;
        set_window(S, Q, T, c, g, i, w);  // a survivor's window is not flat
        res[i] = run_stages(c, w, split, c.n_stages) >= 0 ? -1 : 1;
    }
}

// The whole window sweep for one tile of TW x TH windows of one scale of one image: the tile's
// integral patch (and the tilted one) is staged in LDS once, so every feature's corner reads are
// LDS reads instead of gathers from L2; the stages run in phases, each on the previous phase's
// survivors compacted into the workgroup's first threads (round 6: the tail packed instead of spread
// over the four waves, detector device time -25 %; tests/haar_wave_model.py prices the layouts).
// Same windows, same arithmetic, same res values as k_heval + k_heval_tail.
constexpr int TW = 16, TH = 16;  // windows per tile (256 threads)
#ifndef FM_HAAR_HEADC
#define FM_HAAR_HEADC 1  // compact the survivors after stages 1 and 2 as well
#endif
#ifndef FM_HAAR_TAIL_SPREAD
#define FM_HAAR_TAIL_SPREAD 0  // 1: the last phase's survivors spread over the four waves
#endif

__global__ __launch_bounds__(TW * TH) void k_hdetect(const uint32_t* __restrict__ S, const uint32_t* __restrict__ Q,
                                                     const uint32_t* __restrict__ T, int8_t* __restrict__ res, int split,
                                                     CascadeDev c, Geo g, int pw_max) {
    extern __shared__ uint32_t patch[];  // S patch [ph][pw], then T patch (tilted cascades)
    __shared__ int s_live[2][TW * TH];   // the windows (thread ids) a phase runs, double-buffered
    __shared__ int s_n[4];               // their count, per phase
    __shared__ float s_vnf[TW * TH];
    const int img = blockIdx.y;
    const int s = find_scale(g.toff, g.n, blockIdx.x);
    const int tile = blockIdx.x - g.toff[s];
    const int tyi = tile / g.tnx[s], txi = tile - tyi * g.tnx[s];
    const int step = g.step[s], st = g.sw[s] + 1, ih = g.sh[s] + 1;
    const int gx0 = txi * TW, gy0 = tyi * TH;
    const int px0 = gx0 * step, py0 = gy0 * step;
    const int pw = min((TW - 1) * step + c.win_w + 1, st - px0), ph = min((TH - 1) * step + c.win_h + 1, ih - py0);
    const size_t base = (size_t)img * g.I + g.ioff[s];
    const int tid = threadIdx.x;
    if (tid < 4) s_n[tid] = 0;
    for (int i = tid; i < pw * ph; i += TW * TH) {
        const int y = i / pw, x = i - y * pw;
        const size_t gi = base + (size_t)(py0 + y) * st + px0 + x;
        patch[y * pw_max + x] = S[gi];
        if (c.has_tilted) patch[ph * pw_max + y * pw_max + x] = T[gi];
    }
    __syncthreads();
    const uint32_t* PT = c.has_tilted ? patch + ph * pw_max : nullptr;
    {
        // HaarEvaluator::setWindow of this thread's window: sum from the patch, squared sum from Q; a window
        // that is not flat joins the first phase's list
        const int gx = gx0 + (tid % TW), gy = gy0 + tid / TW;
        if (gx < g.gw[s] && gy < g.gh[s]) {
            const int nr[4] = {1, 1, c.win_w - 2, c.win_h - 2};
            const int32_t valsum = rsum(patch, pw_max, (gx - gx0) * step, (gy - gy0) * step, nr, false);
            const uint32_t valsq = (uint32_t)rsum(Q + base, st, gx * step, gy * step, nr, false);
            const double area = (double)((c.win_w - 2) * (c.win_h - 2));
            double nf = area * (double)valsq - (double)valsum * (double)valsum;
            bool ok = nf > 0.;
            float vnf = 1.f;
            if (ok) {
                nf = sqrt(nf);
                vnf = (float)(1. / nf);
                ok = area * (double)vnf < 1e-1;
            }
            if (ok) {
                s_live[0][atomicAdd(&s_n[0], 1)] = tid;
                s_vnf[tid] = vnf;
            } else {
                res[(long long)img * g.NW + g.woff[s] + (long long)gy * g.gw[s] + gx] = -1;
            }
        }
    }
    __syncthreads();
    // Phases of stages: each runs on the windows the previous one left alive, compacted into the first threads
    // (one window each), so the lanes a wave issues for are mostly live ones: stages [0, 1), [1, 2), [2, split)
    // and [split, n_stages) with FM_HAAR_HEADC, else [0, split) and [split, n_stages).  Each window's stages,
    // stumps and sums are the same in any phase split (only which thread runs them changes).
    int bnd[4], nb = 0;  // end stage of each phase (workgroup-uniform)
    if (FM_HAAR_HEADC) {
        bnd[nb++] = 1;
        if (split > 1) bnd[nb++] = min(2, split);
        if (split > 2) bnd[nb++] = split;
    } else {
        bnd[nb++] = split;
    }
    if (split < c.n_stages) bnd[nb++] = c.n_stages;
    int sb = 0;
    for (int p = 0; p < nb; ++p) {
        const int e = bnd[p], n = s_n[p];
        const bool last = e >= c.n_stages;
        // the last phase's windows packed into the first waves (FM_HAAR_TAIL_SPREAD: window k -> wave k % 4,
        // a few deep windows in parallel on the four SIMDs)
        constexpr int NWV = TW * TH / 64;
        const int k = (last && FM_HAAR_TAIL_SPREAD) ? (tid & 63) * NWV + (tid >> 6) : tid;
        if (k < n) {
            const int t2 = s_live[p & 1][k];
            const int gx2 = gx0 + (t2 % TW), gy2 = gy0 + t2 / TW;
            Win v;
            v.st = pw_max;
            v.x = (gx2 - gx0) * step;
            v.y = (gy2 - gy0) * step;
            v.S = patch;
            v.T = PT;
            v.vnf = s_vnf[t2];
            const long long wi2 = (long long)img * g.NW + g.woff[s] + (long long)gy2 * g.gw[s] + gx2;
            const int f = (FM_HAAR_REC && c.recs) ? run_stages_rec(c, patch + v.y * pw_max + v.x,
                                                                   PT ? PT + v.y * pw_max + v.x : nullptr, v.vnf, sb, e)
                                                  : run_stages(c, v, sb, e);
            if (f >= 0) res[wi2] = f == 0 ? 0 : -1;  // 0: rejected by stage 0 (the row walk's skip)
            else if (!last) s_live[(p + 1) & 1][atomicAdd(&s_n[p + 1], 1)] = t2;
            else res[wi2] = 1;
        }
        if (p + 1 < nb) __syncthreads();  // (uniform: nb and bnd depend on split and the cascade only)
        sb = e;
    }
}

// detectMultiScale's row walk on the device: one thread per window row of one scale of one image walks
// the row as OpenCV visits it (a window stage 0 rejects skips the next one: x += result == 0 ? 2 : 1)
// and appends the accepted windows it reaches (their index in the image's window grid) to the image's
// candidate list; the host sorts each list, which restores OpenCV's scale / row / column order.  Only
// these lists cross PCIe (kCandCap per image; a longer list makes the host read the whole result grid).
constexpr int kCandCap = 1024;
__global__ __launch_bounds__(64) void k_hwalk(const int8_t* __restrict__ res, int* __restrict__ cnt,
                                              int* __restrict__ cand, Geo g, int nimg) {
    const long long i = (long long)blockIdx.x * 64 + threadIdx.x;
    if (i >= (long long)nimg * g.NR) return;
    const int img = (int)(i / g.NR), r = (int)(i - (long long)img * g.NR);
    const int s = find_scale(g.roff, g.n, r);
    const int gy = r - g.roff[s], gw = g.gw[s];
    const int base = g.woff[s] + gy * gw;
    const int8_t* R = res + (size_t)img * g.NW + base;
    for (int gx = 0; gx < gw;) {
        const int8_t v = R[gx];
        if (v > 0) {
            const int k = atomicAdd(&cnt[img], 1);
            if (k < kCandCap) cand[(size_t)img * kCandCap + k] = base + gx;
        }
        gx += v == 0 ? 2 : 1;
    }
}

}  // namespace haar
}  // namespace fm

using namespace fm::haar;

struct fm_haar {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int win_w = 0, win_h = 0, n_stages = 0, has_tilted = 0;
    // device cascade
    void* d_blob = nullptr;
    CascadeDev cd{};
    // grow-only work buffers
    uint8_t *d_src = nullptr, *d_gray = nullptr, *d_rimg = nullptr;
    uint32_t *d_S = nullptr, *d_Q = nullptr, *d_T = nullptr;
    int8_t* d_res = nullptr;
    int *d_live = nullptr, *d_nlive = nullptr;
    size_t cap_live = 0;
    int2* d_taps = nullptr;
    uint8_t *d_raw = nullptr, *d_roi = nullptr;  // fm_haar_detect_frames: source frames, ROI frames
    const uint8_t** d_fptr = nullptr;             // fm_haar_detect_frame_list: the frames' device addresses
    const uint8_t** h_fptr = nullptr;             // their page-locked staging copy (an asynchronous DMA)
    size_t cap_fptr = 0;
    int32_t *d_axo = nullptr, *d_axc = nullptr, *d_ayo = nullptr, *d_ayc = nullptr;
    float *d_axw = nullptr, *d_ayw = nullptr;
    int area_key[4] = {0, 0, 0, 0};  // (W, H, w, h) the area tables are for
    fm::AreaAxis ax, ay;
    size_t cap_raw = 0, cap_roi = 0;
    size_t cap_src = 0, cap_gray = 0, cap_rimg = 0, cap_S = 0, cap_Q = 0, cap_T = 0, cap_res = 0, cap_taps = 0;
    std::vector<int8_t> h_res;
    int *d_ccnt = nullptr, *d_cand = nullptr;  // k_hwalk: per image candidate count, candidate lists
    int *h_ccnt = nullptr, *h_cand = nullptr;  // their page-locked host copies
    size_t cap_cand = 0;
    std::vector<int32_t> cand;  // last call's candidates of image 0 (x, y, w, h)
    double last_ms = 0.;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    // FM_HAAR_TIMES (dev build): host seconds per phase over all calls -- resize setup, geometry + launches,
    // result copy + wait, post-pass -- printed at destroy
    bool times = false;
    double tph[4] = {0, 0, 0, 0};
    long long ncalls = 0;
    // a queued detection (detect_enqueue) and, after detect_finish, its results per image
    bool pending = false;
    int pend_n = 0, pend_min_neighbors = 0;
    std::vector<float> pend_sc;
    std::vector<std::vector<int32_t>> out;  // grouped rects (x, y, w, h) of each image of the last detection
    Geo pend_g{};
    double pend_tA = 0., pend_tB = 0.;
};

static inline double hnow() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int hfail(fm_haar* h, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf;
    return code;
}
#define HH(h, x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return hfail(h, FM_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

template <class T>
static int grow(fm_haar* h, T** p, size_t& cap, size_t count) {
    if (count <= cap && *p) return 0;
    if (*p) HH(h, hipFree(*p));
    *p = nullptr;
    cap = 0;
    HH(h, hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T)));
    cap = count;
    return 0;
}

static inline int rne_d(double v) { return (int)std::nearbyint(v); }
static inline int rne_f(float v) { return (int)std::nearbyintf(v); }

// interpolationLinear<uint8_t>::getCoeffs (resize.cpp), borders folded to weight 0 on the edge
static void linear_exact_taps(int ssize, int dsize, std::vector<int2>& out) {
    const double inv = (double)dsize / ssize;
    const double scale = 1.0 / inv;
    for (int d = 0; d < dsize; ++d) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int i = (int)std::floor(f);
        int2 t;
        if (i >= 0 && ssize > 1) {
            if (i < ssize - 1) {
                t.x = i;
                t.y = rne_d((f - i) * 256.0);
            } else {
                t.x = ssize - 1;
                t.y = 0;
            }
        } else {
            t.x = 0;
            t.y = 0;
        }
        out.push_back(t);
    }
}

extern "C" {

int fm_haar_create(int device, const fm_haar_desc* d, fm_haar** out) {
    if (!out) return FM_EINVAL;
    *out = nullptr;
    auto* h = new fm_haar();
    *out = h;
    h->times = fm::dev_env("FM_HAAR_TIMES") != nullptr;  // (dev build only)
    if (!d || d->win_w < 3 || d->win_h < 3 || d->n_stages < 1 || d->n_trees < 1 || d->n_nodes < 1 ||
        d->n_features < 1 || d->n_leaves != d->n_trees + d->n_nodes)
        return hfail(h, FM_EINVAL, "bad cascade description (window >= 3x3, stages/trees/nodes/features >= 1, "
                                   "leaves == trees + nodes)");
    int tsum = 0;
    for (int s = 0; s < d->n_stages; ++s) {
        if (d->stage_ntrees[s] < 1) return hfail(h, FM_EINVAL, "stage %d has no trees", s);
        tsum += d->stage_ntrees[s];
    }
    if (tsum != d->n_trees) return hfail(h, FM_EINVAL, "stage tree counts sum to %d, not n_trees %d", tsum, d->n_trees);
    int nsum = 0;
    for (int t = 0; t < d->n_trees; ++t) {
        if (d->tree_nodes[t] < 1) return hfail(h, FM_EINVAL, "tree %d has no nodes", t);
        nsum += d->tree_nodes[t];
    }
    if (nsum != d->n_nodes) return hfail(h, FM_EINVAL, "tree node counts sum to %d, not n_nodes %d", nsum, d->n_nodes);
    // node links stay inside their tree; features inside the window
    for (int t = 0, o = 0; t < d->n_trees; o += d->tree_nodes[t], ++t)
        for (int k = 0; k < d->tree_nodes[t]; ++k) {
            const int l = d->node_left[o + k], r = d->node_right[o + k], f = d->node_feature[o + k];
            if (l >= d->tree_nodes[t] || r >= d->tree_nodes[t] || l < -d->tree_nodes[t] || r < -d->tree_nodes[t] ||
                f < 0 || f >= d->n_features)
                return hfail(h, FM_EINVAL, "tree %d node %d: link or feature out of range", t, k);
            if ((l > 0 && l <= k) || (r > 0 && r <= k))
                return hfail(h, FM_EINVAL, "tree %d node %d: links must point forward", t, k);
        }
    int tilted = 0;
    for (int i = 0; i < d->n_features; ++i) {
        const int* r = d->feat_rects + 12 * i;
        const bool tl = d->feat_tilted && d->feat_tilted[i];
        tilted |= tl;
        for (int j = 0; j < 3; ++j) {
            const int x = r[4 * j], y = r[4 * j + 1], w = r[4 * j + 2], hh = r[4 * j + 3];
            if (j > 0 && d->feat_weights[3 * i + j] == 0.f) continue;
            const bool ok = !tl ? (x >= 0 && y >= 0 && w >= 0 && hh >= 0 && x + w <= d->win_w && y + hh <= d->win_h)
                                : (w >= 0 && hh >= 0 && x - hh >= 0 && x + w <= d->win_w && y >= 0 &&
                                   y + w + hh <= d->win_h);
            if (!ok) return hfail(h, FM_EINVAL, "feature %d rect %d outside the %dx%d window", i, j, d->win_w, d->win_h);
        }
    }
    h->device = device;
    HH(h, hipSetDevice(device));
    {   // the detector's stream at the pixel stream's (high) priority: a motion engine on the same device
        // always has a pixel launch queued at high priority, and at normal priority the cascade's
        // launches waited behind them (configs[4]: a 1 ms call took 4.4 ms of wall time).  With the detection
        // asynchronous (round 5) the priority no longer matters: 63.6-63.9 k frames/s either way.
        int lo = 0, hi = 0;
        HH(h, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HH(h, hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi));
    }
    HH(h, hipEventCreate(&h->e0));
    HH(h, hipEventCreate(&h->e1));
    h->win_w = d->win_w;
    h->win_h = d->win_h;
    h->n_stages = d->n_stages;
    h->has_tilted = tilted;

    std::vector<int> sfirst(d->n_stages), tno(d->n_trees), tlo(d->n_trees);
    for (int s = 0, t = 0; s < d->n_stages; t += d->stage_ntrees[s], ++s) sfirst[s] = t;
    for (int t = 0, no = 0, lo = 0; t < d->n_trees; ++t) {
        tno[t] = no;
        tlo[t] = lo;
        no += d->tree_nodes[t];
        lo += d->tree_nodes[t] + 1;
    }
    std::vector<Node> nodes(d->n_nodes);
    for (int k = 0; k < d->n_nodes; ++k)
        nodes[k] = Node{d->node_left[k], d->node_right[k], d->node_feature[k], d->node_threshold[k]};
    std::vector<Feat> feats(d->n_features);
    for (int i = 0; i < d->n_features; ++i) {
        Feat f{};
        for (int j = 0; j < 3; ++j) {
            for (int k = 0; k < 4; ++k) f.r[j][k] = d->feat_rects[12 * i + 4 * j + k];
            f.w[j] = d->feat_weights[3 * i + j];
        }
        f.tilted = d->feat_tilted && d->feat_tilted[i] ? 1 : 0;
        feats[i] = f;
    }
    // one blob: [stage_first][stage_ntrees][stage_thr][tree_node_ofs][tree_leaf_ofs][nodes][leaves][feats]
    auto al = [](size_t v) { return (v + 63) & ~(size_t)63; };
    size_t off[8], tot = 0;
    const size_t sz[8] = {sizeof(int) * d->n_stages, sizeof(int) * d->n_stages, sizeof(float) * d->n_stages,
                          sizeof(int) * d->n_trees, sizeof(int) * d->n_trees, sizeof(Node) * d->n_nodes,
                          sizeof(float) * d->n_leaves, sizeof(Feat) * d->n_features};
    for (int k = 0; k < 8; ++k) {
        off[k] = tot;
        tot += al(sz[k]);
    }
    std::vector<uint8_t> blob(tot, 0);
    std::memcpy(&blob[off[0]], sfirst.data(), sz[0]);
    std::memcpy(&blob[off[1]], d->stage_ntrees, sz[1]);
    std::memcpy(&blob[off[2]], d->stage_threshold, sz[2]);
    std::memcpy(&blob[off[3]], tno.data(), sz[3]);
    std::memcpy(&blob[off[4]], tlo.data(), sz[4]);
    std::memcpy(&blob[off[5]], nodes.data(), sz[5]);
    std::memcpy(&blob[off[6]], d->leaves, sz[6]);
    std::memcpy(&blob[off[7]], feats.data(), sz[7]);
    int stumps = 1;
    for (int t = 0; t < d->n_trees; ++t) stumps &= d->tree_nodes[t] == 1;
    // stump records for k_hdetect: corners as offsets in its LDS patch, whose row stride is
    // (TW - 1) * 2 + win_w + 1 (the widest step, 2) for every launch of this cascade
    const size_t rec_off = tot;
    if (stumps) {
        const int st = (TW - 1) * 2 + d->win_w + 1;
        std::vector<StumpRec> recs(d->n_trees);
        for (int t = 0; t < d->n_trees; ++t) {  // stump t = node t, leaves 2t - left, 2t - right
            const Node& n = nodes[t];
            const Feat& f = feats[n.feat];
            StumpRec r{};
            for (int j = 0; j < 3; ++j) {
                const int x = f.r[j][0], y = f.r[j][1], w = f.r[j][2], hh = f.r[j][3];
                int* o = r.off + 4 * j;
                if (!f.tilted) {
                    o[0] = y * st + x;
                    o[1] = y * st + x + w;
                    o[2] = (y + hh) * st + x;
                    o[3] = (y + hh) * st + x + w;
                } else {
                    o[0] = y * st + x;
                    o[1] = (y + hh) * st + x - hh;
                    o[2] = (y + w) * st + x + w;
                    o[3] = (y + w + hh) * st + x + w - hh;
                }
                r.w[j] = f.w[j];
            }
            r.thr = n.thr;
            r.leaf_lt = d->leaves[2 * t - n.left];
            r.leaf_ge = d->leaves[2 * t - n.right];
            r.flags = (f.tilted ? kRecTilted : 0) | (f.w[2] != 0.f ? kRecThree : 0);
            recs[t] = r;
        }
        blob.resize(tot + recs.size() * sizeof(StumpRec));
        std::memcpy(&blob[tot], recs.data(), recs.size() * sizeof(StumpRec));
        tot = blob.size();
    }
    HH(h, hipMalloc(&h->d_blob, tot));
    HH(h, hipMemcpy(h->d_blob, blob.data(), tot, hipMemcpyHostToDevice));
    auto* b = (uint8_t*)h->d_blob;
    h->cd = CascadeDev{d->win_w, d->win_h, d->n_stages, tilted, stumps,
                       (const int*)(b + off[0]), (const int*)(b + off[1]), (const float*)(b + off[2]),
                       (const int*)(b + off[3]), (const int*)(b + off[4]), (const Node*)(b + off[5]),
                       (const float*)(b + off[6]), (const Feat*)(b + off[7]),
                       stumps ? (const StumpRec*)(b + rec_off) : nullptr, stumps ? d->n_trees : 0};
    return FM_OK;
}

void fm_haar_destroy(fm_haar* h) {
    if (!h) return;
    if (h->times && h->ncalls)
        std::fprintf(stderr, "[fm_haar] %lld calls, host ms per call: resize setup %.3f, geometry + launches %.3f, "
                     "copy + wait %.3f, post-pass %.3f\n", h->ncalls, 1e3 * h->tph[0] / h->ncalls,
                     1e3 * h->tph[1] / h->ncalls, 1e3 * h->tph[2] / h->ncalls, 1e3 * h->tph[3] / h->ncalls);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_blob, (void*)h->d_src, (void*)h->d_gray, (void*)h->d_rimg, (void*)h->d_S,
                    (void*)h->d_Q, (void*)h->d_T, (void*)h->d_res, (void*)h->d_taps, (void*)h->d_raw, (void*)h->d_fptr, (void*)h->d_live, (void*)h->d_nlive,
                    (void*)h->d_roi, (void*)h->d_axo, (void*)h->d_axc, (void*)h->d_ayo, (void*)h->d_ayc,
                    (void*)h->d_axw, (void*)h->d_ayw})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)h->d_ccnt, (void*)h->d_cand})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)h->h_ccnt, (void*)h->h_cand, (void*)h->h_fptr})
        if (p) (void)hipHostFree(p);
    if (h->e0) (void)hipEventDestroy(h->e0);
    if (h->e1) (void)hipEventDestroy(h->e1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char* fm_haar_last_error(const fm_haar* h) { return h ? h->err.c_str() : "null detector"; }

int fm_haar_window(const fm_haar* h, int* w, int* hh) {
    if (!h || !w || !hh) return FM_EINVAL;
    *w = h->win_w;
    *hh = h->win_h;
    return FM_OK;
}

// The detection of n images queued on the detector's stream (nothing waits): scales, pyramid, integrals,
// window sweep, the device row walk and the copies of the candidate lists; detect_finish waits for them and
// runs the host post-pass.  One detection in flight per detector.
static int detect_enqueue_impl(fm_haar* h, const uint8_t* images, int n, int H, int W, int channels, int on_device,
                               double scale_factor, int min_neighbors, int min_w, int min_h, int max_w, int max_h) {
    if (!h || !h->d_blob) return FM_EINVAL;
    if (!images || n < 1 || H < 1 || W < 1 || (channels != 1 && channels != 3) || !(scale_factor > 1.0))
        return hfail(h, FM_EINVAL, "bad arguments (n >= 1, 1 or 3 channels, scale_factor > 1)");
    if (h->pending) return hfail(h, FM_ESTATE, "a detection is already queued: collect it first");
    HH(h, hipSetDevice(h->device));
    const double tA = h->times ? hnow() : 0.;
    h->out.assign(n, {});
    h->pend_n = n;
    h->pend_min_neighbors = min_neighbors;
    h->pend_sc.clear();
    h->pend_g = Geo{};
    h->cand.clear();
    // scales (detectMultiScaleNoGrouping)
    if (max_w == 0 || max_h == 0) {
        max_w = W;
        max_h = H;
    }
    h->pending = true;  // (a detection with no window finishes with empty results)
    if (H < h->win_h || W < h->win_w) return FM_OK;
    std::vector<float> all, sc;
    for (double f = 1;; f *= scale_factor) {
        if (rne_d(h->win_w * f) > W || rne_d(h->win_h * f) > H) break;
        all.push_back((float)f);
        if ((int)all.size() > 4096) break;
    }
    for (float s : all) {
        const int ww = rne_f((float)h->win_w * s), wh = rne_f((float)h->win_h * s);
        if (ww > max_w || wh > max_h) break;
        if (ww < min_w || wh < min_h) continue;
        sc.push_back(s);
    }
    if (sc.empty()) return FM_OK;
    if ((int)sc.size() > MAXSC) return hfail(h, FM_ENOTSUP, "%zu scales (max %d)", sc.size(), MAXSC);
    Geo g{};
    g.n = (int)sc.size();
    int ww0 = 0;
    std::vector<int> ylim(g.n);
    std::vector<int2> taps;
    for (int s = 0; s < g.n; ++s) {
        g.sw[s] = rne_f((float)W / sc[s]);
        g.sh[s] = rne_f((float)H / sc[s]);
        g.step[s] = sc[s] >= 2.f ? 1 : 2;
        const int ww = std::max(g.sw[s] + 1 - h->win_w, 0), wh = std::max(g.sh[s] + 1 - h->win_h, 0);
        if (s == 0) ww0 = ww;
        g.gw[s] = (ww + g.step[s] - 1) / g.step[s];
        ylim[s] = wh;
    }
    const int nstripes = (ww0 + 31) / 32;
    for (int s = 0; s < g.n; ++s) {
        const int wh = std::max(g.sh[s] + 1 - h->win_h, 0);
        const int stripe = nstripes ? std::max((wh / g.step[s] + nstripes - 1) / nstripes, 1) * g.step[s] : 0;
        ylim[s] = std::min(nstripes * stripe, wh);
        g.gh[s] = (ylim[s] + g.step[s] - 1) / g.step[s];
        if (g.gw[s] == 0) g.gh[s] = 0;
    }
    g.P = g.I = g.NW = g.NT = g.NR = 0;
    for (int s = 0; s < g.n; ++s) {
        g.roff[s] = g.NR;
        g.NR += g.gw[s] > 0 ? g.gh[s] : 0;
        g.poff[s] = g.P;
        g.ioff[s] = g.I;
        g.woff[s] = g.NW;
        g.toff[s] = g.NT;
        g.tnx[s] = (g.gw[s] + TW - 1) / TW;
        g.NT += g.tnx[s] * ((g.gh[s] + TH - 1) / TH);
        g.P += g.sw[s] * g.sh[s];
        g.I += (g.sw[s] + 1) * (g.sh[s] + 1);
        g.NW += g.gw[s] * g.gh[s];
        g.xtab[s] = (int)taps.size();
        linear_exact_taps(W, g.sw[s], taps);
        g.ytab[s] = (int)taps.size();
        linear_exact_taps(H, g.sh[s], taps);
    }
    const size_t npx = (size_t)n * H * W;
    int rc;
    if ((rc = grow(h, &h->d_gray, h->cap_gray, npx)) || (rc = grow(h, &h->d_rimg, h->cap_rimg, (size_t)n * g.P)) ||
        (rc = grow(h, &h->d_taps, h->cap_taps, taps.size())) || (rc = grow(h, &h->d_res, h->cap_res, (size_t)n * g.NW)))
        return rc;
    if ((rc = grow(h, &h->d_S, h->cap_S, (size_t)n * g.I)) || (rc = grow(h, &h->d_Q, h->cap_Q, (size_t)n * g.I)) ||
        (h->has_tilted && (rc = grow(h, &h->d_T, h->cap_T, (size_t)n * g.I))))
        return rc;
    const uint8_t* src = images;
    if (!on_device) {
        if ((rc = grow(h, &h->d_src, h->cap_src, npx * channels))) return rc;
        HH(h, hipMemcpyAsync(h->d_src, images, npx * channels, hipMemcpyHostToDevice, h->stream));
        src = h->d_src;
    }
    HH(h, hipMemcpyAsync(h->d_taps, taps.data(), taps.size() * sizeof(int2), hipMemcpyHostToDevice, h->stream));
    HH(h, hipEventRecord(h->e0, h->stream));
    k_hgray<<<(unsigned)((npx + 255) / 256), 256, 0, h->stream>>>(src, h->d_gray, (long long)npx, channels);
    const long long np = (long long)n * g.P;
    k_hresize<<<(unsigned)((np + 255) / 256), 256, 0, h->stream>>>(h->d_gray, h->d_rimg, h->d_taps, g, W, H, n);
    int maxh = 0, maxw = 0;
    for (int s = 0; s < g.n; ++s) {
        maxh = std::max(maxh, g.sh[s]);
        maxw = std::max(maxw, g.sw[s]);
    }
    k_hrows<<<dim3(maxh, g.n, n), 64, 0, h->stream>>>(h->d_rimg, h->d_S, h->d_Q, g, n, maxh);
    k_hcols<<<dim3((maxw + 1 + 63) / 64, g.n, n), 64, 0, h->stream>>>(h->d_S, h->d_Q, g, n);
    if (h->has_tilted)
        k_htilt<<<dim3((unsigned)(((maxw + 1) * (maxh + 1) + 255) / 256), g.n, n), 256, 0, h->stream>>>(h->d_S, h->d_T,
                                                                                                    g, n);
    const long long nw = (long long)n * g.NW;
    if (nw > 0) {
        // stages evaluated for every window before survivors are compacted (FM_HAAR_SPLIT, default 4)
        #ifdef FM_DEV_SWITCHES  // A/B switch of the dev build only (make VARIANT=dev)
        static const int split_env = std::getenv("FM_HAAR_SPLIT") ? std::atoi(std::getenv("FM_HAAR_SPLIT")) : 4;
#else
#ifndef FM_HAAR_SPLIT_DEFAULT
#define FM_HAAR_SPLIT_DEFAULT 4
#endif
        static const int split_env = FM_HAAR_SPLIT_DEFAULT;
#endif
        const int split = std::max(1, std::min(split_env, h->n_stages));
#ifndef FM_HAAR_TILES
#define FM_HAAR_TILES 1  // k_hdetect (LDS integral patches) instead of k_heval + k_heval_tail
#endif
        const int pw_max = (TW - 1) * 2 + h->win_w + 1, ph_max = (TH - 1) * 2 + h->win_h + 1;
        const size_t lds = (size_t)pw_max * ph_max * 4 * (h->has_tilted ? 2 : 1);
        if (FM_HAAR_TILES && lds <= 56 * 1024) {
            if (g.NT > 0)
                hipLaunchKernelGGL(k_hdetect, dim3((unsigned)g.NT, (unsigned)n), dim3(TW * TH), lds, h->stream, h->d_S, h->d_Q,
                                   h->d_T, h->d_res, split, h->cd, g, pw_max);
            goto swept;
        }
        if ((rc = grow(h, &h->d_live, h->cap_live, (size_t)nw))) return rc;
        if (!h->d_nlive) HH(h, hipMalloc((void**)&h->d_nlive, sizeof(int)));
        HH(h, hipMemsetAsync(h->d_nlive, 0, sizeof(int), h->stream));
        k_heval<<<(unsigned)((nw + 255) / 256), 256, 0, h->stream>>>(h->d_S, h->d_Q, h->d_T, h->d_res, h->d_live,
                                                                     h->d_nlive, split, h->cd, g, n);
        // a thread per possible survivor (grid-stride only past 16384 blocks): a smaller fixed grid
        // (1024 blocks) left survivors queued behind each other, 4.3 vs 3.4 ms per 64 ROI frames
        const unsigned tb = (unsigned)std::max<long long>(1, std::min<long long>((nw + 255) / 256, 16384));
        if (split < h->n_stages)
            k_heval_tail<<<tb, 256, 0, h->stream>>>(h->d_S, h->d_Q, h->d_T, h->d_res, h->d_live, h->d_nlive, split,
                                                      h->cd, g, n);
    }
swept:
    HH(h, hipGetLastError());
    HH(h, hipEventRecord(h->e1, h->stream));
    // candidates: the row walk on the device, then only the per-image lists cross PCIe (page-locked)
    if ((size_t)n > h->cap_cand) {
        for (void* p : {(void*)h->d_ccnt, (void*)h->d_cand})
            if (p) HH(h, hipFree(p));
        for (void* p : {(void*)h->h_ccnt, (void*)h->h_cand})
            if (p) HH(h, hipHostFree(p));
        h->d_ccnt = h->d_cand = h->h_ccnt = h->h_cand = nullptr;
        h->cap_cand = 0;
        HH(h, hipMalloc((void**)&h->d_ccnt, (size_t)n * sizeof(int)));
        HH(h, hipMalloc((void**)&h->d_cand, (size_t)n * kCandCap * sizeof(int)));
        HH(h, hipHostMalloc((void**)&h->h_ccnt, (size_t)n * sizeof(int), 0));
        HH(h, hipHostMalloc((void**)&h->h_cand, (size_t)n * kCandCap * sizeof(int), 0));
        h->cap_cand = (size_t)n;
    }
    HH(h, hipMemsetAsync(h->d_ccnt, 0, (size_t)n * sizeof(int), h->stream));
    if (nw > 0 && g.NR > 0)
        k_hwalk<<<(unsigned)(((long long)n * g.NR + 63) / 64), 64, 0, h->stream>>>(h->d_res, h->d_ccnt, h->d_cand, g, n);
    HH(h, hipGetLastError());
    const double tB = h->times ? hnow() : 0.;
    HH(h, hipMemcpyAsync(h->h_ccnt, h->d_ccnt, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HH(h, hipMemcpyAsync(h->h_cand, h->d_cand, (size_t)n * kCandCap * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    h->pend_sc = sc;
    h->pend_g = g;
    h->pend_tA = tA;
    h->pend_tB = tB;
    return FM_OK;
}

static int detect_enqueue(fm_haar* h, const uint8_t* images, int n, int H, int W, int channels, int on_device,
                          double scale_factor, int min_neighbors, int min_w, int min_h, int max_w, int max_h) {
    const int rc = detect_enqueue_impl(h, images, n, H, W, channels, on_device, scale_factor, min_neighbors, min_w,
                                       min_h, max_w, max_h);
    if (rc != FM_OK && h && rc != FM_ESTATE) {  // (a failed call leaves nothing to collect)
        h->pending = false;
        h->out.clear();
    }
    return rc;
}

// Waits for the queued detection and runs the host post-pass: OpenCV's row walk order from the device's
// sorted candidate lists (or the whole result grid when a list overflowed), then groupRectangles.
static int detect_finish(fm_haar* h) {
    if (!h->pending) return FM_OK;
    h->pending = false;
    const int n = h->pend_n, min_neighbors = h->pend_min_neighbors;
    const std::vector<float>& sc = h->pend_sc;
    const Geo& g = h->pend_g;
    if (sc.empty()) return FM_OK;  // no scale (or an image smaller than the window): no detections
    const double tA = h->pend_tA, tB = h->pend_tB;
    const long long nw = (long long)n * g.NW;
    HH(h, hipStreamSynchronize(h->stream));
    bool overflow = false;
    for (int i = 0; i < n; ++i) overflow |= h->h_ccnt[i] > kCandCap;
    if (overflow) {  // some image has more accepted windows than a list holds: walk the whole grid here
        h->h_res.resize((size_t)nw);
        HH(h, hipMemcpy(h->h_res.data(), h->d_res, (size_t)nw, hipMemcpyDeviceToHost));
    }
    const double tC = h->times ? hnow() : 0.;
    float ms = 0.f;
    HH(h, hipEventElapsedTime(&ms, h->e0, h->e1));
    h->last_ms = ms;

    // per image: the row scan with the stage-0 skip, then groupRectangles (eps 0.2); images are
    // independent (each writes only its own counts / rects), so a batch spreads them over threads
    const double eps = 0.2;
    auto post = [&](int img) {
        std::vector<int32_t> c;
        auto emit = [&](int s, int gy, int gx) {
            const float f = sc[s];
            const int wsw = rne_f((float)h->win_w * f), wsh = rne_f((float)h->win_h * f);
            const int x = gx * g.step[s], y = gy * g.step[s];
            c.insert(c.end(), {rne_f((float)x * f), rne_f((float)y * f), wsw, wsh});
        };
        if (!overflow) {  // the device's lists: sorted window indices are OpenCV's visiting order
            const int nc0 = h->h_ccnt[img];
            int* L = h->h_cand + (size_t)img * kCandCap;
            std::sort(L, L + nc0);
            for (int k = 0, s = 0; k < nc0; ++k) {
                while (s + 1 < g.n && L[k] >= g.woff[s + 1]) ++s;
                const int q = L[k] - g.woff[s], gy = q / g.gw[s];
                emit(s, gy, q - gy * g.gw[s]);
            }
        } else {
            const int8_t* R = h->h_res.data() + (size_t)img * g.NW;
            for (int s = 0; s < g.n; ++s)
                for (int gy = 0; gy < g.gh[s]; ++gy)
                    for (int gx = 0; gx < g.gw[s];) {
                        const int8_t v = R[g.woff[s] + gy * g.gw[s] + gx];
                        if (v > 0) emit(s, gy, gx);
                        gx += v == 0 ? 2 : 1;
                    }
        }
        if (img == 0) h->cand = c;
        const int nc = (int)c.size() / 4;
        std::vector<int32_t> outr;
        if (min_neighbors <= 0) {
            outr = c;
        } else if (nc > 0) {
            auto similar = [&](int a, int b) {
                const int32_t* r1 = &c[4 * a];
                const int32_t* r2 = &c[4 * b];
                const double delta = eps * (std::min(r1[2], r2[2]) + std::min(r1[3], r2[3])) * 0.5;
                return std::abs(r1[0] - r2[0]) <= delta && std::abs(r1[1] - r2[1]) <= delta &&
                       std::abs(r1[0] + r1[2] - r2[0] - r2[2]) <= delta && std::abs(r1[1] + r1[3] - r2[1] - r2[3]) <= delta;
            };
            // cv::partition
            std::vector<int> par(nc, -1), rk(nc, 0);
            auto root = [&](int i) {
                while (par[i] >= 0) i = par[i];
                return i;
            };
            for (int i = 0; i < nc; ++i) {
                int r = root(i);
                for (int j = 0; j < nc; ++j) {
                    if (i == j || !similar(i, j)) continue;
                    int r2 = root(j);
                    if (r2 == r) continue;
                    if (rk[r] > rk[r2]) {
                        par[r2] = r;
                    } else {
                        par[r] = r2;
                        rk[r2] += rk[r] == rk[r2];
                        r = r2;
                    }
                    for (int k = j, p; (p = par[k]) >= 0; k = p) par[k] = r;
                    for (int k = i, p; (p = par[k]) >= 0; k = p) par[k] = r;
                }
            }
            std::vector<int> lab(nc), cls_of_root(nc, -1);
            int ncls = 0;
            for (int i = 0; i < nc; ++i) {
                const int r = root(i);
                if (cls_of_root[r] < 0) cls_of_root[r] = ncls++;
                lab[i] = cls_of_root[r];
            }
            std::vector<long long> acc(4 * (size_t)ncls, 0);
            std::vector<int> cnt(ncls, 0);
            for (int i = 0; i < nc; ++i) {
                for (int k = 0; k < 4; ++k) acc[4 * lab[i] + k] += c[4 * i + k];
                cnt[lab[i]]++;
            }
            std::vector<int32_t> avg(4 * (size_t)ncls);
            for (int l = 0; l < ncls; ++l) {
                const float sinv = 1.f / (float)cnt[l];
                for (int k = 0; k < 4; ++k) avg[4 * l + k] = rne_f((float)(int)acc[4 * l + k] * sinv);
            }
            for (int i = 0; i < ncls; ++i) {
                const int32_t* r1 = &avg[4 * i];
                const int n1 = cnt[i];
                if (n1 <= min_neighbors) continue;
                int j = 0;
                for (; j < ncls; ++j) {
                    const int n2 = cnt[j];
                    if (j == i || n2 <= min_neighbors) continue;
                    const int32_t* r2 = &avg[4 * j];
                    const int dx = rne_d(r2[2] * eps), dy = rne_d(r2[3] * eps);
                    if (r1[0] >= r2[0] - dx && r1[1] >= r2[1] - dy && r1[0] + r1[2] <= r2[0] + r2[2] + dx &&
                        r1[1] + r1[3] <= r2[1] + r2[3] + dy && (n2 > std::max(3, n1) || n1 < 3))
                        break;
                }
                if (j == ncls) outr.insert(outr.end(), r1, r1 + 4);
            }
        }
        h->out[img] = std::move(outr);
    };
    // (64 1080p ROI frames of frontalface: 12.1 ms per call single-threaded beside 3.1 ms of kernels, when
    // the host walked every window; with the device's lists only grouping is left, worth threads only for
    // many candidates)
    long long ncand = 0;
    for (int i = 0; i < n; ++i) ncand += overflow ? (long long)g.NW : h->h_ccnt[i];
    const int nth = ncand < 4096 ? 1 : std::min(n, std::max(1, std::min(kPostThreads, (int)std::thread::hardware_concurrency())));
    if (nth <= 1) {
        for (int img = 0; img < n; ++img) post(img);
    } else {
        std::atomic<int> next{0};
        std::vector<std::thread> pool;
        for (int t = 0; t < nth; ++t)
            pool.emplace_back([&] {
                for (int i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) post(i);
            });
        for (auto& t : pool) t.join();
    }
    if (h->times) {
        const double tD = hnow();
        h->tph[1] += tB - tA;
        h->tph[2] += tC - tB;
        h->tph[3] += tD - tC;
        h->ncalls++;
    }
    return FM_OK;
}

// the last detection's results: counts[i] (all of them) and up to cap rects per image
static void detect_copy(const fm_haar* h, int32_t* rects, int cap, int32_t* counts) {
    for (int img = 0; img < (int)h->out.size(); ++img) {
        const int no = (int)h->out[img].size() / 4;
        counts[img] = no;
        const int keep = std::min(no, cap);
        if (keep > 0) std::memcpy(rects + (size_t)img * cap * 4, h->out[img].data(), sizeof(int32_t) * 4 * keep);
    }
}

int fm_haar_detect(fm_haar* h, const uint8_t* images, int n, int H, int W, int channels, int on_device,
                   double scale_factor, int min_neighbors, int min_w, int min_h, int max_w, int max_h,
                   int32_t* rects, int cap, int32_t* counts) {
    if (!h || !h->d_blob) return FM_EINVAL;
    if (cap < 0 || !counts || (cap > 0 && !rects)) return hfail(h, FM_EINVAL, "bad arguments (counts[n], rects[n][cap])");
    if (int rc = detect_finish(h)) return rc;  // (a queued detection the caller never collected)
    if (int rc = detect_enqueue(h, images, n, H, W, channels, on_device, scale_factor, min_neighbors, min_w, min_h,
                                max_w, max_h))
        return rc;
    if (int rc = detect_finish(h)) return rc;
    detect_copy(h, rects, cap, counts);
    return FM_OK;
}

int fm_haar_candidates(const fm_haar* h, int32_t* rects, int cap) {
    if (!h || cap < 0 || (cap > 0 && !rects)) return FM_EINVAL;
    const int nc = (int)h->cand.size() / 4;
    const int k = std::min(nc, cap);
    if (k > 0) std::memcpy(rects, h->cand.data(), sizeof(int32_t) * 4 * k);
    return nc;
}

double fm_haar_last_ms(const fm_haar* h) { return h ? h->last_ms : 0.; }

}  // extern "C"

// find_objects' resize + detect over n frames: consecutive [n][H][W][3] frames at `frames` (host memory,
// or device memory when on_device), or -- list != nullptr -- the n device frames at list[i]
// async: queue the detection (fm_haar_collect takes its results), else detect and return the results
static int detect_frames_impl(fm_haar* h, const uint8_t* frames, const uint8_t* const* list, int n, int H, int W,
                              int on_device, int roi_w, double scale_factor, int min_neighbors, int32_t* rects,
                              int cap, int32_t* counts, int* roi_h_out, bool async = false) {
    if (!h || !h->d_blob) return FM_EINVAL;
    if (h->pending) {
        if (async) return hfail(h, FM_ESTATE, "a detection is already queued: collect it first");
        if (int rc = detect_finish(h)) return rc;  // (queued and never collected)
    }
    if ((!frames && !list) || n < 1 || H < 1 || W < 1 || roi_w < 1)
        return hfail(h, FM_EINVAL, "bad arguments (n >= 1, frame and ROI sizes >= 1)");
    const int rw = roi_w, rh = (int)(H * ((double)roi_w / (double)W));  // imutils.resize(raw, width=roi_w)
    if (roi_h_out) *roi_h_out = rh;
    if (rh < 1) return hfail(h, FM_EINVAL, "ROI height 0 for a %dx%d frame", W, H);
    const double sx = 1. / ((double)rw / W), sy = 1. / ((double)rh / H);
    const bool identity = rw == W && rh == H;
    if (!identity && !(sx >= 1 && sy >= 1))
        return hfail(h, FM_ENOTSUP, "frame width %d < ROI width %d: INTER_AREA upscaling is not supported", W, rw);
    HH(h, hipSetDevice(h->device));
    const double t0 = h->times ? hnow() : 0.;
    const size_t fb = (size_t)H * W * 3;
    const uint8_t* src = frames;
    int rc;
    // a frame list: the resize reads each frame where it lies (k_resize_area_nt's address table) when
    // it can; otherwise the frames are gathered on the detector's stream first
    const uint8_t* const* dlist = nullptr;
    if (list) {
        // from page-locked memory: a pageable source made this small copy cost ~0.5 ms of host time per
        // call beside a busy pixel stream (FM_HAAR_TIMES); the previous call's copy is done (each call
        // ends with a stream synchronize)
        if ((size_t)n > h->cap_fptr) {
            if (h->h_fptr) HH(h, hipHostFree((void*)h->h_fptr));
            h->h_fptr = nullptr;
            size_t cap = h->cap_fptr;
            if ((rc = grow(h, &h->d_fptr, cap, (size_t)n))) return rc;
            HH(h, hipHostMalloc((void**)&h->h_fptr, (size_t)n * sizeof(const uint8_t*), 0));
            h->cap_fptr = cap;
        }
        std::memcpy((void*)h->h_fptr, list, (size_t)n * sizeof(const uint8_t*));
        HH(h, hipMemcpyAsync(h->d_fptr, h->h_fptr, (size_t)n * sizeof(const uint8_t*), hipMemcpyHostToDevice, h->stream));
        dlist = h->d_fptr;
    }
    auto gather = [&]() -> int {
        int r = grow(h, &h->d_raw, h->cap_raw, n * fb);
        if (r) return r;
        for (int i = 0; i < n; i++)
            HH(h, hipMemcpyAsync(h->d_raw + (size_t)i * fb, list[i], fb, hipMemcpyDeviceToDevice, h->stream));
        src = h->d_raw;
        dlist = nullptr;
        return FM_OK;
    };
    if (!list && !on_device) {
        if ((rc = grow(h, &h->d_raw, h->cap_raw, n * fb))) return rc;
        HH(h, hipMemcpyAsync(h->d_raw, frames, n * fb, hipMemcpyHostToDevice, h->stream));
        src = h->d_raw;
    }
    const uint8_t* roi = src;
    if (!identity) {
        if ((rc = grow(h, &h->d_roi, h->cap_roi, (size_t)n * rh * rw * 3))) return rc;
        const int isx = (int)std::lrint(sx), isy = (int)std::lrint(sy);
        if (std::fabs(sx - isx) < 2.220446049250313e-16 && std::fabs(sy - isy) < 2.220446049250313e-16) {
            if (dlist && (rc = gather())) return rc;
            HH(h, fm::launch_resize_area_fast(h->stream, src, h->d_roi, n, H, W, rh, rw, isx, isy));
        } else {
            if (h->area_key[0] != W || h->area_key[1] != H || h->area_key[2] != rw || h->area_key[3] != rh) {
                if (!fm::build_area_axis(W, rw, sx, h->ax) || !fm::build_area_axis(H, rh, sy, h->ay))
                    return hfail(h, FM_ENOTSUP, "INTER_AREA table with non-consecutive taps");
                HH(h, hipStreamSynchronize(h->stream));
                for (void* p : {(void*)h->d_axo, (void*)h->d_axc, (void*)h->d_ayo, (void*)h->d_ayc, (void*)h->d_axw,
                                (void*)h->d_ayw})
                    if (p) HH(h, hipFree(p));
                HH(h, hipMalloc((void**)&h->d_axo, h->ax.ofs.size() * 4));
                HH(h, hipMalloc((void**)&h->d_axc, h->ax.cnt.size() * 4));
                HH(h, hipMalloc((void**)&h->d_axw, h->ax.wt.size() * 4));
                HH(h, hipMalloc((void**)&h->d_ayo, h->ay.ofs.size() * 4));
                HH(h, hipMalloc((void**)&h->d_ayc, h->ay.cnt.size() * 4));
                HH(h, hipMalloc((void**)&h->d_ayw, h->ay.wt.size() * 4));
                HH(h, hipMemcpy(h->d_axo, h->ax.ofs.data(), h->ax.ofs.size() * 4, hipMemcpyHostToDevice));
                HH(h, hipMemcpy(h->d_axc, h->ax.cnt.data(), h->ax.cnt.size() * 4, hipMemcpyHostToDevice));
                HH(h, hipMemcpy(h->d_axw, h->ax.wt.data(), h->ax.wt.size() * 4, hipMemcpyHostToDevice));
                HH(h, hipMemcpy(h->d_ayo, h->ay.ofs.data(), h->ay.ofs.size() * 4, hipMemcpyHostToDevice));
                HH(h, hipMemcpy(h->d_ayc, h->ay.cnt.data(), h->ay.cnt.size() * 4, hipMemcpyHostToDevice));
                HH(h, hipMemcpy(h->d_ayw, h->ay.wt.data(), h->ay.wt.size() * 4, hipMemcpyHostToDevice));
                h->area_key[0] = W;
                h->area_key[1] = H;
                h->area_key[2] = rw;
                h->area_key[3] = rh;
            }
            const bool direct = dlist && ((h->ax.max_taps + 1) & ~1) <= 32 && fb < (1u << 31);
            if (dlist && !direct && (rc = gather())) return rc;
            HH(h, fm::launch_resize_area(h->stream, src, h->d_roi, n, H, W, rh, rw, h->d_axo, h->d_axc, h->d_axw,
                                         h->ax.max_taps, h->d_ayo, h->d_ayc, h->d_ayw, h->ay.max_taps, dlist));
        }
        roi = h->d_roi;
    } else if (dlist && (rc = gather())) {
        return rc;
    } else if (list) {
        roi = src;
    }
    if (h->times) h->tph[0] += hnow() - t0;
    if (async) return detect_enqueue(h, roi, n, rh, rw, 3, 1, scale_factor, min_neighbors, 0, 0, 0, 0);
    return fm_haar_detect(h, roi, n, rh, rw, 3, 1, scale_factor, min_neighbors, 0, 0, 0, 0, rects, cap, counts);
}

extern "C" {
int fm_haar_detect_frames(fm_haar* h, const uint8_t* frames, int n, int H, int W, int on_device, int roi_w,
                          double scale_factor, int min_neighbors, int32_t* rects, int cap, int32_t* counts,
                          int* roi_h_out) {
    return detect_frames_impl(h, frames, nullptr, n, H, W, on_device, roi_w, scale_factor, min_neighbors, rects, cap,
                              counts, roi_h_out);
}

int fm_haar_detect_frame_list(fm_haar* h, const uint8_t* const* frames, int n, int H, int W, int roi_w,
                              double scale_factor, int min_neighbors, int32_t* rects, int cap, int32_t* counts,
                              int* roi_h_out) {
    if (!frames) return h ? hfail(h, FM_EINVAL, "null frame list") : FM_EINVAL;
    for (int i = 0; i < n; i++)
        if (!frames[i]) return hfail(h, FM_EINVAL, "frame %d: null address", i);
    return detect_frames_impl(h, nullptr, frames, n, H, W, 1, roi_w, scale_factor, min_neighbors, rects, cap, counts,
                              roi_h_out);
}

int fm_haar_detect_frame_list_async(fm_haar* h, const uint8_t* const* frames, int n, int H, int W, int roi_w,
                                    double scale_factor, int min_neighbors, int* roi_h_out) {
    if (!frames) return h ? hfail(h, FM_EINVAL, "null frame list") : FM_EINVAL;
    for (int i = 0; i < n; i++)
        if (!frames[i]) return hfail(h, FM_EINVAL, "frame %d: null address", i);
    return detect_frames_impl(h, nullptr, frames, n, H, W, 1, roi_w, scale_factor, min_neighbors, nullptr, 0, nullptr,
                              roi_h_out, true);
}

int fm_haar_collect(fm_haar* h, int32_t* rects, int cap, int32_t* counts, int n) {
    if (!h) return FM_EINVAL;
    if (cap < 0 || !counts || (cap > 0 && !rects)) return hfail(h, FM_EINVAL, "bad arguments (counts[n], rects[n][cap])");
    if (int rc = detect_finish(h)) return rc;
    if (n != (int)h->out.size()) return hfail(h, FM_ESTATE, "%d images asked for, the last detection had %zu", n, h->out.size());
    detect_copy(h, rects, cap, counts);
    return FM_OK;
}

}  // extern "C"
