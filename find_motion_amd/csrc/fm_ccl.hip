// fm_ccl.hip — findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) count + boundingRect
// on the GPU (gfx950); reference call site fm.py:269-272, consumer fm.py:674-694.
//
// Semantics (checked against the literal Suzuki-Abe
// restatement in oracle/fm_oracle.c): foreground 8-connected, background
// 4-connected; a foreground component yields one external contour iff the
// background component left of its raster-first pixel touches the image
// border (= the 1-px zero pad).  boundingRect = the component's pixel bbox.
//
// Work is proportional to motion.  A tile is a CANDIDATE when its dilated mask
// can be non-empty: it has threshold bits, or a neighbour has them within 2 px
// of the shared edge/corner (per-tile flags written by the pixel kernel).
// Every other tile is empty background.  Union-find nodes of a batch slot:
// node f*ntiles + r for the empty-tile region represented by tile r of frame f,
// then a pool from which each labelled candidate tile takes one node per
// component (TileRec::nbase + ordinal) -- memory follows the motion present, not
// the worst case.
//   k_regions    one workgroup per frame: candidate list; empty tiles grouped
//                into 4-connected regions in LDS, one node per region (at its
//                representative tile), "outer" when the region reaches the grid border.
//   k_tile_ccl   one wave per candidate: 5x5 dilation of its bit rows
//                (fm.py:266), run-length labelling in LDS (256 runs), a tile
//                record (edge labels) and one node per component.
//   k_tile_heavy tiles with more runs (a dense texture of blobs): persistent waves,
//                kTileMaxRuns runs each in 46 KB of LDS.
//   k_merge      one wave per candidate: unions along its edges with candidate
//                neighbours (right / below) and empty regions (all sides).
//   k_fold       one wave per candidate tile (lanes = its components) or region:
//                path compression with outer flags, bboxes and raster-first
//                pixels folded into the roots.
//   k_emit       one wave per candidate tile: the external test at each
//                foreground root and the contour records (mapped host memory).
//   k_counts     per frame: counts / overflow flags into mapped host memory.
// A frame whose tiles exhaust the scratch slots or the node pool is flagged
// (count[F+f]); the host relabels it with the pixel-level CCL of fm_kernels.hip.
#include "fm_internal.h"

namespace fm {
namespace cc {

constexpr int TS = 64;
constexpr int MAXR = kTileMaxRuns;
constexpr int LIGHT = 256;      // runs held by the light pass
constexpr int CW = 4;           // waves (tiles) per workgroup in k_tile_ccl / k_merge
// workgroups per frame in k_tile_ccl / k_merge / k_fold / k_emit.  Measured: with the labelling gate
// (round 3) 4 392.3k, 6 389.0k, 8 388.4k frames/s (4 alternating rounds)
constexpr int GW = 4;  // (round 5 with ten slots: 4 / 3 / 2 -> 402-407 / 404-413 / 395-406 k, 3 alternating rounds)
constexpr int RG = 512;         // k_regions threads
// The contour waves run at the pixel waves' issue priority 0.  (Raised -- labelling 2, heavy tiles 3,
// merge 2 -- they gained 4 % in round 2; in round 3, 0 gave the same throughput, 368.1 vs 368.2 k,
// with 6 % shorter pixel launches; every contour kernel at 3: 402.7 vs 413.3 k, round 4.)
constexpr int MAX_REGION_TILES = 8192;
static_assert(MAX_REGION_TILES <= 32 * RG, "k_regions keeps one candidate bit per tile of a thread in a u32");
constexpr uint32_t REF_OUTER = 0x80000000u;
constexpr uint32_t REF_EDGE = 0x40000000u;

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ int lload(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// find with path halving (a pointer only ever moves to a smaller member of the
// same set, so halving by atomicMin cannot undo a concurrent link)
__device__ __forceinline__ int lfind(int* P, int x) {
    for (;;) {
        const int p = lload(&P[x]);
        if (p == x) return x;
        const int gp = lload(&P[p]);
        if (gp == p) return p;
        atomicMin(&P[x], gp);
        x = gp;
    }
}
// link the larger root under the smaller: a root is its set's smallest member
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
// find with path halving by atomicMin: a pointer only moves to a smaller member
// of the same set, so it cannot undo a concurrent link
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

__device__ __forceinline__ bool tile_on_border(const FusedArgs& a, int ti) {
    const int tx = ti % a.ntx, ty = ti / a.ntx;
    return tx == 0 || ty == 0 || tx == a.ntx - 1 || ty == a.nty - 1;
}

// ---------------------------------------------------------------------------
// dilate(thresh, None, iterations=2) = 5x5 max (fm.py:266).  The pixel kernel writes each
// tile's threshold bits column-major (word c = column c, bit r = row r), so the vertical
// half of the separable dilation is shifts inside a word (the tiles above and below give
// rows -2, -1 and 64, 65), the horizontal half is lane shuffles (lane = column; the left
// and right tiles give columns -2, -1 and 64, 65), and one 64x64 bit transpose turns the
// dilated tile into the row words (lane = row) the run-length labelling walks.
__device__ __forceinline__ uint64_t vdil(const uint64_t* B, const FusedArgs& a, int t, int ty, int c) {
    const uint64_t x = B[(size_t)t * 64 + c];
    uint64_t v = x | (x << 1) | (x << 2) | (x >> 1) | (x >> 2);
    if (ty > 0) {  // rows -1 (bit 63) and -2 (bit 62) of the tile above
        const uint64_t u = B[(size_t)(t - a.ntx) * 64 + c];
        v |= ((u >> 63) ? 3ull : 0ull) | ((u >> 62) & 1ull);
    }
    if (ty + 1 < a.nty) {  // rows 64 (bit 0) and 65 (bit 1) of the tile below
        const uint64_t d = B[(size_t)(t + a.ntx) * 64 + c];
        v |= ((d & 1ull) ? (3ull << 62) : 0ull) | (((d >> 1) & 1ull) << 63);
    }
    return v;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src, 64), hi = __shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int lane) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane), hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Wave-wide inclusive prefix sum by DPP (row_shr 1, 2, 4, 8 inside each 16-lane row, then
// row_bcast 15 / 31 across rows): six VALU adds, where a __shfl_up loop is six ds_bpermute
// round trips through the LDS unit (the DPP scans: +1.5 %, 373.0 vs 367.6 k, 4 rounds, round 3).
// Needs every lane active (callers are in wave-uniform flow).
__device__ __forceinline__ int wave_incl_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
// __shfl_up(v, 1) / __shfl_down(v, 1) (lane 0 / 63 keep their own value) by DPP wave shifts
__device__ __forceinline__ int lane_up1(int v) {
    return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ int lane_down1(int v) {
    return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false);  // wave_shl:1
}
__device__ __forceinline__ uint64_t lane_down1_64(uint64_t v) {
    return ((uint64_t)(uint32_t)lane_down1((int)(uint32_t)(v >> 32)) << 32) | (uint32_t)lane_down1((int)(uint32_t)v);
}
// a lane's value broadcast (v_readlane)
__device__ __forceinline__ int lane_at(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ uint64_t lane_at64(uint64_t v, int lane) {
    return ((uint64_t)(uint32_t)lane_at((int)(uint32_t)(v >> 32), lane) << 32) | (uint32_t)lane_at((int)(uint32_t)v, lane);
}

// the value of lane ln ^ J, without LDS: v_permlane32_swap / v_permlane16_swap for 32 / 16, DPP
// row_ror:8 for 8, row_half_mirror then a reversed quad_perm for 4, quad_perm for 2 and 1
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int ln) {
    if constexpr (J == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return ln < 32 ? r[1] : r[0];
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (ln & 16) ? r[0] : r[1];
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
    } else if constexpr (J == 4) {
        const int m = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);
        return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, true);
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
    } else {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
    }
}
template <int J>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v, int ln) {
    return ((uint64_t)lane_xor<J>((uint32_t)(v >> 32), ln) << 32) | lane_xor<J>((uint32_t)v, ln);
}

// 64x64 bit transpose across the wave: lane k holds word k; afterwards lane r holds the
// word whose bit c is bit r of the old word c
__device__ __forceinline__ uint64_t transpose64(uint64_t w, int ln) {
    const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                               0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int s = 0; s < 6; s++) {
        const int j = 32 >> s;
        const uint64_t p = j == 32 ? lane_xor64<32>(w, ln) : j == 16 ? lane_xor64<16>(w, ln) : j == 8 ? lane_xor64<8>(w, ln)
                         : j == 4 ? lane_xor64<4>(w, ln) : j == 2 ? lane_xor64<2>(w, ln) : lane_xor64<1>(w, ln);
        if (ln & j) w ^= ((p >> j) ^ w) & masks[s];
        else w ^= (((w >> j) ^ p) & masks[s]) << j;
    }
    return w;
}

__device__ __forceinline__ uint64_t dilate_tile(const FusedArgs& a, size_t f, int ti, int ln, uint64_t* hv) {
    (void)hv;
    const int tx = ti % a.ntx, ty = ti / a.ntx;
    const uint64_t* B = a.bits + f * (size_t)a.ntiles * 64;
    const bool hl = tx > 0, hr = tx + 1 < a.ntx;
    // columns of the neighbours: lanes 62, 63 hold the left tile's columns 62, 63, lanes 0, 1 the
    // right tile's columns 0, 1 (every lane loads its side column unconditionally -- its own tile's
    // where there is none -- so all six loads are in flight together)
    const int st = (ln >= 62 && hl) ? ti - 1 : (ln <= 1 && hr) ? ti + 1 : ti;
    const uint64_t v = vdil(B, a, ti, ty, ln);
    uint64_t e = vdil(B, a, st, ty, ln);
    if (st == ti) e = 0;
    // neighbour columns by DPP wave shifts (wave_shr:1: lane i <- i-1; wave_shl:1: lane i <- i+1),
    // the four neighbour-tile columns by readlane
    const uint64_t vm1 = dpp64<0x138>(v), vm2 = dpp64<0x138>(vm1);
    const uint64_t vp1 = dpp64<0x130>(v), vp2 = dpp64<0x130>(vp1);
    const uint64_t e62 = rdl64(e, 62), e63 = rdl64(e, 63), e0 = rdl64(e, 0), e1 = rdl64(e, 1);
    uint64_t o = v;
    o |= ln >= 1 ? vm1 : e63;
    o |= ln >= 2 ? vm2 : (ln == 1 ? e63 : e62);
    o |= ln <= 62 ? vp1 : e0;
    o |= ln <= 61 ? vp2 : (ln == 62 ? e0 : e1);
    // columns / rows outside the image are background
    const int x0 = tx * TS, y0 = ty * TS;
    if (x0 + ln >= a.w) o = 0;
    const int vr = a.h - y0;
    if (vr < 64) o &= (1ull << vr) - 1;
    return transpose64(o, ln);
}

// ---------------------------------------------------------------------------
// Run-length CCL of one dilated 64x64 tile (one wave, lane = tile row).
// Runs are numbered in raster order; union-find over runs links the larger
// root under the smaller, so a root is its component's raster-first run.
// Foreground runs of adjacent rows connect 8-wise (x ranges within 1),
// background runs 4-wise (x ranges overlap).  Out-of-image pixels are
// background and, like pixels on the image border, mark their background
// component "outer".  Output: TileRec (nroots, edge labels as component
// ordinals | fg << 15) and NodeRec[ordinal].
struct Scratch {
    int* par;
    int* amin;  // fg root: min x0; bg root: outer flag
    int* amax;
    int* ay;
    uint8_t *rx0, *rx1, *rf;
    int* rb;
    uint16_t* ord;
    uint32_t* pairs;  // run pairs (a | b << 16) to union, capacity 2 * CAP
};

// run index (in the tile's raster numbering) of the run of row `base` / `starts` holding bit p
__device__ __forceinline__ int run_at(int base, uint64_t starts, int p) {
    return base + __popcll(starts & ((2ull << p) - 1)) - 1;
}

#define FM_STAMP(k)                                                                          \
    do {                                                                                     \
        if (a.dbg_ts && ln == 0) a.dbg_ts[((size_t)f * a.ntiles + ti) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

enum : int { TCCL_OK = 0, TCCL_RUNS = 1, TCCL_NODES = 2 };


// the tile's node ids: n consecutive ids from its frame's quota (one counter per frame, so
// the tiles of different frames never contend on one atomic), or past the quota from the
// slot's shared overflow pool; -1 (TCCL_NODES) when that is exhausted too: the frame is
// relabelled by the pixel-level fallback
__device__ __forceinline__ int take_nodes(const FusedArgs& a, size_t f, int n, int ln) {
    const size_t F = (size_t)a.T * a.S;
    const long long q0 = (long long)F * a.ntiles, sh0 = q0 + (long long)F * a.nquota;
    long long first = -1;
    if (ln == 0) {
        const int b = atomicAdd(&a.count[2 * F + 2 + f], n);
        if (b + n <= a.nquota) {
            first = q0 + (long long)f * a.nquota + b;
        } else {
            const int c = atomicAdd(&a.count[2 * F], n);
            if (sh0 + c + n <= (long long)a.nnodes) first = sh0 + c;
        }
    }
    return lane_at((int)first, 0);
}


// bits lo..hi of a 64-bit word (0 <= lo <= hi <= 63)
__device__ __forceinline__ uint64_t bits_between(int lo, int hi) {
    return (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & ~((1ull << lo) - 1);
}
__device__ __forceinline__ int hibit(uint64_t v) { return 63 - __builtin_clzll(v); }  // v != 0

// Simple tiles (round 5): every row of the dilated tile holds at most one foreground run, the rows with one are
// consecutive (r0..r1), and each run touches the one above 8-wise -- one foreground component.  The background
// is then a top region (rows < r0), a bottom region (rows > r1), the runs left of the foreground (x 0 .. xs-1)
// in chains of consecutive rows, and the runs right of it (xe+1 .. 63) likewise: a left run never meets a right
// run of the next row (that would need a gap that breaks the 8-connection), so a chain is one component, or
// part of the top region's (it includes row r0) or the bottom region's (row r1).  Components, their raster-first
// runs (roots), ordinals, outer flags, bounding box, left-background reference and the four edge-label rows come
// from ballots and bit counts: the same TileRec and NodeRecs the run labelling below writes, without the run
// records, the pair lists and the union rounds.  Returns false (nothing written) if the tile is not simple.
__device__ __forceinline__ bool simple_tile(const FusedArgs& a, size_t f, int ti, int ln, uint64_t m, int& rc) {
    const int h = a.h, w = a.w;
    const int x0 = (ti % a.ntx) * TS, y0 = (ti / a.ntx) * TS;
    const uint64_t fgs = m & ~(m << 1);  // foreground run starts
    const int nfg = __popcll(fgs);
    const uint64_t band = __builtin_amdgcn_ballot_w64(nfg == 1);
    if (__builtin_amdgcn_ballot_w64(nfg > 1) != 0 || band == 0) return false;
    const int r0 = __builtin_ctzll(band), r1 = hibit(band);
    if (band != bits_between(r0, r1)) return false;
    const bool in = ln >= r0 && ln <= r1;
    const int xs = in ? __builtin_ctzll(m) : 64, xe = in ? hibit(m) : -1;
    const int xsu = lane_up1(xs), xeu = lane_up1(xe);  // the row above
    if (__builtin_amdgcn_ballot_w64(in && ln > r0 && !(xs <= xeu + 1 && xe >= xsu - 1)) != 0) return false;
    // background chains
    const bool hasL = in && xs > 0, hasR = in && xe < 63;
    const uint64_t Lm = __builtin_amdgcn_ballot_w64(hasL), Rm = __builtin_amdgcn_ballot_w64(hasR);
    const uint64_t Ls = Lm & ~(Lm << 1), Rs = Rm & ~(Rm << 1);  // chain starts
    const uint64_t Le = Lm & ~(Lm >> 1), Re = Rm & ~(Rm >> 1);  // chain ends
    const bool top = r0 > 0, bot = r1 < 63;
    const uint64_t bandm = bits_between(r0, r1);
    const bool mergeTB = top && bot && ((Lm & bandm) == bandm || (Rm & bandm) == bandm);
    const bool L0 = (Lm >> r0) & 1, R0 = (Rm >> r0) & 1, L1 = (Lm >> r1) & 1, R1 = (Rm >> r1) & 1;
    const int sL1 = L1 ? hibit(Ls & bits_between(0, r1)) : 0, sR1 = R1 ? hibit(Rs & bits_between(0, r1)) : 0;
    // roots: x = 0 runs (RL), the foreground (row r0), right runs (RR)
    uint64_t RL = Ls, RR = Rs;
    if (top) {  // the chains through row r0 belong to the top region, whose root is row 0's run
        RL &= ~(1ull << r0);
        RR &= ~(1ull << r0);
        RL |= 1ull;
    }
    if (bot) {  // the chains through row r1 belong to the bottom region
        if (L1) RL &= ~(1ull << sL1);
        if (R1) RR &= ~(1ull << sR1);
    }
    int brow = 0;
    bool bright = false;  // the bottom region's root: row, and whether it is a right run
    if (bot && !mergeTB) {
        // its earliest run: a chain through r1 that does not belong to the top region, or row r1 + 1
        const bool lt = L1 && !(top && sL1 == r0), rt = R1 && !(top && sR1 == r0);
        brow = r1 + 1;
        if (rt && sR1 < brow) brow = sR1, bright = true;
        if (lt && sL1 <= brow) brow = sL1, bright = false;
        if (bright) RR |= 1ull << brow;
        else RL |= 1ull << brow;
    }
    const int nroots = __popcll(RL) + __popcll(RR) + 1;
    if (nroots > 64) return false;
    auto rank = [&](int row, int cls) -> int {  // ordinal of the root at (row, class 0 left / 1 fg / 2 right)
        const uint64_t below = row >= 64 ? ~0ull : ((1ull << row) - 1);
        int r = __popcll(RL & below) + __popcll(RR & below) + (row > r0 ? 1 : 0);
        if (cls >= 1) r += (int)((RL >> row) & 1);
        if (cls == 2 && row == r0) r += 1;
        return r;
    };
    const int ordT = 0;
    const int ordF = rank(r0, 1);
    const int ordB = !bot ? -1 : mergeTB ? ordT : rank(brow, bright ? 2 : 0);
    // component of row ln's left / right run (chains identified by their start row)
    auto comp_left = [&](int row) -> int {
        const int st = hibit(Ls & bits_between(0, row));
        const int en = __builtin_ctzll(Le & bits_between(row, 63));
        if (top && st == r0) return ordT;
        if (bot && en == r1) return ordB;
        return rank(st, 0);
    };
    auto comp_right = [&](int row) -> int {
        const int st = hibit(Rs & bits_between(0, row));
        const int en = __builtin_ctzll(Re & bits_between(row, 63));
        if (top && st == r0) return ordT;
        if (bot && en == r1) return ordB;
        return rank(st, 2);
    };
    // outer runs (background touching the image border or beyond it), per row
    const int gy = y0 + ln;
    const bool rowo = gy == 0 || gy >= h - 1;
    const bool oL = hasL && (x0 == 0 || x0 + xs - 1 >= w - 1 || rowo);
    const bool oR = hasR && (x0 + 63 >= w - 1 || rowo);
    const bool oRow = !in && (x0 == 0 || x0 + 63 >= w - 1 || rowo);
    const uint64_t OL = __builtin_amdgcn_ballot_w64(oL), OR = __builtin_amdgcn_ballot_w64(oR),
                   ORow = __builtin_amdgcn_ballot_w64(oRow);
    auto chain_mask = [&](uint64_t S, uint64_t E, int row) -> uint64_t {  // the chain through `row`
        return bits_between(hibit(S & bits_between(0, row)), __builtin_ctzll(E & bits_between(row, 63)));
    };
    bool outT = false, outB = false;
    if (top) {
        outT = (ORow & bits_between(0, r0 - 1)) != 0;
        if (L0) outT |= (OL & chain_mask(Ls, Le, r0)) != 0;
        if (R0) outT |= (OR & chain_mask(Rs, Re, r0)) != 0;
    }
    if (bot) {
        outB = (ORow & bits_between(r1 + 1, 63)) != 0;
        if (L1) outB |= (OL & chain_mask(Ls, Le, r1)) != 0;
        if (R1) outB |= (OR & chain_mask(Rs, Re, r1)) != 0;
        if (mergeTB) outT = outB = outT || outB;
    }
    const int nb = take_nodes(a, f, nroots, ln);
    if (nb < 0) {
        rc = TCCL_NODES;
        return true;
    }
    TileRec* TR = a.tiles + f * a.ntiles + ti;
    if (ln == 63) {
        TR->nroots = nroots;
        TR->nbase = nb;
    }
    if (FM_OOB(a, (long long)nb + nroots <= (long long)a.nnodes, 3)) {
        rc = TCCL_NODES;
        return true;
    }
    NodeRec* NR = a.nodes + nb;
    // the roots of row ln: its left run, the foreground (row r0), its right run
    auto bg_node = [&](int ord, bool outer) {
        NodeRec nrec;
        nrec.key = 0;
        nrec.parent = nb + ord;
        nrec.flags = outer ? 2u : 0u;
        nrec.minx = nrec.maxx = nrec.maxy = nrec.pad = 0;
        NR[ord] = nrec;
    };
    if ((RL >> ln) & 1) {
        bool outer;
        if (top && ln == 0) outer = outT;
        else if (bot && !mergeTB && !bright && ln == brow) outer = outB;
        else outer = (OL & chain_mask(Ls, Le, ln)) != 0;
        bg_node(rank(ln, 0), outer);
    }
    if ((RR >> ln) & 1) {
        const bool outer = (bot && !mergeTB && bright && ln == brow) ? outB : (OR & chain_mask(Rs, Re, ln)) != 0;
        bg_node(rank(ln, 2), outer);
    }
    // the foreground component's record: bbox over the band, raster-first pixel, the background left of it
    int mn = in ? xs : 64, mx = xe;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, __shfl_xor(mn, o));
        mx = max(mx, __shfl_xor(mx, o));
    }
    if (ln == r0) {
        uint32_t ref;
        if (x0 + xs == 0) ref = REF_OUTER;
        else if (xs == 0) ref = REF_EDGE | (uint32_t)ln;
        else ref = (uint32_t)comp_left(ln);
        NodeRec nrec;
        nrec.key = ((uint64_t)(uint32_t)(gy * w + x0 + xs) << 32) | ref;
        nrec.parent = nb + ordF;
        nrec.flags = 1u;
        nrec.minx = x0 + mn;
        nrec.maxx = x0 + mx;
        nrec.maxy = y0 + r1;
        nrec.pad = 0;
        NR[ordF] = nrec;
    }
    // edge labels: component ordinal | fg << 15
    const uint16_t FG = (uint16_t)(ordF | 0x8000);
    auto row_label = [&](int row, int c) -> uint16_t {  // pixel (row, c)
        if (row < r0) return (uint16_t)ordT;
        if (row > r1) return (uint16_t)ordB;
        const int rxs = lane_at(xs, row), rxe = lane_at(xe, row);
        if (c < rxs) return (uint16_t)comp_left(row);
        if (c > rxe) return (uint16_t)comp_right(row);
        return FG;
    };
    TR->edges[ln] = !in ? (uint16_t)(ln < r0 ? ordT : ordB) : xs == 0 ? FG : (uint16_t)comp_left(ln);
    TR->edges[64 + ln] = !in ? (uint16_t)(ln < r0 ? ordT : ordB) : xe == 63 ? FG : (uint16_t)comp_right(ln);
    TR->edges[128 + ln] = row_label(0, ln);
    TR->edges[192 + ln] = row_label(63, ln);
    rc = TCCL_OK;
    return true;
}

// Tiles that are neither simple nor full, with at most 64 runs once each streak of identical consecutive rows is
// kept once (the bench video's other tiles: the jagged edges of large regions, ~100 runs over 64 rows, ~30 runs over
// ~10 distinct rows).  A row identical to the one above adds nothing to the components -- each of its runs touches
// exactly the same run above and nothing else -- so it takes the labels of its streak's first row, and the streak's
// last row is the runs' lowest row.  With one lane per run instead of one per row there are no per-row run loops:
// a run finds its row from a ballot of the rows' first runs, its extent by clearing the row's lower run starts, the
// runs it touches in the row above as one range; the union rounds run over those ranges, the fold by LDS atomics,
// ordinals and the root count by ballot.  Writes the same TileRec and NodeRecs as the run labelling below (roots are
// raster-first runs, which never lie in a repeated row).  Returns false (nothing written) past 64 runs.
__device__ __forceinline__ uint64_t lane_up1_64(uint64_t v) {
    return ((uint64_t)(uint32_t)lane_up1((int)(uint32_t)(v >> 32)) << 32) | (uint32_t)lane_up1((int)(uint32_t)v);
}
__device__ __forceinline__ bool compact_tile(const FusedArgs& a, size_t f, int ti, int ln, uint64_t m, const Scratch& sc,
                                             int& rc) {
    const int h = a.h, w = a.w;
    const int x0 = (ti % a.ntx) * TS, y0 = (ti / a.ntx) * TS;
    // ---- lane = row
    const uint64_t starts = (m ^ (m << 1)) | 1ull;  // run starts (bit 0 always)
    const uint64_t mu = lane_up1_64(m), su = lane_up1_64(starts);  // the row above (row 0: its own)
    const bool dup = ln > 0 && m == mu;
    const int nrr = __popcll(starts);
    const int nr = dup ? 0 : nrr;
    const int incl = wave_incl_sum(nr);
    const int total = lane_at(incl, 63);
    if (total > 64) return false;
    const int base = incl - nr;
    const uint64_t ND = __builtin_amdgcn_ballot_w64(!dup);  // each streak's first row (bit 0 always)
    const int sr = hibit(ND & bits_between(0, ln));
    const uint64_t nxt = ND & ~bits_between(0, ln);
    const int se = nxt ? __builtin_ctzll(nxt) - 1 : 63;  // the streak's last row
    const int bs = __shfl(base, sr, 64);                 // the streak's first run
    const int ab = lane_up1(bs);                         // first run of the row above (its streak's)
    int* mark = sc.rb;
    int* aux = reinterpret_cast<int*>(sc.ord);
    uint4* rows = reinterpret_cast<uint4*>(sc.pairs);
    mark[ln] = 0;
    if (nr > 0) mark[base] = ln + 1;  // (same wave: the stores land in order)
    rows[2 * ln] = make_uint4((uint32_t)starts, (uint32_t)(starts >> 32), (uint32_t)m, (uint32_t)(m >> 32));
    rows[2 * ln + 1] = make_uint4((uint32_t)su, (uint32_t)(su >> 32), (uint32_t)mu, (uint32_t)(mu >> 32));
    aux[ln] = ab | (se << 8);
    lds_fence();
    // ---- lane = run (ln < total)
    const bool live = ln < total;
    const int mk = mark[ln];
    const uint64_t SEG = __builtin_amdgcn_ballot_w64(mk != 0);  // runs that start a row (bit 0 always)
    const int st = hibit(SEG & bits_between(0, ln));
    const int r = __shfl(mk, st, 64) - 1;  // the run's row
    const int k = live ? ln - st : 0;      // its index in the row
    const uint4 q0 = rows[2 * r], q1 = rows[2 * r + 1];
    const int ax = aux[r];
    uint64_t sk = (uint64_t)q0.x | ((uint64_t)q0.y << 32);
    const uint64_t mr = (uint64_t)q0.z | ((uint64_t)q0.w << 32);
    for (int i = 0; i < k; i++) sk &= sk - 1;
    const int xs = __builtin_ctzll(sk);
    const uint64_t sk2 = sk & (sk - 1);
    const int xe = sk2 ? __builtin_ctzll(sk2) - 1 : 63;
    const bool fg = (mr >> xs) & 1;
    const int rab = ax & 0xFF, rse = ax >> 8;
    // the same-colour runs it touches in the row above: ia, ia + 2, .., ib (8-connected foreground, 4-connected background)
    int ia = 1, ib = 0;
    if (live && r > 0) {
        const uint64_t sU = (uint64_t)q1.x | ((uint64_t)q1.y << 32), mU = (uint64_t)q1.z | ((uint64_t)q1.w << 32);
        const int w0 = fg ? max(xs - 1, 0) : xs, w1 = fg ? min(xe + 1, 63) : xe;
        const uint64_t hits = (fg ? mU : ~mU) & bits_between(w0, w1);
        if (hits) {
            ia = run_at(rab, sU, __builtin_ctzll(hits));
            ib = run_at(rab, sU, hibit(hits));
        }
    }
    int* par = sc.par;
    int* amin = sc.amin;
    int* amax = sc.amax;
    int* ay = sc.ay;
    if (live) par[ln] = ln;
    lds_fence();
    // union rounds as tile_ccl's (hook the larger parent under the smaller, then shortcut)
    for (int round = 0; round < 64; round++) {
        bool ch = false;
        for (int j = ia; j <= ib; j += 2) {
            const int ra = lload(&par[ln]), rb2 = lload(&par[j]);
            if (ra != rb2) {
                atomicMin(&par[max(ra, rb2)], min(ra, rb2));
                ch = true;
            }
        }
        lds_fence();
        if (live) {
            const int pi = lload(&par[ln]);
            const int ppi = lload(&par[pi]);
            if (ppi != pi) {
                atomicMin(&par[ln], ppi);
                ch = true;
            }
        }
        lds_fence();
        if (__builtin_amdgcn_ballot_w64(ch) == 0) break;
    }
    // fold into the roots: bounding box and lowest row of foreground components, the outer flag of background ones
    const int gy = y0 + r;
    const bool outer = !fg && (x0 + xs == 0 || x0 + xe >= w - 1 || gy == 0 || y0 + rse >= h - 1);
    const int rt = live ? lload(&par[ln]) : ln;
    if (live) {
        amin[ln] = fg ? xs : (int)outer;
        amax[ln] = xe;
        ay[ln] = rse;
    }
    lds_fence();
    if (live && rt != ln) {
        if (fg) {
            atomicMin(&amin[rt], xs);
            atomicMax(&amax[rt], xe);
            atomicMax(&ay[rt], rse);
        } else if (outer) {
            atomicOr(&amin[rt], 1);
        }
    }
    lds_fence();
    const uint64_t RM = __builtin_amdgcn_ballot_w64(live && rt == ln);  // roots, in raster order
    const int nroots = __popcll(RM);
    auto ordof = [&](int root) -> int { return __popcll(RM & ((1ull << root) - 1)); };
    const int nb = take_nodes(a, f, nroots, ln);
    if (nb < 0) {
        rc = TCCL_NODES;
        return true;
    }
    TileRec* TR = a.tiles + f * a.ntiles + ti;
    if (ln == 63) {
        TR->nroots = nroots;
        TR->nbase = nb;
    }
    if (FM_OOB(a, (long long)nb + nroots <= (long long)a.nnodes, 3)) {
        rc = TCCL_NODES;
        return true;
    }
    NodeRec* NR = a.nodes + nb;
    if (live && rt == ln) {
        const int o = ordof(ln);
        NodeRec nrec;
        nrec.parent = nb + o;
        nrec.key = 0;
        nrec.minx = nrec.maxx = nrec.maxy = nrec.pad = 0;
        if (fg) {
            uint32_t ref;
            if (x0 + xs == 0) ref = REF_OUTER;
            else if (xs == 0) ref = REF_EDGE | (uint32_t)r;
            else ref = (uint32_t)ordof(lload(&par[ln - 1]));  // the background run left of it (same row: k > 0)
            nrec.key = ((uint64_t)(uint32_t)(gy * w + x0 + xs) << 32) | ref;
            nrec.flags = 1u;
            nrec.minx = x0 + amin[ln];
            nrec.maxx = x0 + amax[ln];
            nrec.maxy = y0 + ay[ln];
        } else {
            nrec.flags = amin[ln] ? 2u : 0u;
        }
        NR[o] = nrec;
    }
    // ---- lane = row again: edge labels (component ordinal | fg << 15)
    const uint64_t mask_c = (2ull << ln) - 1;
    const uint64_t s0 = lane_at64(starts, 0), m0 = lane_at64(m, 0);
    const uint64_t s63 = lane_at64(starts, 63), m63 = lane_at64(m, 63);
    const int id0 = __popcll(s0 & mask_c) - 1;
    const int id63 = lane_at(bs, 63) + __popcll(s63 & mask_c) - 1;
    TR->edges[ln] = (uint16_t)(ordof(lload(&par[bs])) | (int)((m & 1ull) << 15));
    TR->edges[64 + ln] = (uint16_t)(ordof(lload(&par[bs + nrr - 1])) | (int)((m >> 63) << 15));
    TR->edges[128 + ln] = (uint16_t)(ordof(lload(&par[id0])) | (int)(((m0 >> ln) & 1ull) << 15));
    TR->edges[192 + ln] = (uint16_t)(ordof(lload(&par[id63])) | (int)(((m63 >> ln) & 1ull) << 15));
    rc = TCCL_OK;
    return true;
}

// TCCL_RUNS (nothing written) if the tile has more than CAP runs
template <int CAP>
__device__ int tile_ccl(const FusedArgs& a, size_t f, int ti, int ln, uint64_t m, const Scratch& sc) {
    int* par = sc.par;
    int* amin = sc.amin;
    int* amax = sc.amax;
    int* ay = sc.ay;
    uint8_t* rx0 = sc.rx0;
    uint8_t* rx1 = sc.rx1;
    uint8_t* rf = sc.rf;
    int* rb = sc.rb;
    uint16_t* ord = sc.ord;
    const int h = a.h, w = a.w;
    const int x0 = (ti % a.ntx) * TS, y0 = (ti / a.ntx) * TS;
    TileRec* TR = a.tiles + f * a.ntiles + ti;

    bool empty = __ballot(m != 0) == 0;
#ifdef FM_DEV_SWITCHES
    // profiling-only ablations (results invalid): 512 = every tile that is not full takes the empty-tile
    // record; 256 = every tile that is neither full nor simple does
    if ((a.dbg_skip & 512) && __ballot(m != ~0ull) != 0) empty = true;
    if ((a.dbg_skip & 256) && !empty && __ballot(m != ~0ull) != 0) {
        int rc = TCCL_OK;
        if (simple_tile(a, f, ti, ln, m, rc)) return rc;
        empty = true;
    }
#endif
    if (empty) {  // empty tile: one background component
        const int nb = take_nodes(a, f, 1, ln);
        if (nb < 0) return TCCL_NODES;
        TR->edges[ln] = 0;
        TR->edges[64 + ln] = 0;
        TR->edges[128 + ln] = 0;
        TR->edges[192 + ln] = 0;
        if (ln == 0) {
            TR->nroots = 1;
            TR->nbase = nb;
            const bool outer = x0 == 0 || y0 == 0 || x0 + TS - 1 >= w - 1 || y0 + TS - 1 >= h - 1;
            NodeRec nrec;
            nrec.key = 0;
            nrec.parent = nb;
            nrec.flags = outer ? 2u : 0u;
            nrec.minx = nrec.maxx = nrec.maxy = nrec.pad = 0;
            a.nodes[nb] = nrec;
        }
        return TCCL_OK;
    }
    // full tile (every pixel set after dilation; tiles cut by the image edge never are): one
    // foreground component whose root is run 0 = row 0, columns 0..63, and no background -- what the
    // labelling below ends with after its ~7 pointer-jumping rounds over the 64-run chain
    if (__ballot(m != ~0ull) == 0) {  // a fully set tile takes a closed-form record (no run labelling)
        const int nb = take_nodes(a, f, 1, ln);
        if (nb < 0) return TCCL_NODES;
        TR->edges[ln] = 0x8000u;
        TR->edges[64 + ln] = 0x8000u;
        TR->edges[128 + ln] = 0x8000u;
        TR->edges[192 + ln] = 0x8000u;
        if (ln == 0) {
            TR->nroots = 1;
            TR->nbase = nb;
            NodeRec nrec;
            nrec.key = ((uint64_t)(uint32_t)(y0 * w + x0) << 32) | (x0 == 0 ? REF_OUTER : REF_EDGE);
            nrec.parent = nb;
            nrec.flags = 1u;
            nrec.minx = x0;
            nrec.maxx = x0 + TS - 1;
            nrec.maxy = y0 + TS - 1;
            nrec.pad = 0;
            a.nodes[nb] = nrec;
        }
        return TCCL_OK;
    }

    {  // one foreground run per row at most, one component: closed-form records (68 % of the bench video's
       // non-empty tiles; the driver's command 405.9 -> 416.6 k frames/s, 3 alternating rounds, round 5)
        int rc = TCCL_OK;
        if (simple_tile(a, f, ti, ln, m, rc)) return rc;
        if (compact_tile(a, f, ti, ln, m, sc, rc)) return rc;
    }
    const uint64_t starts = (m ^ (m << 1)) | 1ull;  // run starts (bit 0 always)
    const int nr = __popcll(starts);
    const int incl = wave_incl_sum(nr);
    const int total = lane_at(incl, 63);
    const int base = incl - nr;
    if (total > CAP) return TCCL_RUNS;
    FM_STAMP(3);
    rb[ln] = base;
    if (ln == 63) rb[64] = total;
    const int gy = y0 + ln;
    {
        uint64_t sb = starts;
        int id = base;
        while (sb) {
            const int xs = __builtin_ctzll(sb);
            sb &= sb - 1;
            const int xe = sb ? __builtin_ctzll(sb) - 1 : 63;
            const int fg = (int)((m >> xs) & 1);
            const int outer = !fg && (x0 + xs == 0 || x0 + xe >= w - 1 || gy == 0 || gy >= h - 1);
            rx0[id] = (uint8_t)xs;
            rx1[id] = (uint8_t)xe;
            rf[id] = (uint8_t)(fg | (outer << 1));
            par[id] = id;
            amin[id] = fg ? xs : outer;
            amax[id] = xe;
            ay[id] = ln;
            id++;
        }
    }
    FM_STAMP(4);
    // Adjacent-row run pairs to union, from the bit masks (no LDS walk): a run B of
    // row ln+1 touches a contiguous range of same-colour runs of row ln -- window
    // [b0-1, b1+1] for foreground (8-connected), [b0, b1] for background (4-connected).
    const uint64_t m2 = lane_down1_64(m), s2 = lane_down1_64(starts);
    const int base2 = lane_down1(base);
    int npl = 0;
    // count pass
    if (ln < 63) {
        uint64_t sb = s2;
        while (sb) {
            const int b0 = __builtin_ctzll(sb);
            sb &= sb - 1;
            const int b1 = sb ? __builtin_ctzll(sb) - 1 : 63;
            const bool fgB = (m2 >> b0) & 1;
            const int w0 = fgB ? max(b0 - 1, 0) : b0, w1 = fgB ? min(b1 + 1, 63) : b1;
            const uint64_t win = (w1 == 63 ? ~0ull : ((2ull << w1) - 1)) & ~((1ull << w0) - 1);
            const uint64_t hits = (fgB ? m : ~m) & win;
            if (hits) npl += ((run_at(base, starts, 63 - __builtin_clzll(hits)) - run_at(base, starts, __builtin_ctzll(hits))) >> 1) + 1;
        }
    }
    const int pin = wave_incl_sum(npl);
    const int np = lane_at(pin, 63);
    if (np > 2 * CAP) return TCCL_RUNS;
    const int pbase = pin - npl;
    if (ln < 63) {  // write pass
        uint64_t sb = s2;
        int id2 = base2;
        int k = pbase;
        while (sb) {
            const int b0 = __builtin_ctzll(sb);
            sb &= sb - 1;
            const int b1 = sb ? __builtin_ctzll(sb) - 1 : 63;
            const bool fgB = (m2 >> b0) & 1;
            const int w0 = fgB ? max(b0 - 1, 0) : b0, w1 = fgB ? min(b1 + 1, 63) : b1;
            const uint64_t win = (w1 == 63 ? ~0ull : ((2ull << w1) - 1)) & ~((1ull << w0) - 1);
            const uint64_t hits = (fgB ? m : ~m) & win;
            if (hits) {
                const int ia = run_at(base, starts, __builtin_ctzll(hits));
                const int ib = run_at(base, starts, 63 - __builtin_clzll(hits));
                for (int r = ia; r <= ib; r += 2) sc.pairs[k++] = (uint32_t)r | ((uint32_t)id2 << 16);
            }
            id2++;
        }
    }
    lds_fence();
    FM_STAMP(5);
    // Shiloach-Vishkin style rounds: hook the larger of the two parents under the
    // smaller (atomicMin, so parents only decrease), then shortcut par[i] = par[par[i]];
    // at the fixed point every component is a star rooted at its smallest run,
    // i.e. its raster-first run.
    for (int round = 0; round < 64; round++) {
        bool ch = false;
        for (int p = ln; p < np; p += 64) {
            const uint32_t pr = sc.pairs[p];
            const int ra = lload(&par[pr & 0xFFFF]), rb2 = lload(&par[pr >> 16]);
            if (ra != rb2) {
                atomicMin(&par[max(ra, rb2)], min(ra, rb2));
                ch = true;
            }
        }
        lds_fence();
        for (int i = ln; i < total; i += 64) {
            const int pi = lload(&par[i]);
            const int ppi = lload(&par[pi]);
            if (ppi != pi) {
                atomicMin(&par[i], ppi);
                ch = true;
            }
        }
        lds_fence();
        if (__ballot(ch) == 0) break;
    }
    FM_STAMP(6);
    // fold into roots (par[] is flat now); this row's roots (raster-first runs of their components)
    // kept in a bit mask, so the ordinal and node loops below visit the roots only and re-read nothing
    uint64_t rmask = 0;
    for (int i = base; i < base + nr; i++) {
        const int rt = (par[i]);
        if (rt != i) {
            if (rf[i] & 1) {
                atomicMin(&amin[rt], (int)rx0[i]);
                atomicMax(&amax[rt], (int)rx1[i]);
                atomicMax(&ay[rt], ln);
            } else if (rf[i] & 2) {
                atomicOr(&amin[rt], 1);
            }
        } else {
            rmask |= 1ull << (i - base);
        }
    }
    lds_fence();
    FM_STAMP(7);
    // ordinals of the roots in raster order
    const int myr = __popcll(rmask);
    const int rin = wave_incl_sum(myr);
    const int nroots = lane_at(rin, 63);
    const int nb = take_nodes(a, f, nroots, ln);
    if (nb < 0) return TCCL_NODES;
    if (ln == 63) {
        TR->nroots = nroots;
        TR->nbase = nb;
    }
    {
        int kk = rin - myr;
        for (uint64_t q = rmask; q; q &= q - 1) ord[base + __builtin_ctzll(q)] = (uint16_t)kk++;
    }
    lds_fence();
    if (FM_OOB(a, (long long)nb + nroots <= (long long)a.nnodes, 3)) return TCCL_NODES;
    NodeRec* NR = a.nodes + nb;
    int kr = rin - myr;  // ordinal of the row's next root
    for (uint64_t q = rmask; q; q &= q - 1, kr++) {
        const int i = base + __builtin_ctzll(q);
        const int fg = rf[i] & 1;
        NodeRec nrec;
        nrec.parent = nb + kr;
        nrec.key = 0;
        nrec.minx = nrec.maxx = nrec.maxy = nrec.pad = 0;
        if (fg) {
            const int xs = rx0[i];
            uint32_t ref;
            if (x0 + xs == 0) ref = REF_OUTER;
            else if (xs == 0) ref = REF_EDGE | (uint32_t)ln;
            else ref = (uint32_t)ord[(par[i - 1])];  // the background run left of this run
            nrec.key = ((uint64_t)(uint32_t)(gy * w + x0 + xs) << 32) | ref;
            nrec.flags = 1u;
            nrec.minx = x0 + amin[i];
            nrec.maxx = x0 + amax[i];
            nrec.maxy = y0 + ay[i];
        } else {
            nrec.flags = amin[i] ? 2u : 0u;
        }
        NR[kr] = nrec;
    }
    const uint64_t mask_c = (2ull << ln) - 1;
    const uint64_t s0 = lane_at64(starts, 0), s63 = lane_at64(starts, 63);
    const uint64_t m0 = lane_at64(m, 0), m63 = lane_at64(m, 63);
    const int id0 = rb[0] + __popcll(s0 & mask_c) - 1;
    const int id63 = rb[63] + __popcll(s63 & mask_c) - 1;
    TR->edges[ln] = (uint16_t)(ord[(par[base])] | ((rf[base] & 1) << 15));
    TR->edges[64 + ln] = (uint16_t)(ord[(par[base + nr - 1])] | ((rf[base + nr - 1] & 1) << 15));
    TR->edges[128 + ln] = (uint16_t)(ord[(par[id0])] | (((m0 >> ln) & 1) << 15));
    TR->edges[192 + ln] = (uint16_t)(ord[(par[id63])] | (((m63 >> ln) & 1) << 15));
    FM_STAMP(8);
    return TCCL_OK;
}

// candidate: the tile's dilated mask can be non-empty.  With threshold bits
// (dilate) that is: its own bits, or a neighbour's bits within 2 px of the
// shared edge or corner; with already dilated bits, its own bits.
// the tile's FLAG_* bits: one word per tile (k_fused), or one per wave of the pixel
// kernel's workgroup (k_pix writes them with plain stores, no atomics), ORed here
__device__ __forceinline__ uint32_t tile_flags(const FusedArgs& a, size_t f, int ti) {
    if (a.tflag_waves == 1) return a.tflag[f * a.ntiles + ti];
    const uint4* q = reinterpret_cast<const uint4*>(a.tflag + (f * a.ntiles + ti) * 8);
    const uint4 x = q[0], y = q[1];
    return x.x | x.y | x.z | x.w | y.x | y.y | y.z | y.w;
}

// the candidate test (above) over the frame's flag words staged in LDS (fl[t] = tile_flags of tile t)
__device__ __forceinline__ bool is_candidate_lds(const int* fl, const FusedArgs& a, int ti, bool dilate) {
    if (fl[ti]) return true;
    if (!dilate) return false;
    const int ntx = a.ntx, tx = ti % ntx, ty = ti / ntx;
    const bool l = tx > 0, r = tx + 1 < ntx, u = ty > 0, d = ty + 1 < a.nty;
    uint32_t m = 0;
    if (l) m |= (uint32_t)fl[ti - 1] & FLAG_R;
    if (r) m |= (uint32_t)fl[ti + 1] & FLAG_L;
    if (u) m |= (uint32_t)fl[ti - ntx] & FLAG_B;
    if (d) m |= (uint32_t)fl[ti + ntx] & FLAG_T;
    if (u && l) m |= (uint32_t)fl[ti - ntx - 1] & FLAG_BR;
    if (u && r) m |= (uint32_t)fl[ti - ntx + 1] & FLAG_BL;
    if (d && l) m |= (uint32_t)fl[ti + ntx - 1] & FLAG_TR;
    if (d && r) m |= (uint32_t)fl[ti + ntx + 1] & FLAG_TL;
    return m != 0;
}

// one workgroup per frame: candidate list, empty-tile regions (4-connected: two
// empty tiles share a whole background edge), one node per region
// (uf is sized to the frame's tiles at launch: a fixed MAX_REGION_TILES array was 32 KB of LDS per
// workgroup, which the contour kernels resident beside the pixel kernel often did not leave free,
// so a batch's k_regions waited for the pixel kernel to end: 269 µs instead of 10)
// RG threads of one workgroup; SLOT: frame 0 also zeroes the slot-wide counters (node pool, heavy list)
template <bool DILATE, int RG, bool SLOT>
__device__ __forceinline__ void regions_frame(const FusedArgs& a, int f, int* uf, int& s_nc, int& s_nr) {
    const int nt = a.ntiles, ntx = a.ntx, nty = a.nty;
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_nc = s_nr = 0;
        // this batch's counters (the slot's previous batch was read back before reuse)
        a.count[f] = 0;
        a.count[(size_t)a.T * a.S + f] = 0;
        a.count[2 * (size_t)a.T * a.S + 2 + f] = 0;
        if (SLOT && f == 0) {  // node pool and heavy scratch of the slot (read only by later kernels)
            a.count[2 * (size_t)a.T * a.S] = 0;
            a.count[2 * (size_t)a.T * a.S + 1] = 0;
        }
    }
    // each tile's flag words read once into LDS (uf doubles as the staging array), then the
    // candidate test over LDS: is_candidate from global memory read every tile's words up to 9 times
    for (int t = tid; t < nt; t += RG) uf[t] = (int)tile_flags(a, f, t);
    __syncthreads();
    uint32_t cm = 0;  // bit i: tile tid + i * RG (nt <= MAX_REGION_TILES = 16 * RG)
    for (int t = tid, i = 0; t < nt; t += RG, i++)
        if (is_candidate_lds(uf, a, t, DILATE)) cm |= 1u << i;
    __syncthreads();
    for (int t = tid, i = 0; t < nt; t += RG, i++) {
        const bool c = (cm >> i) & 1;
        a.candf[(size_t)f * nt + t] = c ? 1 : 0;
        uf[t] = c ? -1 : t;
        if (c) a.clist[(size_t)f * nt + atomicAdd(&s_nc, 1)] = t;
    }
    __syncthreads();
    for (int t = tid; t < nt; t += RG) {
        if (uf[t] < 0) continue;
        const int tx = t % ntx;
        if (tx + 1 < ntx && uf[t + 1] >= 0) lunion(uf, t, t + 1);
        if (t + ntx < nt && uf[t + ntx] >= 0) lunion(uf, t, t + ntx);
    }
    __syncthreads();
    for (int t = tid; t < nt; t += RG)
        if (uf[t] >= 0) uf[t] = lfind(uf, t);
    __syncthreads();
    // region representative = its smallest tile; "outer" if any tile is on the grid border.
    // The representative's node is (re)initialised first: the slot's nodes still hold an
    // earlier batch's records, where this tile may have been a candidate
    for (int t = tid; t < nt; t += RG) {
        const int r = uf[t];
        if (r < 0) continue;
        a.regrep[(size_t)f * nt + t] = r;
        if (t == r) {
            NodeRec* rep = a.nodes + (size_t)f * nt + r;
            rep->parent = (int)((size_t)f * nt + r);
            rep->flags = 0u;
            a.rlist[(size_t)f * nt + atomicAdd(&s_nr, 1)] = r;
        }
    }
    __syncthreads();
    for (int t = tid; t < nt; t += RG) {
        const int r = uf[t];
        if (r < 0) continue;
        const int tx = t % ntx, ty = t / ntx;
        if (tx == 0 || ty == 0 || tx == ntx - 1 || ty == nty - 1)
            atomicOr(&a.nodes[(size_t)f * nt + r].flags, 2u);
    }
    __syncthreads();
    if (tid == 0) {
        a.ncr[2 * f] = s_nc;
        a.ncr[2 * f + 1] = s_nr;
    }
}

template <bool DILATE>
__global__ __launch_bounds__(RG) void k_regions(FusedArgs a) {
    extern __shared__ int uf[];  // [a.ntiles]
    __shared__ int s_nc, s_nr;
#ifdef FM_DEV_SWITCHES
    kstamp_begin_grid(a.kstamp);
    kstamp_end_wg(a.kstamp);  // (the window of interest is the chain's start)
#endif
    regions_frame<DILATE, RG, true>(a, blockIdx.x, uf, s_nc, s_nr);
}


// grid (GW, F); each wave labels candidates of the frame's list with a stride, in LDS
// (LIGHT runs); a tile with more runs (a dense texture of small blobs) goes to the
// heavy list
// k_tile_ccl is compiled for 6 waves per SIMD: 80 VGPRs (was 96, no spills), so two of its workgroups
// fit beside two k_pix5 workgroups (4 x 88 VGPRs per SIMD): +1.2 %, 4 rounds.  Its scratch is dynamic
// LDS, so the compiler takes its occupancy from that, not from a static 30 KB (see k_tile_heavy).
// dilation (fm.py:266) of candidate ti into its dbits, then the light labelling (tile_ccl)
template <bool DILATE>
__device__ __forceinline__ int label_tile(const FusedArgs& a, size_t f, int ti, int ln, const Scratch& sc) {
    FM_STAMP(1);
    uint64_t m;
    if (DILATE && !(a.dbg_skip & 128)) {
        m = dilate_tile(a, f, ti, ln, nullptr);
        a.dbits[(f * a.ntiles + ti) * 64 + ln] = m;
    } else {
        m = a.dbits[(f * a.ntiles + ti) * 64 + ln];
    }
    FM_STAMP(2);
    return tile_ccl<LIGHT>(a, f, ti, ln, m, sc);
}

constexpr size_t TC_WAVE_LDS = ((size_t)(6 * LIGHT + 66) * 4 + 2 * LIGHT + 3 * LIGHT + 15) / 16 * 16;
constexpr size_t TC_LDS = CW * TC_WAVE_LDS;
// wave wv's light scratch: par, amin, amax, ay, pairs (u32), rb | ord (u16) | rx0, rx1, rf (u8)
__device__ __forceinline__ Scratch light_scratch(int* lds, int wv) {
    int* wb = lds + (size_t)wv * (TC_WAVE_LDS / 4);
    uint16_t* word = reinterpret_cast<uint16_t*>(wb + 6 * LIGHT + 66);
    uint8_t* wbyte = reinterpret_cast<uint8_t*>(word + LIGHT);
    return Scratch{wb, wb + LIGHT, wb + 2 * LIGHT, wb + 3 * LIGHT, wbyte, wbyte + LIGHT, wbyte + 2 * LIGHT,
                   wb + 6 * LIGHT, word, reinterpret_cast<uint32_t*>(wb + 4 * LIGHT)};
}
template <bool DILATE>
__global__ __launch_bounds__(64 * CW) __attribute__((amdgpu_waves_per_eu(6))) void k_tile_ccl(FusedArgs a) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    extern __shared__ __attribute__((aligned(16))) int tc_lds[];
    const Scratch sc = light_scratch(tc_lds, wv);
    const size_t f = blockIdx.y;
    const size_t F = (size_t)a.T * a.S;
    const int nc = a.ncr[2 * f];
    if (FM_OOB(a, nc >= 0 && nc <= a.ntiles, 1)) return;
    for (int k = blockIdx.x * CW + wv; k < nc; k += gridDim.x * CW) {
        const int ti = a.clist[f * a.ntiles + k];
        if (FM_OOB(a, ti >= 0 && ti < a.ntiles, 1)) continue;
        if (a.dbg_skip & 64) continue;  // profiling ablation (results invalid)
        const int r = label_tile<DILATE>(a, f, ti, ln, sc);
        if (ln == 0) {
            if (r == TCCL_RUNS) {
                const int hi = atomicAdd(&a.count[2 * F + 1], 1);
                if (!FM_OOB(a, hi < (int)(F * a.ntiles), 2)) a.heavy[hi] = (int)(f * a.ntiles + ti);
            }
            else if (r != TCCL_OK) a.count[F + f] = 1;
        }
    }
}

// heavy pass: NHW persistent waves drain the heavy list (kTileMaxRuns runs per tile), all scratch
// in 46 KB of LDS: beside k_pix5's two ~30 KB workgroups a CU has room for it (measured 3.5 %
// faster end to end than keeping the per-run arrays in global memory, which k_pix's ~52 KB
// workgroups needed)
constexpr int NHW = kHeavyWaves;
// The scratch is dynamic LDS: with a static 46 KB the compiler derives an occupancy of one wave per
// SIMD from the LDS alone and then sizes the kernel's VGPR allocation for that occupancy (264
// registers for 67 used), which no CU holding two k_pix5 workgroups (4 waves x 88 VGPRs per SIMD)
// can fit: every batch's heavy tiles then waited for the pixel kernel to end (trace r03h: 300-370 us
// beside it, 26 us alone).  Sized at launch, the allocation is what the code uses.
constexpr int HV_INT = 4 * MAXR + 2 * MAXR + 68;   // par, amin, amax, ay | pairs (u32) | rb
constexpr size_t HEAVY_LDS = (size_t)HV_INT * 4 + 3 * MAXR + 2 * MAXR;  // + rx0, rx1, rf (u8), ord (u16)
__device__ __forceinline__ Scratch heavy_scratch(int* lds) {
    int* par = lds;
    int* amin = par + MAXR;
    int* amax = amin + MAXR;
    int* ay = amax + MAXR;
    uint32_t* pairs = reinterpret_cast<uint32_t*>(ay + MAXR);
    int* rb = reinterpret_cast<int*>(pairs + 2 * MAXR);
    uint16_t* ord = reinterpret_cast<uint16_t*>(rb + 68);
    uint8_t* rx0 = reinterpret_cast<uint8_t*>(ord + MAXR);
    uint8_t* rx1 = rx0 + MAXR;
    uint8_t* rf = rx1 + MAXR;
    return Scratch{par, amin, amax, ay, rx0, rx1, rf, rb, ord, pairs};
}
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1))) void k_tile_heavy(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) int hv_lds[];
    const size_t F = (size_t)a.T * a.S;
    const int n = a.count[2 * F + 1];
    const int ln = threadIdx.x;
    if (FM_OOB(a, n <= (int)(F * a.ntiles), 2)) return;
    const Scratch sc = heavy_scratch(hv_lds);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int item = a.heavy[i];
        if (FM_OOB(a, item >= 0 && item < (int)(F * a.ntiles), 4)) continue;
        const size_t f = item / a.ntiles;
        const int ti = (int)(item - (long long)f * a.ntiles);
        const int r = tile_ccl<MAXR>(a, f, ti, ln, a.dbits[(f * a.ntiles + ti) * 64 + ln], sc);
        if (r != TCCL_OK && ln == 0) a.count[F + f] = 1;
    }
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ int efg(uint16_t e) { return e >> 15; }
// node of the component with edge label e of candidate tile `tile`
__device__ __forceinline__ int enode(const TileRec* TR, int tile, uint16_t e) { return TR[tile].nbase + (e & 0x7FFF); }

// Union-find of the edge merge: over the global NodeRec parents.  (A per-frame union-find in LDS,
// k_merge + k_fold + k_emit + k_counts of one frame in one workgroup -- k_resolve, round 4 -- measured
// 401.6 vs 415.7 k frames/s: its long-lived per-frame workgroups held CU slots the pixel kernel needed.)
struct GlobalUF {
    NodeRec* N;
    __device__ void uni(int x, int y) const { gunion(N, x, y); }
    __device__ bool outer(int n) const { return (N[n].flags & 2) != 0; }
    __device__ void mark_outer(int n) const { atomicOr(&N[n].flags, 2u); }
};

// Background component `nd` of a candidate touches empty region `rep`.  An outer
// region only contributes its outer-ness, so the node is marked directly (no union:
// every candidate around a moving object borders the big outer background, and
// unions into that one root serialise on its atomics); an enclosed region is unioned.
// (rnode = f*ntiles + a representative tile < F*ntiles: regrep is written for every
// empty tile by k_regions of this batch)
template <class UF>
__device__ __forceinline__ void touch_region(const UF& U, int nd, int rnode) {
    if (U.outer(rnode)) U.mark_outer(nd);
    else U.uni(nd, rnode);
}

// candidate tile t of frame f, lane = edge position: unions along its right / bottom edges with
// candidate neighbours, its corner diagonals, and every edge against empty regions
template <class UF>
__device__ __forceinline__ void merge_tile(const FusedArgs& a, size_t f, int t, int ln, const UF& U) {
    const int ntx = a.ntx, nt = a.ntiles;
    const uint8_t* cf = a.candf + f * nt;
    const int32_t* rr = a.regrep + f * nt;
    const TileRec* TR = a.tiles + f * nt;
    const int rb0 = (int)(f * nt);  // region node ids of this frame: rb0 + representative tile
    const int tx = t % ntx, ty = t / ntx;
    const bool hasR = tx + 1 < ntx, hasD = ty + 1 < a.nty;
    // right edge
    if (hasR) {
        const uint16_t A = TR[t].edges[64 + ln];
        const int Ap = lane_up1((int)A);
        if (cf[t + 1]) {
            const uint16_t B = TR[t + 1].edges[ln];
            const int Bp = lane_up1((int)B);
            if (efg(A) == efg(B) && !(ln > 0 && Ap == A && Bp == B)) U.uni(enode(TR, t, A), enode(TR, t + 1, B));
            if (efg(A)) {
                if (ln > 0) {
                    const uint16_t Bu = TR[t + 1].edges[ln - 1];
                    if (efg(Bu) && Bu != B) U.uni(enode(TR, t, A), enode(TR, t + 1, Bu));
                }
                if (ln < 63) {
                    const uint16_t Bd = TR[t + 1].edges[ln + 1];
                    if (efg(Bd) && Bd != B) U.uni(enode(TR, t, A), enode(TR, t + 1, Bd));
                }
            }
        } else if (!efg(A) && !(ln > 0 && Ap == A)) {
            touch_region(U, enode(TR, t, A), rb0 + rr[t + 1]);
        }
    }
    // bottom edge
    if (hasD) {
        const int n = t + ntx;
        const uint16_t A = TR[t].edges[192 + ln];
        const int Ap = lane_up1((int)A);
        if (cf[n]) {
            const uint16_t B = TR[n].edges[128 + ln];
            const int Bp = lane_up1((int)B);
            if (efg(A) == efg(B) && !(ln > 0 && Ap == A && Bp == B)) U.uni(enode(TR, t, A), enode(TR, n, B));
            if (efg(A)) {
                if (ln > 0) {
                    const uint16_t Bl = TR[n].edges[128 + ln - 1];
                    if (efg(Bl) && Bl != B) U.uni(enode(TR, t, A), enode(TR, n, Bl));
                }
                if (ln < 63) {
                    const uint16_t Br = TR[n].edges[128 + ln + 1];
                    if (efg(Br) && Br != B) U.uni(enode(TR, t, A), enode(TR, n, Br));
                }
            }
        } else if (!efg(A) && !(ln > 0 && Ap == A)) {
            touch_region(U, enode(TR, t, A), rb0 + rr[n]);
        }
        // corner diagonals (foreground only: both tiles candidates)
        if (ln == 0 && hasR && cf[n + 1]) {  // (63,63) <-> (0,0) of the down-right tile
            const uint16_t P = TR[t].edges[192 + 63], Q = TR[n + 1].edges[128];
            if (efg(P) && efg(Q)) U.uni(enode(TR, t, P), enode(TR, n + 1, Q));
        }
        if (ln == 0 && tx > 0 && cf[n - 1]) {  // (0,63) <-> (63,0) of the down-left tile
            const uint16_t P = TR[t].edges[192], Q = TR[n - 1].edges[128 + 63];
            if (efg(P) && efg(Q)) U.uni(enode(TR, t, P), enode(TR, n - 1, Q));
        }
    }
    // left / top edges against empty regions (candidate pairs are done by the neighbour)
    if (tx > 0 && !cf[t - 1]) {
        const uint16_t A = TR[t].edges[ln];
        const int Ap = lane_up1((int)A);
        if (!efg(A) && !(ln > 0 && Ap == A)) touch_region(U, enode(TR, t, A), rb0 + rr[t - 1]);
    }
    if (ty > 0 && !cf[t - ntx]) {
        const uint16_t A = TR[t].edges[128 + ln];
        const int Ap = lane_up1((int)A);
        if (!efg(A) && !(ln > 0 && Ap == A)) touch_region(U, enode(TR, t, A), rb0 + rr[t - ntx]);
    }
}

// candidates wave, wave + nwaves, ... of frame f's list (nc of them)
__device__ __forceinline__ void merge_frame(const FusedArgs& a, size_t f, int nc, int wave, int nwaves, int ln) {
    const int nt = a.ntiles;
    const TileRec* TR = a.tiles + f * nt;
    (void)TR;  // (read by the bounds check of the checked build)
    const GlobalUF U{a.nodes};
    for (int k = wave; k < nc; k += nwaves) {
        const int t = a.clist[f * nt + k];
        if (FM_OOB(a, t >= 0 && t < nt && TR[t].nbase >= 0 && TR[t].nbase + TR[t].nroots <= a.nnodes, 5)) continue;
        merge_tile(a, f, t, ln, U);
    }
}

// one wave per candidate, lane = edge position
__global__ __launch_bounds__(64 * CW) void k_merge(FusedArgs a) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const size_t f = blockIdx.y;
    const size_t F = (size_t)a.T * a.S;
    if (a.count[F + f]) return;
    merge_frame(a, f, a.ncr[2 * f], blockIdx.x * CW + wv, gridDim.x * CW, ln);
}

__device__ __forceinline__ void fold_node(NodeRec* N, int n) {
    const int rt = gfind(N, n);
    if (rt == n) return;
    N[n].parent = rt;
    const uint32_t fl = N[n].flags;
    if (fl & 1) {
        atomicMin((unsigned long long*)&N[rt].key, (unsigned long long)N[n].key);
        atomicMin(&N[rt].minx, N[n].minx);
        atomicMax(&N[rt].maxx, N[n].maxx);
        atomicMax(&N[rt].maxy, N[n].maxy);
    } else if (fl & 2) {
        atomicOr(&N[rt].flags, 2u);
    }
}

// one wave per candidate tile (lanes = its components) or per empty-tile region: path
// compression with outer flags, bboxes and raster-first pixels folded into the roots
__device__ __forceinline__ void fold_frame(const FusedArgs& a, size_t f, int nc, int nr, int wave, int nwaves, int ln) {
    NodeRec* N = a.nodes;
    const TileRec* TRf = a.tiles + f * a.ntiles;
    for (int k = wave; k < nc + nr; k += nwaves) {
        if (k < nc) {
            const int t = a.clist[f * a.ntiles + k];
            if (FM_OOB(a, t >= 0 && t < a.ntiles, 1)) continue;
            const int k1 = TRf[t].nroots, nb = TRf[t].nbase;
            if (FM_OOB(a, nb >= 0 && (long long)nb + k1 <= a.nnodes, 5)) continue;
            for (int i = ln; i < k1; i += 64) fold_node(N, nb + i);
        } else if (ln == 0) {
            const int r = a.rlist[f * a.ntiles + (k - nc)];
            if (FM_OOB(a, r >= 0 && r < a.ntiles, 6)) continue;
            fold_node(N, (int)(f * a.ntiles) + r);
        }
    }
}

__global__ __launch_bounds__(64 * CW) void k_fold(FusedArgs a) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const size_t f = blockIdx.y;
    const size_t F = (size_t)a.T * a.S;
    if (a.count[F + f]) return;  // relabelled by the host's pixel-level fallback
    fold_frame(a, f, a.ncr[2 * f], a.ncr[2 * f + 1], blockIdx.x * CW + wv, gridDim.x * CW, ln);
}

// one wave per candidate tile, lanes = its components: the external test at every
// foreground root and its contour record (after k_fold: every node points at its root).
// Records beyond cap are counted, not written (fm_wait re-emits such a frame whole with
// k_emit_all, so len(frame.contours) and the records kept never depend on the cap).
__device__ __forceinline__ void emit_frame(const FusedArgs& a, size_t f, int wave, int nwaves, int ln, int32_t* recs,
                                           int32_t* cnt, int cap) {
    const NodeRec* N = a.nodes;
    const TileRec* TRf = a.tiles + f * a.ntiles;
    const uint8_t* cf = a.candf + f * a.ntiles;
    const int32_t* rr = a.regrep + f * a.ntiles;
    const int rb0 = (int)(f * a.ntiles);
    const int nc = a.ncr[2 * f];
    for (int k = wave; k < nc; k += nwaves) {
        const int t = a.clist[f * a.ntiles + k];
        if (FM_OOB(a, t >= 0 && t < a.ntiles, 1)) continue;
        const int k1 = TRf[t].nroots, nbt = TRf[t].nbase;
        for (int i = ln; i < k1; i += 64) {
            const int n = nbt + i;
            if (N[n].parent != n || !(N[n].flags & 1)) continue;
            const uint64_t key = N[n].key;
            const uint32_t first = (uint32_t)(key >> 32), ref = (uint32_t)key;
            const int fx = (int)(first % (uint32_t)a.w), fy = (int)(first / (uint32_t)a.w);
            bool ext;
            if (ref & REF_OUTER) {
                ext = true;
            } else {
                const int tf = (fy / TS) * a.ntx + fx / TS;  // tile of the raster-first pixel (a candidate)
                if (FM_OOB(a, tf >= 0 && tf < a.ntiles && (!(ref & REF_EDGE) || tf % a.ntx > 0), 7)) continue;
                int bn;
                if (ref & REF_EDGE) {
                    const int lt = tf - 1;
                    bn = cf[lt] ? enode(TRf, lt, TRf[lt].edges[64 + (ref & 63)]) : rb0 + rr[lt];
                } else {
                    bn = TRf[tf].nbase + (int)ref;
                }
                if (FM_OOB(a, bn >= 0 && bn < a.nnodes && N[bn].parent >= 0 && N[bn].parent < a.nnodes, 5)) continue;
                ext = (N[N[bn].parent].flags & 2) != 0;
            }
            if (!ext) continue;
            const int id = atomicAdd(cnt, 1);
            if (id < cap) {
                int32_t* rec = recs + (size_t)id * 5;
                rec[0] = (int32_t)first;
                rec[1] = N[n].minx;
                rec[2] = fy;
                rec[3] = N[n].maxx;
                rec[4] = N[n].maxy;
            }
        }
    }
}

__global__ __launch_bounds__(64 * CW) void k_emit(FusedArgs a) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const size_t f = blockIdx.y;
    const size_t F = (size_t)a.T * a.S;
    if (a.count[F + f]) return;
    emit_frame(a, f, blockIdx.x * CW + wv, gridDim.x * CW, ln, a.rec + f * a.cap * 5, &a.count[f], a.cap);
}

// one frame of a finished batch, every record (cap = its known count)
__global__ __launch_bounds__(64 * CW) void k_emit_all(FusedArgs a, int f, int32_t* recs, int32_t* cnt, int cap) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    emit_frame(a, (size_t)f, blockIdx.x * CW + wv, gridDim.x * CW, ln, recs, cnt, cap);
}


// one workgroup per frame: counts and overflow flags straight into mapped host memory
// (no copy after the kernel); the k_fused path's tile flags cleared for the slot's next
// batch (k_pix rewrites its per-wave flag words every frame)
constexpr int FT = 256;
__global__ __launch_bounds__(FT) void k_counts(FusedArgs a) {
    const size_t f = blockIdx.x;
    const size_t F = (size_t)a.T * a.S;
#ifdef FM_DEV_SWITCHES
    kstamp_begin_grid(a.kstamp);
#endif
    if (a.tflag_waves == 1)
        for (int t = threadIdx.x; t < a.ntiles; t += FT) a.tflag[f * a.ntiles + t] = 0;
    if (threadIdx.x == 0) {
        const bool ovf = a.count[F + f] != 0;
        a.h_count[f] = ovf ? 0 : a.count[f];
        a.h_overflow[f] = ovf ? 1 : 0;
        if (f == 0) {
            a.h_stats[0] = a.count[2 * F];
            a.h_stats[1] = a.count[2 * F + 1];
        }
    }
#ifdef FM_DEV_SWITCHES
    kstamp_end_wg(a.kstamp);
#endif
}

// one thread per 8 mask bytes of one frame; non-candidate tiles are empty
__global__ __launch_bounds__(256) void k_expand_bits(const uint64_t* __restrict__ dbits, const uint8_t* __restrict__ candf,
                                                     uint8_t* __restrict__ out, int h, int w, int ntx) {
    const int x8 = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    const int xs = 8 * x8;
    if (xs >= w) return;
    const int tx = xs >> 6, ty = y >> 6;
    const int ti = ty * ntx + tx;
    const uint64_t row = candf[ti] ? dbits[(size_t)ti * 64 + (y & 63)] : 0ull;
    const uint32_t b = (uint32_t)(row >> (xs & 63)) & 0xFFu;
    uint8_t* dst = out + (size_t)y * w + xs;
    for (int i = 0; i < 8 && xs + i < w; i++) dst[i] = ((b >> i) & 1) ? 255 : 0;
}

// ---------------------------------------------------------------------------
// cv2.contourArea of an external contour (fm.py:679), for the area filter of fm.py:684.
// One thread per contour follows its outer border from the start pixel with the rule of
// OpenCV's icvFetchContour (restated in oracle/fm_oracle.c fetch_contour; the path depends
// only on which pixels are non-zero) and sums the shoelace over the CHAIN_APPROX_SIMPLE
// points (the direction changes).  Out-of-image pixels are zero (the 1-px pad).
struct AreaMask {
    const uint64_t* dbits;
    const uint8_t* candf;
    const uint8_t* mask;
    int ntiles, ntx, h, w;
    __device__ __forceinline__ bool px(int f, int x, int y) const {
        if ((unsigned)x >= (unsigned)w || (unsigned)y >= (unsigned)h) return false;
        if (mask) return mask[((size_t)f * h + y) * w + x] != 0;
        const size_t t = (size_t)f * ntiles + (y >> 6) * ntx + (x >> 6);
        return candf[t] && ((dbits[t * 64 + (y & 63)] >> (x & 63)) & 1ull);
    }
};

__global__ __launch_bounds__(256) void k_contour_area(AreaMask m, const int32_t* __restrict__ jobs, int n,
                                                      int32_t* __restrict__ area2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    constexpr int dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
    constexpr int dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
    const int f = jobs[3 * i], x0 = jobs[3 * i + 1], y0 = jobs[3 * i + 2];
    int s = 4, x1 = x0, y1 = y0;
    do {  // first non-zero neighbour clockwise from the left (outer border: s_end = 4)
        s = (s - 1) & 7;
        x1 = x0 + dx[s];
        y1 = y0 + dy[s];
    } while (!m.px(f, x1, y1) && s != 4);
    if (s == 4) {  // an isolated pixel: one point, area 0
        area2[i] = 0;
        return;
    }
    int x3 = x0, y3 = y0, prev_s = s ^ 4;
    long long a = 0;
    int fx = 0, fy = 0, lx = 0, ly = 0, np = 0;
    const long long cap = 4ll * ((long long)m.w + 2) * ((long long)m.h + 2) + 16;
    for (long long it = 0;; it++) {
        if (it > cap) {  // not a border start of this mask: report, never loop forever
            area2[i] = -1;
            return;
        }
        int x4 = x3, y4 = y3;
        while (s < 15) {
            ++s;
            x4 = x3 + dx[s & 7];
            y4 = y3 + dy[s & 7];
            if (m.px(f, x4, y4)) break;
        }
        s &= 7;
        if (s != prev_s) {  // CHAIN_APPROX_SIMPLE keeps the point where the direction changes
            if (np == 0) {
                fx = x3;
                fy = y3;
            } else {
                a += (long long)lx * y3 - (long long)ly * x3;
            }
            lx = x3;
            ly = y3;
            np++;
            prev_s = s;
        }
        if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
        x3 = x4;
        y3 = y4;
        s = (s + 4) & 7;
    }
    if (np > 0) a += (long long)lx * fy - (long long)ly * fx;
    area2[i] = (int32_t)(a < 0 ? -a : a);
}

// ---------------------------------------------------------------------------
// Small work images (round 5): the whole contour pass of one frame in one workgroup.  Mode D's 100 x 56
// image is two tiles; the seven-kernel chain above spent its time in launch and cross-queue latency
// (each batch's chain ran 0.5-1.4 ms after its pixel stage, so with six slots the host waited for
// chains and the input stream's resizes went idle).  Here the same steps run back to back in one
// launch, separated by workgroup barriers: regions, dilation + light labelling (a wave per candidate),
// heavy tiles (wave 0, the workgroup's whole LDS), edge merge, fold, external test + records, counts.
// Every union-find node a frame touches is its own (its region nodes and its quota; only the shared
// overflow pool is slot-wide), so no step waits for other frames.  Global writes of one step are read
// by other waves of the same workgroup in the next: workgroup scope, which a barrier gives on one CU (its
// L1 is shared by the workgroup).  (Agent-scope fences around each barrier -- an L2 write-back and
// invalidate each -- made the kernel 500 us per 256 frames and the resize beside it 2.4x slower.)
constexpr int FW = 4;                     // waves per frame workgroup
constexpr size_t FR_SCRATCH = FW * TC_WAVE_LDS > HEAVY_LDS ? FW * TC_WAVE_LDS : HEAVY_LDS;
__device__ __forceinline__ void step_barrier() { __syncthreads(); }
template <bool DILATE>
__global__ __launch_bounds__(64 * FW) void k_frame_contours(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) int fr_lds[];  // FR_SCRATCH, then uf and hl: a.ntiles ints each
    int* uf = fr_lds + FR_SCRATCH / 4;
    int* hl = uf + a.ntiles;
    __shared__ int s_nc, s_nr, s_nh, s_ovf;
    const int tid = threadIdx.x, wv = tid >> 6, ln = tid & 63;
    const size_t f = blockIdx.x;
    const size_t F = (size_t)a.T * a.S;
#ifdef FM_DEV_SWITCHES
    kstamp_begin_grid(a.kstamp);
#endif
    if (tid == 0) s_nh = s_ovf = 0;
    regions_frame<DILATE, 64 * FW, false>(a, (int)f, uf, s_nc, s_nr);  // (ends with a barrier)
    step_barrier();
    const int nc = s_nc, nr = s_nr;
    {
        const Scratch sc = light_scratch(fr_lds, wv);
        for (int k = wv; k < nc; k += FW) {
            const int ti = a.clist[f * a.ntiles + k];
            if (FM_OOB(a, ti >= 0 && ti < a.ntiles, 1)) continue;
            const int r = label_tile<DILATE>(a, f, ti, ln, sc);
            if (ln == 0) {
                if (r == TCCL_RUNS) hl[atomicAdd(&s_nh, 1)] = ti;
                else if (r != TCCL_OK) s_ovf = 1;
            }
        }
    }
    step_barrier();
    const int nh = s_nh;
    if (nh && wv == 0) {  // tiles with more than LIGHT runs: the whole scratch, one wave
        const Scratch sc = heavy_scratch(fr_lds);
        for (int i = 0; i < nh; i++) {
            const int ti = hl[i];
            const int r = tile_ccl<MAXR>(a, f, ti, ln, a.dbits[(f * a.ntiles + ti) * 64 + ln], sc);
            if (r != TCCL_OK && ln == 0) s_ovf = 1;
        }
    }
    step_barrier();
    const bool ovf = s_ovf != 0;  // (workgroup-uniform) the host relabels the frame (pixel-level fallback)
    if (!ovf) {
        merge_frame(a, f, nc, wv, FW, ln);
        step_barrier();
        fold_frame(a, f, nc, nr, wv, FW, ln);
        step_barrier();
        emit_frame(a, f, wv, FW, ln, a.rec + f * a.cap * 5, &a.count[f], a.cap);
        step_barrier();
    }
    if (tid == 0) {
        if (ovf) a.count[F + f] = 1;
        a.h_count[f] = ovf ? 0 : a.count[f];
        a.h_overflow[f] = ovf ? 1 : 0;
        // slot-wide tallies: the frame's heavy tiles; the last frame to finish reports them with the shared
        // pool's use and re-arms the three words for the slot's next batch (the next launch sees the stores).
        // Every pool and heavy-tally atomic of a workgroup has returned before its frames-done increment is
        // issued (take_nodes uses its result; the tally's is tested below), so the last workgroup's reads
        // see them all.
        const int hb = nh ? atomicAdd(&a.count[2 * F + 1], nh) : 0;
        if (atomicAdd(&a.count[3 * F + 2], hb < 0 ? 0 : 1) == (int)F - 1) {
            const int shared = __hip_atomic_load(&a.count[2 * F], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int heavy = __hip_atomic_load(&a.count[2 * F + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.h_stats[0] = shared;
            a.h_stats[1] = heavy;
            a.count[2 * F] = 0;
            a.count[2 * F + 1] = 0;
            a.count[3 * F + 2] = 0;
        }
    }
    if (a.tflag_waves == 1)  // (the k_fused path's per-tile flag words, as k_counts)
        for (int t = tid; t < a.ntiles; t += 64 * FW) a.tflag[f * a.ntiles + t] = 0;
#ifdef FM_DEV_SWITCHES
    kstamp_end_wg(a.kstamp);
#endif
}

}  // namespace cc

hipError_t launch_contour_area(hipStream_t st, const uint64_t* dbits, const uint8_t* candf, const uint8_t* mask, int ntiles,
                               int ntx, int h, int w, const int32_t* jobs, int n, int32_t* area2) {
    if (n <= 0) return hipSuccess;
    const cc::AreaMask m{dbits, candf, mask, ntiles, ntx, h, w};
    hipLaunchKernelGGL(cc::k_contour_area, dim3((n + 255) / 256), dim3(256), 0, st, m, jobs, n, area2);
    return hipGetLastError();
}

hipError_t launch_frame_contours(hipStream_t st, const FusedArgs& a, bool dilate) {
    if (a.ntiles > cc::MAX_REGION_TILES) return hipErrorInvalidValue;
    const unsigned F = (unsigned)(a.T * a.S);
    const size_t lds = cc::FR_SCRATCH + 2 * sizeof(int) * (size_t)a.ntiles;
    if (lds > 65536) return hipErrorInvalidValue;
    if (dilate) hipLaunchKernelGGL(cc::k_frame_contours<true>, dim3(F), dim3(64 * cc::FW), lds, st, a);
    else hipLaunchKernelGGL(cc::k_frame_contours<false>, dim3(F), dim3(64 * cc::FW), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_tile_ccl(hipStream_t st, const FusedArgs& a, bool dilate, KernelTimer* tm, hipEvent_t gate_wait,
                           hipEvent_t gate_done) {
    if (a.ntiles > cc::MAX_REGION_TILES) return hipErrorInvalidValue;
    const unsigned F = (unsigned)(a.T * a.S);
    const dim3 gf(cc::GW, F);
    int tok = tm ? tm->begin("regions", st) : -1;
    const size_t rg_lds = (size_t)a.ntiles * sizeof(int);
    FusedArgs ar = a, ac = a;  // (dev build: the chain's first and last kernels stamped, for pipeline traces)
#ifdef FM_DEV_SWITCHES
    ar.kstamp = tm ? tm->stamp("chain_regions") : nullptr;
    ac.kstamp = tm ? tm->stamp("chain_counts") : nullptr;
#endif
    if (dilate) hipLaunchKernelGGL(cc::k_regions<true>, dim3(F), dim3(cc::RG), rg_lds, st, ar);
    else hipLaunchKernelGGL(cc::k_regions<false>, dim3(F), dim3(cc::RG), rg_lds, st, ar);
    if (tm) tm->end(tok);
    if (gate_wait) {
        const hipError_t e = hipStreamWaitEvent(st, gate_wait, 0);
        if (e != hipSuccess) return e;
    }
    tok = tm ? tm->begin("tile_ccl", st) : -1;
    if (dilate) hipLaunchKernelGGL(cc::k_tile_ccl<true>, gf, dim3(64 * cc::CW), cc::TC_LDS, st, a);
    else hipLaunchKernelGGL(cc::k_tile_ccl<false>, gf, dim3(64 * cc::CW), cc::TC_LDS, st, a);
    if (gate_done) {
        const hipError_t e = hipEventRecord(gate_done, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(cc::k_tile_heavy, dim3(cc::NHW), dim3(64), cc::HEAVY_LDS, st, a);
    if (tm) tm->end(tok);
    tok = tm ? tm->begin("merge", st) : -1;
    hipLaunchKernelGGL(cc::k_merge, gf, dim3(64 * cc::CW), 0, st, a);
    if (tm) tm->end(tok);
    tok = tm ? tm->begin("fold_emit", st) : -1;
    hipLaunchKernelGGL(cc::k_fold, gf, dim3(64 * cc::CW), 0, st, a);
    hipLaunchKernelGGL(cc::k_emit, gf, dim3(64 * cc::CW), 0, st, a);
    hipLaunchKernelGGL(cc::k_counts, dim3(F), dim3(cc::FT), 0, st, ac);
    if (tm) tm->end(tok);
    return hipGetLastError();
}

hipError_t launch_emit_all(hipStream_t st, const FusedArgs& a, int f, int32_t* rec, int32_t* cnt, int cap) {
    hipLaunchKernelGGL(cc::k_emit_all, dim3(cc::GW), dim3(64 * cc::CW), 0, st, a, f, rec, cnt, cap);
    return hipGetLastError();
}

hipError_t launch_expand_bits(hipStream_t st, const uint64_t* dbits, const uint8_t* candf, uint8_t* out, int h, int w,
                              int ntx) {
    dim3 grid((unsigned)(((w + 7) / 8 + 255) / 256), (unsigned)h);
    hipLaunchKernelGGL(cc::k_expand_bits, grid, dim3(256), 0, st, dbits, candf, out, h, w, ntx);
    return hipGetLastError();
}



}  // namespace fm
