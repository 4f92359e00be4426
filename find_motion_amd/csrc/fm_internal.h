// fm_internal.h — shared declarations between the C ABI (fm_capi.cpp) and the
// gfx950 kernels (fm_kernels.hip).  Not part of the public boundary.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/find_motion_amd.h"

namespace fm {

template <int I> struct IntC { static constexpr int value = I; };
// compile-time unrolled loop: fn(IntC<0>{}), ..., fn(IntC<N-1>{})
template <int N, int I = 0, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
    if constexpr (I < N) {
        fn(IntC<I>{});
        static_for<N, I + 1>(fn);
    }
}

// Developer switches (A/B experiments, profiling stamps) are read from the environment
// only by the dev build (make VARIANT=dev -> libfm_hip_dev.so); the product library
// ignores the environment.
inline const char* dev_env(const char* name) {
#ifdef FM_DEV_SWITCHES
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Bounds checks on every data-dependent index of the contour pass (make VARIANT=checked ->
// libfm_hip_checked.so): a violation sets bit `code` of the mapped error word, the access is
// skipped, and fm_wait fails with the codes.  Compiled out of the product library.
#ifdef FM_BOUNDS_CHECK
#define FM_OOB(a, cond, code) (!(cond) ? (atomicOr((a).dbg_err, 1 << (code)), true) : false)
#else
#define FM_OOB(a, cond, code) false
#endif

constexpr int kMaxK = 255;        // largest Gaussian size handled by the tiled kernel
constexpr int kCclBlock = 32;     // CCL block edge (pixels)
constexpr int kTileMaxRuns = 1600; // runs per 64x64 tile of a dilated mask (<= 24 per row => 1536)
constexpr int kHeavyWaves = 64;       // k_tile_heavy persistent waves (fm_ccl.hip)
constexpr int kNodesPerTileFrame = 32; // union-find nodes each frame owns per tile (its quota)
constexpr int kFrameCclTiles = 16;     // work images of at most this many tiles: one contour workgroup per frame
constexpr int kNodesShared = 16;       // + a shared overflow pool of this many per tile-frame (at least one
                                       //   worst-case frame), taken from only by frames past their quota

// Host-built INTER_AREA tables (computeResizeAreaTab restated in fm_capi.cpp).
// Per destination index d: taps start at src index ofs[d], cnt[d] taps, weights
// wt[d * max_taps + j] (float32 exactly as OpenCV stores DecimateAlpha::alpha).
struct AreaAxis {
    int n_dst = 0, max_taps = 0;
    std::vector<int32_t> ofs, cnt;
    std::vector<float> wt;
};

// Everything the per-frame pixel kernel needs for one batch step.
struct PixelArgs {
    const uint8_t* src;          // work-size BGR for this batch frame t: [S][h][w][3]
    double* bg;                  // [S][h*w]
    const uint8_t* keep;         // [S][h*w] (only read where has_keep[s])
    const uint8_t* has_keep;     // [S]
    const uint8_t* init;         // [S] 1 => bg := blur before the diff (first frame), or nullptr
    uint8_t* mask_out;           // dilated threshold [S][h*w]
    uint8_t* gray_out;           // optional planes [S][h*w] (nullptr when not kept)
    uint8_t* blur_out;
    uint8_t* delta_out;
    int S, h, w;
    int ksize;
    int thresh;
    double alpha, beta;          // beta = 1 - alpha
    long long acc_vec_end;       // h*w - (h*w % 16): AVX2 fma body vs scalar tail
    int cvt_simd;                // h*w >= 16: f64->f32->rne path of convertScaleAbs
    int32_t coef[kMaxK];         // fixed-point Gaussian taps (sum 256)
};

struct CclArgs {
    const uint8_t* mask;         // [F][h*w]
    int32_t* label;              // [F][h*w]
    uint8_t* outer;              // [F][h*w]
    int32_t* cid;                // [F][h*w]
    int32_t* count;              // [F]
    int32_t* rec;                // [F][cap][5]: first, minx, miny, maxx, maxy
    int F, h, w, cap;
};

// Temporally blocked fused kernel + tile-summary CCL (fm_fused.hip, fm_ccl.hip).
// Global CCL nodes of one batch slot: ids [0, F*ntiles) are the empty-tile regions
// (node f*ntiles + representative tile); a labelled candidate tile takes nroots
// consecutive ids (TileRec::nbase) from its frame's quota [F*ntiles + f*nquota, +nquota),
// or past that from the slot's shared overflow pool (ids from F*ntiles + F*nquota).
struct NodeRec {
    uint64_t key;     // foreground: (raster-first pixel << 32) | left-background reference
    int32_t parent;   // global union-find
    uint32_t flags;   // bit0 foreground, bit1 background touching the image border (outer)
    int32_t minx, maxx, maxy, pad;
};
struct TileRec {
    int32_t nroots;                   // components of the tile (ordinals 0..nroots-1, raster order)
    int32_t nbase;                    // node id of ordinal 0 (nodes of a candidate tile are consecutive)
    int32_t pad[2];
    uint16_t edges[256];              // 0..63 left col, 64.. right col, 128.. top row, 192.. bottom row:
                                      // component ordinal | fg << 15
};

// per-tile threshold-bit flags written by the pixel kernel (decide which tiles the
// 5x5 dilation can make non-empty: the tile itself or a neighbour's 2-px margin)
enum : uint32_t {
    FLAG_ANY = 1u, FLAG_L = 2u, FLAG_R = 4u, FLAG_T = 8u, FLAG_B = 16u,
    FLAG_TL = 32u, FLAG_TR = 64u, FLAG_BL = 128u, FLAG_BR = 256u,
};

struct FusedArgs {
    const uint8_t* src;          // work-size BGR frames [T][S][h][w][3]
    const double* bg_in;         // [S][h*w] background before the batch
    double* bg_out;              // [S][h*w] background after the batch
    const uint8_t* keep;         // [S][h*w]
    const uint8_t* has_keep;     // [S]
    const uint8_t* init;         // [S] or nullptr: 1 => bg := blur at the batch's first frame
    uint8_t* mask_out;           // [T][S][h*w] dilated threshold
    uint8_t* planes;             // optional [3][T][S][h*w] gray, blur, frame_delta
    uint64_t* bits;              // [F][ntiles][64] threshold rows as bit masks (k_pix output, k_dilate_ccl input)
    uint64_t* dbits;             // [F][ntiles][64] dilated rows (VideoFrame.thresh as bits; == bits when the
                                 // pixel kernel dilates itself, i.e. the generic-k k_fused path)
    TileRec* tiles;              // [F][ntiles]
    uint32_t* tflag;             // [F][ntiles][tflag_waves] FLAG_* bits: where the tile has threshold bits (dilated
                                 // bits on the k_fused path, which sets FLAG_ANY only)
    uint8_t* candf;              // [F][ntiles] 1: the tile's dilated mask may be non-empty (labelled)
    int32_t* clist;              // [F][ntiles] candidate tiles of each frame
    int32_t* rlist;              // [F][ntiles] representative tile of each empty-tile region
    int32_t* regrep;             // [F][ntiles] empty tile -> its region's representative tile
    int32_t* ncr;                // [F][2] candidates, regions
    NodeRec* nodes;              // [nnodes]: F*ntiles region nodes, then the pool of candidate-tile nodes
    int32_t* count;              // [3F+3]: [f] external contours, [F+f] overflow flag, [2F] shared node-pool
                                 // fill, [2F+1] heavy tiles listed, [2F+2+f] frame f's node-quota fill, [3F+2]
                                 // frames done (k_frame_contours; its last workgroup re-arms [2F], [2F+1], [3F+2])
    int32_t* h_stats;            // mapped host [2]: nodes taken from the shared pool, heavy tiles (written by
                                 // k_counts, or by the last k_frame_contours workgroup; diagnostics)
    int32_t* heavy;              // [F * ntiles] tiles with more runs than the light CCL pass holds
    int32_t* rec;                // [F][cap][5]
    int32_t* h_count;            // mapped host [F]: external contours per frame (written by k_fold_emit)
    int32_t* h_overflow;         // mapped host [F]: frame needs the pixel-level fallback
    int T, S, h, w, ksize, thresh;
    int t_begin, t_end;          // k_pix: frames of the batch this launch processes
    int ntx, nty, ntiles, nnodes, cap, cvt_simd;
    int nquota;                  // nodes per frame quota
    int tflag_waves;             // words per tile-frame in tflag: 1 (k_fused, atomicOr) or 8 (k_pix, one per wave)
    int dbg_skip;                // profiling-only stage ablation (FM_DEBUG_SKIP); 0 in normal use
    uint64_t* dbg_ts;            // profiling-only s_memtime stamps [F][ntiles][16] (FM_TS); nullptr in normal use
    uint64_t* dbg_pts;           // profiling-only k_pix workgroup stamps [S][ntiles][4] (FM_PTS); nullptr in normal use
    int32_t* dbg_err;            // mapped host word: FM_OOB violation bits (checked build only)
    double alpha, beta;
    long long acc_vec_end;
    int any_keep;                // some stream of the context has a keep-mask (k_pix5 variant choice)
    uint64_t* kstamp;            // this launch's [first start, last end] stamp pair (KernelTimer::stamp) or nullptr
    int32_t coef[kMaxK];
};

// In-kernel launch stamps (KernelTimer::stamp): thread 0 of every workgroup takes the 100 MHz
// s_memrealtime counter at its start into ks[0] (atomic min), lane 0 of every wave at its end into
// ks[1] (atomic max), so ks[1] - ks[0] is the launch from its first workgroup's start to its last
// wave's end.  Plain (vector) global atomics that return nothing.
__device__ __forceinline__ void kstamp_begin(uint64_t* ks) {
    if (ks && threadIdx.x == 0)
        atomicMin(reinterpret_cast<unsigned long long*>(ks), (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void kstamp_end(uint64_t* ks) {
    if (ks && (threadIdx.x & 63) == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(ks) + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
// Kernels of thousands of short workgroups (the INTER_AREA resize): the start from the first 8
// workgroups dispatched, the end from wave 0 of every workgroup (one atomic per workgroup).
__device__ __forceinline__ void kstamp_begin_grid(uint64_t* ks) {
    if (blockIdx.x + blockIdx.y * gridDim.x < 8) kstamp_begin(ks);
}
__device__ __forceinline__ void kstamp_end_wg(uint64_t* ks) {
    if (threadIdx.x < 64) kstamp_end(ks);
}

// computeResizeAreaTab restated (fm_capi.cpp); false if a destination's taps are not consecutive
bool build_area_axis(int ssize, int dsize, double scale, AreaAxis& A);

// Kernel launchers (fm_kernels.hip, fm_fused.hip).  All asynchronous on `st`.
hipError_t launch_resize_area(hipStream_t st, const uint8_t* src, uint8_t* dst, int F, int H, int W,
                              int h, int w, const int32_t* xofs, const int32_t* xcnt, const float* xwt,
                              int xtaps, const int32_t* yofs, const int32_t* ycnt, const float* ywt,
                              int ytaps, const uint8_t* const* srcs = nullptr, uint64_t* kstamp = nullptr);
hipError_t launch_resize_area_fast(hipStream_t st, const uint8_t* src, uint8_t* dst, int F, int H, int W,
                                   int h, int w, int sx, int sy, uint64_t* kstamp = nullptr);
hipError_t launch_pixel(hipStream_t st, const PixelArgs& a);
struct KernelTimer;
hipError_t launch_ccl(hipStream_t st, const CclArgs& a, KernelTimer* timer);
hipError_t launch_fused(hipStream_t st, const FusedArgs& a, KernelTimer* timer);
int fused_lds_bytes(int ksize);
int fused_max_ksize();
// k_pix (fm_pix.hip): chain once per pixel, threshold bits out; dilation in the CCL kernel
// frames [a.t_begin, a.t_end) of the batch; init: a.init may mark first frames (only at t_begin)
hipError_t launch_pix(hipStream_t st, const FusedArgs& a, bool planes, bool init);
int pix_lds_bytes(int ksize);
bool pix_supported(int ksize);
// small work images (fm_small.hip): k_small_blur (every frame of the launch in parallel) + k_small_scan
// (one wave per column and tile row, lane = row); sblur: small_scratch_bytes of the batch's frames
bool small_supported(int h, int w, int ksize);
size_t small_scratch_bytes(int h, int w, int nty, size_t frames);
hipError_t launch_small(hipStream_t st, const FusedArgs& a, uint8_t* sblur, uint64_t* ks_blur, uint64_t* ks_scan);
// CCL over tile summaries; dilate = true: a.bits are threshold rows to dilate into a.dbits
// gate_wait / gate_done (optional): the labelling kernel waits for gate_wait (the previous batch's
// labelling) and gate_done is recorded after it, so that one batch's labelling runs at a time
hipError_t launch_tile_ccl(hipStream_t st, const FusedArgs& a, bool dilate, KernelTimer* timer,
                           hipEvent_t gate_wait = nullptr, hipEvent_t gate_done = nullptr);
// the whole contour pass of each frame in one workgroup (a.ntiles <= kFrameCclTiles; count[] sized 3F + 3, the
// slot-wide words count[2F], count[2F + 1], count[3F + 2] zero before the first batch: the kernel re-arms them)
hipError_t launch_frame_contours(hipStream_t st, const FusedArgs& a, bool dilate);
// every external-contour record of frame f of a finished batch (all of them, unlike the
// capped k_emit), into rec [cap][5]; *cnt must be 0 before
hipError_t launch_emit_all(hipStream_t st, const FusedArgs& a, int f, int32_t* rec, int32_t* cnt, int cap);
// 2 x contourArea of external contours by border following (fm_ccl.hip): jobs [n][3] = (frame, origin x,
// origin y); the dilated mask of frame f is dbits/candf (fused path, [F][ntiles]...) or mask [F][h*w] bytes
hipError_t launch_contour_area(hipStream_t st, const uint64_t* dbits, const uint8_t* candf, const uint8_t* mask, int ntiles,
                               int ntx, int h, int w, const int32_t* jobs, int n, int32_t* area2);
// dilated bit rows of one frame -> mask bytes (VideoFrame.thresh) [h][w]; non-candidate tiles are 0
hipError_t launch_expand_bits(hipStream_t st, const uint64_t* dbits, const uint8_t* candf, uint8_t* out, int h, int w,
                              int ntx);

// Optional per-kernel timing.  FM_FLAG_PROFILE: events recorded on the launch stream around each
// kernel, read back after the stream syncs.  FM_FLAG_PROFILE_PIX: the pixel kernel and the INTER_AREA
// resize only, EVERY launch timed by in-kernel stamps (stamp(): no event packet enters the streams);
// other kernels on the pixel / input stream by events on one launch in kSample.
struct KernelTimer {
    bool enabled = false;
    bool pixel_only = false;
    static constexpr int kSample = 4;
    static constexpr int kStampRing = 4096;  // stamped launches held between two folds (more go untimed)
    std::vector<int64_t> calls;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;  // also timed in the pixel-only mode: the input stream's resize
    hipStream_t stream3 = nullptr;  // (the second input stream)
    std::vector<hipStream_t> extra; // other streams stamped kernels run on (the contour streams; dev-build stamps)
    struct Rec { int id; hipEvent_t a, b; hipStream_t st; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    std::vector<const char*> names;
    std::vector<double> ms;
    std::vector<int64_t> launches;
    std::vector<double> ms_sq;      // sum of squared stamped launch times (ms^2)
    std::vector<int64_t> stamped;   // launches timed by stamps (ms_sq's count; `launches` adds event-timed ones)
    std::vector<double> stamped_ms; // their summed time (ms)
    struct Busy { double ms = 0; uint64_t s = 0, e = 0; bool open = false; };
    std::vector<Busy> busy;         // union of the stamped launch windows (closed part + the open interval)
    uint64_t* d_stamps = nullptr;   // device [kStampRing][2]: (first start, last end), ticks of 10 ns
    std::vector<int> stamp_ids;     // name id of ring entries [0, stamp_ids.size()) not yet folded
    int64_t unstamped = 0;          // launches that found the ring full
    int id_of(const char* name);
    int begin(const char* name, hipStream_t st = nullptr);  // token for end(), -1 when disabled
    void end(int token);
    void collect();                // folds in every pair whose end event has completed
    uint64_t* stamp(const char* name);  // this launch's stamp pair, nullptr when not stamping
    int fold_stamps();             // waits for the stamped streams, folds and re-arms the entries
    void reset();
    ~KernelTimer();
};

}  // namespace fm

// decode side (fm_jpeg.hip): queue the decode of n JPEGs into BGR frames at device address out on
// stream st; FM_* status, the message in fm_mjpeg_last_error
int fm_mjpeg_enqueue(fm_mjpeg* d, const uint8_t* const* jpegs, const size_t* sizes, int n, uint8_t* out, hipStream_t st);
