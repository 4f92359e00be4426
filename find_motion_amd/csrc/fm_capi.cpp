// fm_capi.cpp — C ABI of the MI355X motion-detection hot path (include/find_motion_amd.h).
//
// Owns the per-context device state (background models, masks, batch
// buffers), builds the host-side tables OpenCV builds per call (INTER_AREA
// taps, fixed-point Gaussian taps) once at fm_create, and sequences the
// kernels of fm_kernels.hip on one HIP stream per context.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "fm_internal.h"

namespace fm {
hipError_t launch_pixel_pp(hipStream_t st, const PixelArgs& a, const double* bg_in, double* bg_out);
int pixel_lds_bytes(int ksize);
}  // namespace fm

using namespace fm;

namespace {

thread_local std::string g_last_error;

enum class ResizeMode { Identity, Fast, General };

}  // namespace

// One batch's device results.  The fused paths keep kSlots slots: the pixel
// kernels run in submission order on the pixel stream (the background
// recurrence), each slot's contour pass on its own stream, so the latency-bound
// contour passes of consecutive batches overlap each other and the next
// batches' pixel kernels.
#ifndef FM_SLOTS
// with the labelling gate a chain finishes later, and 4 slots left the pixel stream idle while the host waited
// to reuse one: 6 slots 406.4 vs 396.4 k frames/s (4 alternating rounds, round 3).  Round 5, 6 / 8 / 10 slots
// (profiles/r05q_slots_ab.txt): the driver's command 374-409 / 401-403 / 393-413 k, mode D (60 steps)
// 762-767 / 775-792 / 801-805 k; a slot is ~0.41 GB of device memory at the headline shape
#define FM_SLOTS 10
#endif
constexpr int kSlots = FM_SLOTS;
struct BatchSlot {
    uint8_t* d_in = nullptr;        // host-fed staging [T][S][H][W][3]
    uint8_t* d_work = nullptr;      // resized BGR [T][S][h][w][3] (mode D)
    uint8_t* d_planes = nullptr;    // [3][T][S][h*w] gray, blur, frame_delta (FM_FLAG_KEEP_PLANES)
    uint64_t* d_bits = nullptr;     // threshold bit rows (k_pix output)
    uint8_t* d_sblur = nullptr;     // small work images: blur bytes [T*S][w][nty * 64] (k_small_blur -> k_small_scan)
    uint64_t* d_dbits = nullptr;    // dilated bit rows = VideoFrame.thresh
    TileRec* d_tiles = nullptr;
    NodeRec* d_nodes = nullptr;
    uint32_t* d_tflag = nullptr;    // [F][ntiles] where tiles have threshold bits
    uint8_t* d_candf = nullptr;     // [F][ntiles] tiles the contour pass labelled
    int32_t* d_clist = nullptr;     // [F][ntiles] candidate lists
    int32_t* d_rlist = nullptr;     // [F][ntiles] empty-region representatives
    int32_t* d_regrep = nullptr;    // [F][ntiles] empty tile -> region representative
    int32_t* d_ncr = nullptr;       // [F][2]
    int32_t* d_heavy = nullptr;     // [F * ntiles] heavy-tile list
    int32_t* d_count = nullptr;     // [3F+3]: counts, overflow flags, pool / heavy words, frame quotas, frames done
    int32_t* h_count = nullptr;     // pinned [F]
    int32_t* h_overflow = nullptr;  // pinned [F]
    int32_t* dh_count = nullptr;     // device aliases of the two (mapped): the fused path's k_counts writes them
    int32_t* dh_overflow = nullptr;
    int32_t* h_stats = nullptr;     // mapped [2]: shared-pool nodes, heavy tiles (k_counts)
    int32_t* dh_stats = nullptr;
    int32_t* h_rec = nullptr;       // mapped pinned [F][cap][5], written by the kernels
    int32_t* d_rec = nullptr;       // device alias of h_rec
    uint8_t* h_init = nullptr;      // pinned [S]
    hipEvent_t ev_pix = nullptr, ev_done = nullptr, ev_rs = nullptr, ev_lab = nullptr;  // (ev_lab: labelling done)
    hipStream_t ccl_stream = nullptr;  // this slot's contour pass (slots' passes run concurrently)
    int n = 0;                      // frames in flight in this slot (0 = none)
    FusedArgs fa{};                 // the contour pass's arguments (fm_wait re-emits frames past the cap)
    uint64_t gen = 0;               // submits into this slot
    size_t ccl_F = 0;               // frames (T*S) of the slot's last k_frame_contours batch (its re-armed words)
    const uint8_t* src = nullptr;   // the batch's source frames [T][S][H][W][3] on the device (fm_read_frame)
};

struct fm_ctx {
    fm_params p{};
    int h = 0, w = 0;
    size_t src_frame_bytes = 0, work_plane = 0;
    ResizeMode rmode = ResizeMode::Identity;
    int fast_sx = 1, fast_sy = 1;
    AreaAxis ax, ay;
    std::vector<int32_t> coef;

    // streams: pixel work (caller-replaceable), contour pass, synchronous reads
    hipStream_t own_stream = nullptr, stream = nullptr, aux_stream = nullptr;
    hipStream_t rs_stream = nullptr;  // input stream: host copies + resize, ahead of the pixel stream
    hipStream_t rs_stream2 = nullptr; // second input stream (odd slots' resizes), created with the first resize
    hipStream_t ccl_streams[kSlots] = {};
    int lab_prev = -1;  // slot of the last batch whose labelling was enqueued (the labelling gate)
    int nccl = 1;
    KernelTimer timer;

    // device state shared by all batches
    double* d_bg[2] = {nullptr, nullptr};
    int bg_cur = 0;
    uint8_t* d_keep = nullptr;    // [S][h*w]
    uint8_t* d_has_keep = nullptr;
    uint8_t* d_init = nullptr;
    uint8_t* d_mask = nullptr;    // fused: one plane (fm_read_mask expansion, pixel-CCL fallback); v1: [T][S][h*w]
    int32_t* d_label = nullptr;   // pixel-level CCL (v1 path, fused-path overflow fallback)
    int32_t* d_cid = nullptr;
    uint8_t* d_outer = nullptr;
    int32_t* d_rec_dev = nullptr;  // per-frame path: the batch's pixel-level CCL records [frames][max_contours][5]
    int32_t* d_rec_one = nullptr;  // relabel_frame: one frame's records [rec_one_cap][5] (grown on demand)
    size_t rec_one_cap = 0;
    int32_t* d_area = nullptr;     // FM_FLAG_CONTOUR_AREA: jobs [area_cap][3] + areas [area_cap]
    size_t area_cap = 0;
    int32_t* d_rec_all = nullptr;  // k_emit_all records of one frame [rec_all_cap][5] + counter
    size_t rec_all_cap = 0;
    int rec_cap = 0;          // records per frame in each slot's mapped buffer (the first fetch; more -> k_emit_all)
    size_t dev_bytes = 0;     // device bytes the context holds now (fm_footprint)
    std::unordered_map<const void*, size_t> dev_sizes;  // (so that a freed buffer leaves dev_bytes)
    size_t pinned_bytes = 0;  // and its page-locked host allocations
    bool use_fused = false;
    bool use_pix = false;          // k_pix + dilating tile CCL (else k_fused dilates itself)
    bool use_small = false;        // the pixel stage as k_small_blur + k_small_scan (small work images)
    bool frame_ccl = false;        // the contour pass as one workgroup per frame (ntiles <= kFrameCclTiles)
    int ntx = 0, nty = 0, ntiles = 0, nnodes = 0;  // nnodes: per batch slot
    int nquota = 0;                                             // nodes of each frame's quota
    int32_t *d_xofs = nullptr, *d_xcnt = nullptr, *d_yofs = nullptr, *d_ycnt = nullptr;
    float *d_xwt = nullptr, *d_ywt = nullptr;

    // batches
    BatchSlot slots[kSlots];
    int nslots = 1;
    int next_slot = 0;
    std::vector<int> inflight;     // FIFO of submitted, not yet waited slots
    int ready_slot = -1;           // slot of the last waited batch
    uint64_t ready_gen = 0;
    int ready = 0;                 // frames of the last waited batch
    int fallbacks = 0;             // its frames relabelled by the pixel-level CCL (node pool exhausted)
    int32_t stats[2] = {0, 0};     // its contour pass: nodes from the shared pool, heavy tiles
    std::vector<int32_t> ready_counts;                    // [ready * S]
    std::vector<std::vector<fm_contour>> contours;        // per (t*S+s), sorted

    std::vector<uint8_t> bg_init, has_keep;
    std::string err;
    uint64_t* d_ts = nullptr;     // FM_TS: contour-pass phase stamps (profiling)
    uint64_t* d_pts = nullptr;    // FM_PTS=<file>: k_pix workgroup stamps of the last launch (profiling)
    int pts_ring = 1;             // FM_PTS_RING=<n>: stamps of the last n launches, oldest first (profiling)
    long long pts_launches = 0;
    int32_t* h_err = nullptr;     // mapped: FM_OOB violation bits (checked build), 0 otherwise
    int32_t* dh_err = nullptr;
    std::vector<double> ts_sum;   // summed phase deltas (cycles)
    std::vector<int64_t> ts_n;
    bool serial = false;  // FM_SERIAL: contour pass on the pixel stream (profiling: no overlap)
    int dbg_skip = 0;  // FM_DEBUG_SKIP: profiling-only stage ablation of k_fused (results invalid)
};

namespace {

int fail(fm_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    if (c) c->err = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) return fail(ctx, FM_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

// computeResizeAreaTab (OpenCV imgproc resize.cpp) restated on the product
// side: for each destination index the weights over consecutive source
// indices, in the order OpenCV accumulates them.
}  // namespace
namespace fm {
bool build_area_axis(int ssize, int dsize, double scale, AreaAxis& A) {
    A.n_dst = dsize;
    std::vector<std::vector<std::pair<int, float>>> taps(dsize);
    for (int dx = 0; dx < dsize; dx++) {
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cell = std::min(scale, ssize - fsx1);
        int sx1 = (int)std::ceil(fsx1), sx2 = (int)std::floor(fsx2);
        sx2 = std::min(sx2, ssize - 1);
        sx1 = std::min(sx1, sx2);
        auto& t = taps[dx];
        if (sx1 - fsx1 > 1e-3) t.emplace_back(sx1 - 1, (float)((sx1 - fsx1) / cell));
        for (int sx = sx1; sx < sx2; sx++) t.emplace_back(sx, (float)(1.0 / cell));
        if (fsx2 - sx2 > 1e-3) t.emplace_back(sx2, (float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell));
    }
    A.max_taps = 1;
    for (auto& t : taps) A.max_taps = std::max<int>(A.max_taps, (int)t.size());
    A.ofs.assign(dsize, 0);
    A.cnt.assign(dsize, 0);
    A.wt.assign((size_t)dsize * A.max_taps, 0.f);
    for (int d = 0; d < dsize; d++) {
        auto& t = taps[d];
        if (t.empty()) return false;
        A.ofs[d] = t[0].first;
        A.cnt[d] = (int)t.size();
        for (size_t j = 0; j < t.size(); j++) {
            if (t[j].first != t[0].first + (int)j) return false;  // taps must be consecutive
            A.wt[(size_t)d * A.max_taps + j] = t[j].second;
        }
    }
    return true;
}
}  // namespace fm
namespace {

// getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (OpenCV imgproc
// smooth.dispatch.cpp) restated: the 8-bit fixed-point taps GaussianBlur
// uses for CV_8U with sigma = 0.
bool gaussian_taps(int n, std::vector<int32_t>& out) {
    if (n < 1 || (n & 1) == 0 || n > kMaxK) return false;
    std::vector<double> kd(n);
    switch (n) {
        case 1: kd = {1.0}; break;
        case 3: kd = {0.25, 0.5, 0.25}; break;
        case 5: kd = {0.0625, 0.25, 0.375, 0.25, 0.0625}; break;
        case 7: kd = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125}; break;
        case 9: kd = {4 / 256., 13 / 256., 30 / 256., 51 / 256., 60 / 256., 51 / 256., 30 / 256., 13 / 256., 4 / 256.}; break;
        default: {
            const double sigma = std::fma((double)n, 0.15, 0.35);
            const double scale2 = -0.125 / (sigma * sigma);
            const int half = (n - 1) / 2;
            std::vector<double> v(half);
            double sum = 0;
            for (int i = 0, x = 1 - n; i < half; i++, x += 2) {
                v[i] = std::exp((double)(x * x) * scale2);
                sum += v[i];
            }
            sum = sum * 2 + 1;
            for (int i = 0; i < half; i++) kd[i] = kd[n - 1 - i] = v[i] / sum;
            kd[half] = 1 / sum;
        }
    }
    out.assign(n, 0);
    const int half = n / 2;
    double err = 0;
    int64_t s = 0;
    for (int i = 0; i < half; i++) {
        const double adj = kd[i] * 256 + err;
        const int64_t v0 = (int64_t)std::nearbyint(adj);
        err = adj - (double)v0;
        out[i] = out[n - 1 - i] = (int32_t)v0;
        s += v0;
    }
    out[half] = (int32_t)(256 - 2 * s);
    return true;
}

template <class T>
int dalloc(fm_ctx* c, T** p, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return fail(c, FM_ENOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
    if (c) {
        c->dev_bytes += count * sizeof(T);
        c->dev_sizes[*p] = count * sizeof(T);
    }
    return FM_OK;
}

// page-locked host memory of the context (counted for fm_footprint)
template <class T>
hipError_t halloc(fm_ctx* c, T** p, size_t bytes, unsigned flags) {
    hipError_t e = hipHostMalloc((void**)p, bytes, flags);
    if (e == hipSuccess) c->pinned_bytes += bytes;
    return e;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}
// a buffer freed while the context lives on (re-grown): its bytes leave the footprint
template <class T>
void dfree(fm_ctx* c, T*& p) {
    if (p) {
        auto it = c->dev_sizes.find(p);
        if (it != c->dev_sizes.end()) {
            c->dev_bytes -= it->second;
            c->dev_sizes.erase(it);
        }
    }
    dfree(p);
}

int check_idle(fm_ctx* c) {
    if (!c->inflight.empty()) return fail(c, FM_ESTATE, "a submit is in flight: call fm_wait first");
    return FM_OK;
}

// results of the last waited batch (device-side ones live until its slot is resubmitted)
int check_frame(fm_ctx* c, int frame, int stream, bool device_data) {
    if (stream < 0 || stream >= c->p.n_streams) return fail(c, FM_EINVAL, "stream %d out of range", stream);
    if (frame < 0 || frame >= c->ready) return fail(c, FM_EINVAL, "frame %d not in the last batch (%d frames)", frame, c->ready);
    if (device_data && (c->ready_slot < 0 || c->slots[c->ready_slot].gen != c->ready_gen))
        return fail(c, FM_ESTATE, "the batch's device results were overwritten by a later submit");
    return FM_OK;
}

// every record of frame f of a finished fused-path batch (count known from k_emit)
int emit_all(fm_ctx* c, BatchSlot& B, size_t f, int count, std::vector<int32_t>& out) {
    if ((size_t)count > c->rec_all_cap) {
        dfree(c, c->d_rec_all);
        c->rec_all_cap = 0;
        if (int rc = dalloc(c, &c->d_rec_all, (size_t)count * 5 + 1)) return rc;
        c->rec_all_cap = (size_t)count;
    }
    hipStream_t st = c->aux_stream;
    int32_t* cnt = c->d_rec_all + (size_t)count * 5;
    HIP_TRY(c, hipMemsetAsync(cnt, 0, sizeof(int32_t), st));
    HIP_TRY(c, launch_emit_all(st, B.fa, (int)f, c->d_rec_all, cnt, count));
    out.resize((size_t)count * 5 + 1);
    HIP_TRY(c, hipMemcpyAsync(out.data(), c->d_rec_all, out.size() * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    if (out.back() != count) return fail(c, FM_EHIP, "re-emit of frame %zu found %d contours, not %d", f, out.back(), count);
    out.pop_back();
    return FM_OK;
}

// frame f of a fused-path batch through the pixel-level CCL (from its dilated bit rows):
// all records into out, the count into count
int relabel_frame(fm_ctx* c, BatchSlot& B, size_t f, std::vector<int32_t>& out, int& count) {
    hipStream_t st = c->aux_stream;
    int32_t* dcnt = B.d_count + f;  // this frame's contour counter (the batch is finished)
    const uint8_t* mask = c->d_mask + f * c->work_plane;  // per-frame path: the batch's dilated masks
    if (c->use_fused) {
        HIP_TRY(c, launch_expand_bits(st, B.d_dbits + f * c->ntiles * 64, B.d_candf + f * c->ntiles, c->d_mask, c->h,
                                      c->w, c->ntx));
        mask = c->d_mask;
    }
    for (int pass = 0; pass < 2; pass++) {
        HIP_TRY(c, hipMemsetAsync(dcnt, 0, sizeof(int32_t), st));
        HIP_TRY(c, hipMemsetAsync(c->d_outer, 0, c->work_plane, st));
        // its own record buffer: the per-frame path's d_rec_dev holds [frames][max_contours] records
        // for every submit and must keep that size
        CclArgs ca{mask, c->d_label, c->d_outer, c->d_cid, dcnt, c->d_rec_one, 1, c->h, c->w, (int)c->rec_one_cap};
        HIP_TRY(c, launch_ccl(st, ca, nullptr));
        int32_t n = 0;
        HIP_TRY(c, hipMemcpyAsync(&n, dcnt, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipStreamSynchronize(st));
        if ((size_t)n <= c->rec_one_cap) {
            count = n;
            out.resize((size_t)n * 5);
            HIP_TRY(c, hipMemcpyAsync(out.data(), c->d_rec_one, out.size() * sizeof(int32_t), hipMemcpyDeviceToHost, st));
            HIP_TRY(c, hipStreamSynchronize(st));
            return FM_OK;
        }
        dfree(c, c->d_rec_one);
        c->rec_one_cap = 0;
        if (int rc = dalloc(c, &c->d_rec_one, (size_t)n * 5)) return rc;
        c->rec_one_cap = (size_t)n;
    }
    return fail(c, FM_EHIP, "pixel-level relabel of frame %zu did not converge", f);
}

// FM_FLAG_CONTOUR_AREA: 2 x contourArea of every contour of the finished batch in slot B, traced
// on the GPU from its start pixel on the batch's dilated masks (fm.py:679)
int contour_areas(fm_ctx* c, BatchSlot& B, size_t F) {
    std::vector<int32_t> jobs;
    for (size_t f = 0; f < F; f++)
        for (const fm_contour& o : c->contours[f]) {
            jobs.push_back((int32_t)f);
            jobs.push_back(o.origin_x);
            jobs.push_back(o.origin_y);
        }
    const size_t n = jobs.size() / 3;
    if (n == 0) return FM_OK;
    if (n > c->area_cap) {
        dfree(c, c->d_area);
        c->area_cap = 0;
        if (int rc = dalloc(c, &c->d_area, n * 4)) return rc;
        c->area_cap = n;
    }
    hipStream_t st = c->aux_stream;
    std::vector<int32_t> a2(n);
    HIP_TRY(c, hipMemcpyAsync(c->d_area, jobs.data(), n * 3 * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(c, launch_contour_area(st, c->use_fused ? B.d_dbits : nullptr, c->use_fused ? B.d_candf : nullptr,
                                   c->use_fused ? nullptr : c->d_mask, c->ntiles, c->ntx, c->h, c->w, c->d_area, (int)n,
                                   c->d_area + n * 3));
    HIP_TRY(c, hipMemcpyAsync(a2.data(), c->d_area + n * 3, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    size_t k = 0;
    for (size_t f = 0; f < F; f++)
        for (fm_contour& o : c->contours[f]) {
            if (a2[k] < 0) return fail(c, FM_EHIP, "contour of frame %zu at (%d, %d) has no closed border", f, o.origin_x,
                                       o.origin_y);
            o.area2 = a2[k++];
        }
    return FM_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// KernelTimer
namespace fm {
int KernelTimer::id_of(const char* name) {
    for (size_t i = 0; i < names.size(); i++)
        if (names[i] == name || std::strcmp(names[i], name) == 0) return (int)i;
    names.push_back(name);
    ms.push_back(0);
    ms_sq.push_back(0);
    stamped.push_back(0);
    stamped_ms.push_back(0);
    busy.push_back(Busy{});
    launches.push_back(0);
    calls.push_back(0);
    return (int)names.size() - 1;
}
int KernelTimer::begin(const char* name, hipStream_t st) {
    if (!enabled) return -1;
    if (!st) st = stream;
    if (pixel_only && st != stream && st != stream2) return -1;
    const int id = id_of(name);
    // events on every launch cost the pipeline ~7% (each record is a barrier packet):
    // the pixel-only mode times a sample of the launches of the kernels it cannot stamp
    if (pixel_only && calls[id]++ % kSample != 0) return -1;
    hipEvent_t a, b;
    if (pool.size() >= 2) {
        a = pool.back(); pool.pop_back();
        b = pool.back(); pool.pop_back();
    } else {
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
    }
    (void)hipEventRecord(a, st);
    pending.push_back({id, a, b, st});
    return (int)pending.size() - 1;
}
void KernelTimer::end(int token) {
    if (token < 0 || token >= (int)pending.size()) return;
    (void)hipEventRecord(pending[token].b, pending[token].st);
}
void KernelTimer::collect() {
    std::vector<Rec> keep;
    for (auto& r : pending) {
        if (hipEventQuery(r.b) == hipErrorNotReady) {  // a later batch still running
            keep.push_back(r);
            continue;
        }
        float t = 0;
        if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
            ms[r.id] += t;
            launches[r.id] += 1;
        }
        pool.push_back(r.a);
        pool.push_back(r.b);
    }
    pending.swap(keep);
}
// Stamped launches (pixel-only mode): the round-4 sampled events opened their window at the marker
// ahead of the kernel, so it took in the queue's waits, and one launch in four was a biased sample
// (a sampled mean of 709 us against a 655.5 us step).  Stamps time every launch from its first
// workgroup's start to its last wave's end.
uint64_t* KernelTimer::stamp(const char* name) {
    if (!enabled || !pixel_only) return nullptr;
    if (!d_stamps) {
        if (hipMalloc(&d_stamps, sizeof(uint64_t) * 2 * kStampRing) != hipSuccess) {
            d_stamps = nullptr;
            enabled = false;
            return nullptr;
        }
        std::vector<uint64_t> init(2 * kStampRing);
        for (int i = 0; i < kStampRing; i++) init[2 * i] = ~0ull, init[2 * i + 1] = 0;
        if (hipMemcpy(d_stamps, init.data(), init.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess) {
            enabled = false;
            return nullptr;
        }
    }
    const int id = id_of(name);
    if ((int)stamp_ids.size() >= kStampRing) {
        unstamped++;
        return nullptr;
    }
    stamp_ids.push_back(id);
    return d_stamps + 2 * (stamp_ids.size() - 1);
}
int KernelTimer::fold_stamps() {
    if (stamp_ids.empty()) return 0;
    if (stream) (void)hipStreamSynchronize(stream);
    if (stream2) (void)hipStreamSynchronize(stream2);
    if (stream3) (void)hipStreamSynchronize(stream3);
    for (hipStream_t st : extra) (void)hipStreamSynchronize(st);  // (an entry read while its kernel runs is lost)
    const size_t n = stamp_ids.size();
    std::vector<uint64_t> v(2 * n);
    if (hipMemcpy(v.data(), d_stamps, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    const bool dump = dev_env("FM_STAMP_DUMP") != nullptr;  // dev build: every launch's window to stderr
    for (size_t i = 0; i < n; i++) {
        if (dump) std::fprintf(stderr, "kstamp %s %llu %llu\n", names[stamp_ids[i]], (unsigned long long)v[2 * i],
                               (unsigned long long)v[2 * i + 1]);
        if (v[2 * i] == ~0ull || v[2 * i + 1] <= v[2 * i]) continue;  // (a kernel that does not stamp)
        const double t = (double)(v[2 * i + 1] - v[2 * i]) * 1e-5;  // 100 MHz ticks -> ms
        ms[stamp_ids[i]] += t;
        ms_sq[stamp_ids[i]] += t * t;
        stamped[stamp_ids[i]] += 1;
        stamped_ms[stamp_ids[i]] += t;
        launches[stamp_ids[i]] += 1;
    }
    // the union of each kernel's launch windows (launches of one kernel may overlap: two input streams)
    std::vector<std::pair<uint64_t, uint64_t>> iv;
    for (size_t id = 0; id < names.size(); id++) {
        iv.clear();
        for (size_t i = 0; i < n; i++)
            if (stamp_ids[i] == (int)id && v[2 * i] != ~0ull && v[2 * i + 1] > v[2 * i]) iv.emplace_back(v[2 * i], v[2 * i + 1]);
        std::sort(iv.begin(), iv.end());
        Busy& b = busy[id];
        for (const auto& [s0, e0] : iv) {
            if (b.open && s0 <= b.e) {
                b.e = std::max(b.e, e0);
                continue;
            }
            if (b.open) b.ms += (double)(b.e - b.s) * 1e-5;
            b.s = s0, b.e = e0, b.open = true;
        }
    }
    for (size_t i = 0; i < n; i++) v[2 * i] = ~0ull, v[2 * i + 1] = 0;
    stamp_ids.clear();
    return hipMemcpy(d_stamps, v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
void KernelTimer::reset() {
    fold_stamps();  // (launches stamped before the reset are dropped with the sums below)
    std::fill(ms.begin(), ms.end(), 0.0);
    std::fill(ms_sq.begin(), ms_sq.end(), 0.0);
    std::fill(stamped.begin(), stamped.end(), 0);
    std::fill(stamped_ms.begin(), stamped_ms.end(), 0.0);
    std::fill(busy.begin(), busy.end(), Busy{});
    std::fill(launches.begin(), launches.end(), 0);
    std::fill(calls.begin(), calls.end(), 0);
    unstamped = 0;
}
KernelTimer::~KernelTimer() {
    if (d_stamps) (void)hipFree(d_stamps);
    for (auto& r : pending) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
}
}  // namespace fm

// ---------------------------------------------------------------------------
extern "C" {

int fm_abi_version(void) { return FM_ABI_VERSION; }

const char* fm_last_error(const fm_ctx* ctx) { return ctx ? ctx->err.c_str() : g_last_error.c_str(); }

int fm_create(fm_ctx** out, const fm_params* prm) {
    if (!out || !prm) return fail(nullptr, FM_EINVAL, "null argument");
    *out = nullptr;
    const fm_params& p = *prm;
    if (p.n_streams < 1 || p.src_w < 1 || p.src_h < 1 || p.box_size < 1 || p.max_batch < 1 || p.max_contours < 1)
        return fail(nullptr, FM_EINVAL, "invalid geometry (streams %d, src %dx%d, box %d, batch %d, contours %d)",
                    p.n_streams, p.src_w, p.src_h, p.box_size, p.max_batch, p.max_contours);
    if (p.ksize < 1 || (p.ksize & 1) == 0 || p.ksize > kMaxK)
        return fail(nullptr, FM_EINVAL, "ksize %d must be odd and in [1, %d]", p.ksize, kMaxK);
    if (!(p.avg == p.avg)) return fail(nullptr, FM_EINVAL, "avg is NaN");

    std::unique_ptr<fm_ctx> c(new fm_ctx());
    c->p = p;
    c->w = p.box_size;
    c->h = (int)(p.src_h * ((double)p.box_size / (double)p.src_w));  // imutils.resize
    if (c->h < 1) return fail(nullptr, FM_EINVAL, "work height is 0 (box %d, src %dx%d)", p.box_size, p.src_w, p.src_h);
    if ((int64_t)c->h * c->w >= (1ll << 31) / 2) return fail(nullptr, FM_ENOTSUP, "work image too large");

    // resize mode (cv::resize: copy if same size; INTER_AREA needs scale >= 1)
    if (c->h == p.src_h && c->w == p.src_w) {
        c->rmode = ResizeMode::Identity;
    } else {
        const double sx = 1. / ((double)c->w / p.src_w), sy = 1. / ((double)c->h / p.src_h);
        if (!(sx >= 1 && sy >= 1))
            return fail(nullptr, FM_ENOTSUP, "box_size %d > frame width %d: INTER_AREA upscaling is bilinear in OpenCV, not supported",
                        p.box_size, p.src_w);
        const int isx = (int)std::lrint(sx), isy = (int)std::lrint(sy);
        if (std::fabs(sx - isx) < 2.220446049250313e-16 && std::fabs(sy - isy) < 2.220446049250313e-16) {
            c->rmode = ResizeMode::Fast;
            c->fast_sx = isx;
            c->fast_sy = isy;
        } else {
            c->rmode = ResizeMode::General;
            if (!build_area_axis(p.src_w, c->w, sx, c->ax) || !build_area_axis(p.src_h, c->h, sy, c->ay))
                return fail(nullptr, FM_ENOTSUP, "INTER_AREA table with non-consecutive taps");
        }
    }
    if (!gaussian_taps(p.ksize, c->coef)) return fail(nullptr, FM_EINVAL, "bad ksize %d", p.ksize);
    if (pixel_lds_bytes(p.ksize) > 160 * 1024) return fail(nullptr, FM_ENOTSUP, "ksize %d too large for the LDS tile", p.ksize);

    fm_ctx* cp = c.get();
    HIP_TRY(cp, hipSetDevice(p.device));
    c->use_fused = p.ksize <= fused_max_ksize() && fused_lds_bytes(p.ksize) <= 160 * 1024 &&
                   ((c->w + 63) / 64) * ((c->h + 63) / 64) <= 8192;  // region labelling holds the tile grid in LDS
    // small work images (mode D: 1080p -> 100 x 56), any k: frame-parallel blur + per-pixel scan
    // (fm_small.hip; mode D 634 -> 746 k frames/s, round 5), unless the caller keeps the gray / blur /
    // delta planes (k_pix writes them).  Both it and k_pix write threshold bits for the dilating contour pass.
    c->use_small = c->use_fused && (size_t)c->h * c->w >= 16 && !(p.flags & FM_FLAG_KEEP_PLANES) &&
                   small_supported(c->h, c->w, p.ksize) && dev_env("FM_NO_PIX") == nullptr;
    if (const char* e = dev_env("FM_SMALL")) c->use_small = c->use_small && std::atoi(e) != 0;
    c->use_pix = c->use_small || (c->use_fused && pix_supported(p.ksize) && (size_t)c->h * c->w >= 16 &&
                                  pix_lds_bytes(p.ksize) <= 160 * 1024 && dev_env("FM_NO_PIX") == nullptr);
    // The pixel stream at high priority: it gets a hardware queue of its own instead of sharing one (in
    // order) with a contour-pass stream.  (Round 4 gave small work images' pixel stream 8 CUs of its own
    // -- k_pix5's chain / producer waves on two tiles were a latency chain the next resize starved; the
    // small-image path of round 5 runs a batch's frames in parallel over every CU instead.)
    {
        int lo = 0, hi = 0;
        HIP_TRY(cp, hipDeviceGetStreamPriorityRange(&lo, &hi));
        if (dev_env("FM_PIX_PRIO_OFF")) hi = lo;
        HIP_TRY(cp, hipStreamCreateWithPriority(&c->own_stream, hipStreamNonBlocking, hi));
    }
#ifndef FM_CCL_QMODE_DEFAULT
#define FM_CCL_QMODE_DEFAULT 2  // contour streams take their own hardware queues (A/B: +3 %)
#endif
#ifndef FM_NCCL_DEFAULT
// three contour streams.  Round 5, 3 alternating rounds each: the driver's command 1 stream 363-367 k (chains in
// a row fall behind), 2 streams 400-403 k, 3 streams 388-403 k (pixel launch std 14-22 us either way but for
// one 58 us run); mode D (60 steps) 2 streams 679-697 k, 3 streams 803-810 k (profiles/r05m_ccl_streams_ab.txt,
// r05o_ccl_streams_ab.txt)
#define FM_NCCL_DEFAULT 3
#endif
    int ccl_qmode = FM_CCL_QMODE_DEFAULT;
    if (const char* e = dev_env("FM_CCL_QMODE")) ccl_qmode = std::atoi(e);
    c->nccl = FM_NCCL_DEFAULT;
    if (const char* e = dev_env("FM_CCL_STREAMS")) c->nccl = std::max(1, std::min(kSlots, std::atoi(e)));
    if (ccl_qmode == 2)  // contour streams take hardware queues before the rarely used aux / input streams
        for (int i = 0; i < c->nccl; i++) HIP_TRY(cp, hipStreamCreateWithFlags(&c->ccl_streams[i], hipStreamNonBlocking));
    HIP_TRY(cp, hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
    // input stream: host-to-device copies and the resize run here, ahead of the pixel stream
    if (!dev_env("FM_RESIZE_INLINE")) HIP_TRY(cp, hipStreamCreateWithFlags(&c->rs_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    c->timer.enabled = (p.flags & (FM_FLAG_PROFILE | FM_FLAG_PROFILE_PIX)) != 0;
    c->timer.pixel_only = !(p.flags & FM_FLAG_PROFILE);
    c->timer.stream = c->stream;
    c->timer.stream2 = c->rs_stream;

    const size_t S = p.n_streams, T = p.max_batch;
    c->work_plane = (size_t)c->h * c->w;
    c->src_frame_bytes = (size_t)p.src_h * p.src_w * 3;
    const size_t frames = S * T, px = frames * c->work_plane;
    int rc;
    c->nslots = c->use_fused ? kSlots : 1;
    // contour-pass streams shared round-robin by the slots: few streams, because the
    // runtime multiplexes streams onto GPU_MAX_HW_QUEUES (4) hardware queues in order,
    // and a contour kernel queued ahead of a pixel kernel on a shared queue stalls it
    for (int i = 0; i < 2; i++)
        if ((rc = dalloc(cp, &c->d_bg[i], S * c->work_plane))) return rc;
    if ((rc = dalloc(cp, &c->d_keep, S * c->work_plane)) || (rc = dalloc(cp, &c->d_has_keep, S)) ||
        (rc = dalloc(cp, &c->d_init, S)) || (rc = dalloc(cp, &c->d_mask, c->use_fused ? c->work_plane : px)))
        return rc;
    if (c->use_fused) {
        c->ntx = (c->w + 63) / 64;
        c->nty = (c->h + 63) / 64;
        c->ntiles = c->ntx * c->nty;
        c->frame_ccl = c->ntiles <= kFrameCclTiles;
        // (dev: 0 = never, 2 = at any size)
        if (const char* e = dev_env("FM_FRAME_CCL")) c->frame_ccl = std::atoi(e) == 2 || (c->frame_ccl && std::atoi(e) != 0);
        // union-find nodes: one per empty-tile region slot, each frame's quota, and a shared
        // overflow pool that holds at least one worst-case frame (frames past it take the
        // pixel-level fallback)
        const size_t tf = frames * (size_t)c->ntiles;
        c->nquota = c->ntiles * kNodesPerTileFrame;
        const size_t nn = tf + tf * kNodesPerTileFrame + std::max(tf * kNodesShared, (size_t)c->ntiles * kTileMaxRuns);
        if (nn >= (size_t)INT32_MAX) return fail(nullptr, FM_ENOTSUP, "batch too large for 32-bit node ids (%zu)", nn);
        c->nnodes = (int)nn;
    }
    // Contour records: the fused path's mapped buffer holds the first rec_cap records of each frame (a
    // frame with more is re-emitted whole at fm_wait, so max_contours never changes the results): about
    // 32 MB per slot however many frames a batch has -- [frames][max_contours] records of 20 B were 671 MB
    // per slot at 8 streams x 256 frames and max_contours 1 << 14 (4 GB pinned per rank).  The per-frame
    // path copies [frames][max_contours] records from the device and keeps that size.
    c->rec_cap = p.max_contours;
    if (c->use_fused)
        c->rec_cap = (int)std::min<size_t>((size_t)p.max_contours,
                                           std::max<size_t>(64, (size_t(32) << 20) / (frames * 5 * sizeof(int32_t))));
    for (int i = 0; i < c->nslots; i++) {
        BatchSlot& b = c->slots[i];
        if (c->rmode != ResizeMode::Identity && (rc = dalloc(cp, &b.d_work, px * 3))) return rc;
        if ((rc = dalloc(cp, &b.d_count, 3 * frames + 3))) return rc;
        // (k_frame_contours re-arms its slot-wide words at the end of each batch: they start at zero)
        if (hipMemset(b.d_count, 0, (3 * frames + 3) * sizeof(int32_t)) != hipSuccess)
            return fail(cp, FM_EHIP, "hipMemset of the batch counters failed");
        if ((p.flags & FM_FLAG_KEEP_PLANES) && (rc = dalloc(cp, &b.d_planes, px * 3))) return rc;
        if (c->use_fused) {
            if ((rc = dalloc(cp, &b.d_heavy, frames * c->ntiles)) ||
                (rc = dalloc(cp, &b.d_tiles, frames * c->ntiles)) ||
                (rc = dalloc(cp, &b.d_tflag, frames * c->ntiles * 8)) || (rc = dalloc(cp, &b.d_candf, frames * c->ntiles)) ||
                (rc = dalloc(cp, &b.d_clist, frames * c->ntiles)) || (rc = dalloc(cp, &b.d_rlist, frames * c->ntiles)) ||
                (rc = dalloc(cp, &b.d_regrep, frames * c->ntiles)) || (rc = dalloc(cp, &b.d_ncr, frames * 2)) ||
                (rc = dalloc(cp, &b.d_dbits, frames * c->ntiles * 64)) ||
                (c->use_pix && (rc = dalloc(cp, &b.d_bits, frames * c->ntiles * 64))) ||
                (c->use_small && (rc = dalloc(cp, &b.d_sblur, small_scratch_bytes(c->h, c->w, c->nty, frames)))) ||
                (rc = dalloc(cp, &b.d_nodes, (size_t)c->nnodes)))
                return rc;
        }
        // contour records: mapped pinned host memory written directly by the kernels
        // (only the records that exist cross PCIe)
        HIP_TRY(cp, halloc(cp, &b.h_rec, frames * (size_t)c->rec_cap * 5 * sizeof(int32_t), hipHostMallocMapped));
        HIP_TRY(cp, hipHostGetDevicePointer((void**)&b.d_rec, b.h_rec, 0));
        HIP_TRY(cp, halloc(cp, &b.h_count, frames * sizeof(int32_t), hipHostMallocMapped));
        HIP_TRY(cp, hipHostGetDevicePointer((void**)&b.dh_count, b.h_count, 0));
        HIP_TRY(cp, halloc(cp, &b.h_overflow, frames * sizeof(int32_t), hipHostMallocMapped));
        HIP_TRY(cp, halloc(cp, &b.h_stats, 2 * sizeof(int32_t), hipHostMallocMapped));
        HIP_TRY(cp, hipHostGetDevicePointer((void**)&b.dh_stats, b.h_stats, 0));
        HIP_TRY(cp, hipHostGetDevicePointer((void**)&b.dh_overflow, b.h_overflow, 0));
        if (b.d_tflag) HIP_TRY(cp, hipMemset(b.d_tflag, 0, frames * c->ntiles * 8 * sizeof(uint32_t)));
        HIP_TRY(cp, halloc(cp, &b.h_init, S, 0));
        if (i < c->nccl && ccl_qmode != 2) {
            if (ccl_qmode == 1) {
                int lo = 0, hi = 0;
                HIP_TRY(cp, hipDeviceGetStreamPriorityRange(&lo, &hi));
                HIP_TRY(cp, hipStreamCreateWithPriority(&c->ccl_streams[i], hipStreamNonBlocking, hi));
            } else {
                HIP_TRY(cp, hipStreamCreateWithFlags(&c->ccl_streams[i], hipStreamNonBlocking));
            }
        }
        b.ccl_stream = c->ccl_streams[i % c->nccl];
        if (i < c->nccl) c->timer.extra.push_back(b.ccl_stream);  // fold_stamps waits for it too
        HIP_TRY(cp, hipEventCreateWithFlags(&b.ev_pix, hipEventDisableTiming));
        HIP_TRY(cp, hipEventCreateWithFlags(&b.ev_done, hipEventDisableTiming));
        HIP_TRY(cp, hipEventCreateWithFlags(&b.ev_rs, hipEventDisableTiming));
        HIP_TRY(cp, hipEventCreateWithFlags(&b.ev_lab, hipEventDisableTiming));
    }
    // pixel-level CCL: the whole batch on the v1 path, one frame for the fused path's overflow fallback
    const size_t ccl_px = c->use_fused ? c->work_plane : px;
    if ((rc = dalloc(cp, &c->d_label, ccl_px)) || (rc = dalloc(cp, &c->d_cid, ccl_px)) ||
        (rc = dalloc(cp, &c->d_outer, ccl_px)) ||
        (!c->use_fused && (rc = dalloc(cp, &c->d_rec_dev, frames * (size_t)p.max_contours * 5))) ||
        (rc = dalloc(cp, &c->d_rec_one, (size_t)p.max_contours * 5)))
        return rc;
    c->rec_one_cap = (size_t)p.max_contours;
    HIP_TRY(cp, halloc(cp, &c->h_err, sizeof(int32_t), hipHostMallocMapped));
    HIP_TRY(cp, hipHostGetDevicePointer((void**)&c->dh_err, c->h_err, 0));
    *c->h_err = 0;
    HIP_TRY(cp, hipMemset(c->d_has_keep, 0, S));
    HIP_TRY(cp, hipMemset(c->d_bg[0], 0, S * c->work_plane * sizeof(double)));
    HIP_TRY(cp, hipMemset(c->d_bg[1], 0, S * c->work_plane * sizeof(double)));
    if (c->rmode == ResizeMode::General) {
        auto up = [&](auto** d, const auto& v) -> int {
            int r = dalloc(cp, d, v.size());
            if (r) return r;
            hipError_t e = hipMemcpy(*d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice);
            return e == hipSuccess ? 0 : fail(cp, FM_EHIP, "hipMemcpy tables: %s", hipGetErrorString(e));
        };
        if ((rc = up(&c->d_xofs, c->ax.ofs)) || (rc = up(&c->d_xcnt, c->ax.cnt)) || (rc = up(&c->d_xwt, c->ax.wt)) ||
            (rc = up(&c->d_yofs, c->ay.ofs)) || (rc = up(&c->d_ycnt, c->ay.cnt)) || (rc = up(&c->d_ywt, c->ay.wt)))
            return rc;
    }
    c->bg_init.assign(S, 0);
    c->has_keep.assign(S, 0);
    if (const char* e = dev_env("FM_DEBUG_SKIP")) c->dbg_skip = std::atoi(e);
    c->serial = dev_env("FM_SERIAL") != nullptr;
    if (dev_env("FM_PTS") && c->use_pix) {
        // per launch: [S][ntiles][4] workgroup stamps, then [S][ntiles][8 waves][4] k_pix5 phase cycles
        if (const char* e = dev_env("FM_PTS_RING")) c->pts_ring = std::max(1, std::min(256, std::atoi(e)));
        const size_t n = (size_t)S * c->ntiles * 36 * c->pts_ring;
        if ((rc = dalloc(cp, &c->d_pts, n))) return rc;
        HIP_TRY(cp, hipMemset(c->d_pts, 0, n * sizeof(uint64_t)));
    }
    if (dev_env("FM_TS") && c->use_fused) {
        if ((rc = dalloc(cp, &c->d_ts, frames * c->ntiles * 16))) return rc;
        c->ts_sum.assign(16, 0.0);
        c->ts_n.assign(16, 0);
    }
    // the initialising hipMemset calls run on the null stream, which does not order the
    // context's non-blocking streams: finish them before the first submit can read the buffers
    HIP_TRY(cp, hipDeviceSynchronize());
    *out = c.release();
    return FM_OK;
}

void fm_destroy(fm_ctx* c) {
    if (!c) return;
    if (c->d_pts) {  // profiling: per-workgroup (hw_id, xcc_id, realtime start/end, memtime start/end) of the last k_pix
        const size_t rec = (size_t)c->p.n_streams * c->ntiles * 36, n = rec * c->pts_ring;
        std::vector<uint64_t> v(n);
        if (hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(v.data(), c->d_pts, n * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE* fh = std::fopen(dev_env("FM_PTS"), "wb")) {  // dev build only (d_pts); oldest launch first
                const size_t r0 = (size_t)(c->pts_launches % c->pts_ring);
                for (int k = 0; k < c->pts_ring; k++)
                    std::fwrite(v.data() + ((r0 + k) % c->pts_ring) * rec, sizeof(uint64_t), rec, fh);
                std::fclose(fh);
            }
        }
        dfree(c->d_pts);
    }
    if (c->d_ts) {
        std::fprintf(stderr, "[fm] contour-pass phase cycles (mean per labelled tile):");
        for (int k = 2; k < 16; k++)
            if (c->ts_n[k]) std::fprintf(stderr, " %d:%.0f(n=%lld)", k, c->ts_sum[k] / c->ts_n[k], (long long)c->ts_n[k]);
        std::fprintf(stderr, "\n");
        dfree(c->d_ts);
    }
    (void)hipSetDevice(c->p.device);
    for (hipStream_t st : {c->own_stream, c->stream, c->aux_stream, c->rs_stream, c->rs_stream2})
        if (st) (void)hipStreamSynchronize(st);
    for (hipStream_t& st : c->ccl_streams)
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
            st = nullptr;
        }
    for (auto& b : c->slots) {
        dfree(b.d_in); dfree(b.d_work); dfree(b.d_planes); dfree(b.d_bits); dfree(b.d_dbits); dfree(b.d_tiles); dfree(b.d_sblur);
        dfree(b.d_nodes); dfree(b.d_heavy); dfree(b.d_count); dfree(b.d_tflag); dfree(b.d_candf);
        dfree(b.d_clist); dfree(b.d_rlist); dfree(b.d_regrep); dfree(b.d_ncr);
        for (auto* hp : {(void*)b.h_count, (void*)b.h_overflow, (void*)b.h_rec, (void*)b.h_init, (void*)b.h_stats})
            if (hp) (void)hipHostFree(hp);
        if (b.ev_pix) (void)hipEventDestroy(b.ev_pix);
        if (b.ev_done) (void)hipEventDestroy(b.ev_done);
        if (b.ev_rs) (void)hipEventDestroy(b.ev_rs);
        if (b.ev_lab) (void)hipEventDestroy(b.ev_lab);
    }
    dfree(c->d_bg[0]); dfree(c->d_bg[1]); dfree(c->d_keep); dfree(c->d_has_keep); dfree(c->d_init); dfree(c->d_mask);
    dfree(c->d_label); dfree(c->d_cid); dfree(c->d_outer); dfree(c->d_rec_dev); dfree(c->d_rec_one); dfree(c->d_rec_all); dfree(c->d_area);
    dfree(c->d_xofs); dfree(c->d_xcnt); dfree(c->d_xwt); dfree(c->d_yofs); dfree(c->d_ycnt); dfree(c->d_ywt);
    for (hipStream_t st : {c->own_stream, c->aux_stream, c->rs_stream, c->rs_stream2})
        if (st) (void)hipStreamDestroy(st);
    if (c->h_err) (void)hipHostFree(c->h_err);
    delete c;
}

int fm_host_alloc(fm_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    *out = nullptr;
    HIP_TRY(c, hipSetDevice(c->p.device));
    HIP_TRY(c, hipHostMalloc(out, bytes, hipHostMallocPortable));
    return FM_OK;
}

int fm_host_free(fm_ctx* c, void* ptr) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (ptr) HIP_TRY(c, hipHostFree(ptr));
    return FM_OK;
}

int fm_max_inflight(const fm_ctx* c) { return c ? c->nslots : fail(nullptr, FM_EINVAL, "null context"); }

int fm_work_size(const fm_ctx* c, int* h, int* w) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (h) *h = c->h;
    if (w) *w = c->w;
    return FM_OK;
}

int fm_set_mask(fm_ctx* c, int stream, const uint8_t* keep) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (int rc = check_idle(c)) return rc;
    if (stream < 0 || stream >= c->p.n_streams) return fail(c, FM_EINVAL, "stream %d out of range", stream);
    HIP_TRY(c, hipSetDevice(c->p.device));
    const uint8_t flag = keep ? 1 : 0;
    if (keep)
        HIP_TRY(c, hipMemcpyAsync(c->d_keep + (size_t)stream * c->work_plane, keep, c->work_plane,
                                  hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->d_has_keep + stream, &flag, 1, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->has_keep[stream] = flag;
    return FM_OK;
}

int fm_reset_stream(fm_ctx* c, int stream) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (int rc = check_idle(c)) return rc;
    if (stream < 0 || stream >= c->p.n_streams) return fail(c, FM_EINVAL, "stream %d out of range", stream);
    c->bg_init[stream] = 0;
    return FM_OK;
}

int fm_set_hip_stream(fm_ctx* c, void* s) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (int rc = check_idle(c)) return rc;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    c->timer.stream = c->stream;
    return FM_OK;
}

// fm_submit / fm_submit_jpeg: frames from host memory (copied), device memory, or JPEGs decoded
// on the input stream into the batch's device buffer (dec != nullptr)
static int submit_impl(fm_ctx* c, const uint8_t* frames, int n, int on_device, fm_mjpeg* dec,
                       const uint8_t* const* jpegs, const size_t* sizes, const uint8_t* const* per_stream = nullptr) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if ((int)c->inflight.size() >= c->nslots)
        return fail(c, FM_ESTATE, "%d batch(es) already in flight: call fm_wait first", (int)c->inflight.size());
    if (per_stream) {
        for (int s = 0; s < c->p.n_streams; s++)
            if (!per_stream[s]) return fail(c, FM_EINVAL, "null frames for stream %d", s);
        if (on_device && c->p.n_streams == 1) {  // one stream: [n][1] is the contiguous layout, read in place
            frames = per_stream[0];
            per_stream = nullptr;
        }
    }
    if ((!frames && !dec && !per_stream) || n < 1 || n > c->p.max_batch)
        return fail(c, FM_EINVAL, "n_frames %d outside [1, max_batch=%d] or null frames", n, c->p.max_batch);
    HIP_TRY(c, hipSetDevice(c->p.device));
    const int si = c->next_slot;
    BatchSlot& B = c->slots[si];
    const int S = c->p.n_streams;
    const size_t F = (size_t)n * S;
    hipStream_t ps = c->stream;  // pixel stream: pixel kernel (bg recurrence is ordered here)
    // input copy and resize: on their own stream when there is a resize, so batch i+1's
    // resize (many workgroups, HBM-bound) overlaps batch i's pixel kernel (few, when the
    // work image is small); the pixel stream waits for it below
    hipStream_t rs = c->rs_stream ? c->rs_stream : ps;
#ifndef FM_RS_TWO
#define FM_RS_TWO 1
#endif
    // Consecutive batches' resizes on two input streams (odd slots on the second): in one in-order stream each
    // waited for the previous one's last wave and then its own dispatch (6-19 us a batch in mode D), on two the
    // next one's workgroups fill the previous one's tail.  Each batch's resize writes its own slot's buffer, and
    // the pixel stream waits for its batch's event, so the order of the batches is unchanged.
    if (FM_RS_TWO && c->rs_stream && !dec && c->rmode != ResizeMode::Identity && (si & 1)) {
        if (!c->rs_stream2) {
            HIP_TRY(c, hipStreamCreateWithFlags(&c->rs_stream2, hipStreamNonBlocking));
            c->timer.stream3 = c->rs_stream2;
        }
        rs = c->rs_stream2;
    }
    const uint8_t* src = frames;
    if (dec) {  // the decode side (§8(f)-3): JPEGs -> BGR frames in the batch's device buffer
        if (!B.d_in) {
            int rc = dalloc(c, &B.d_in, (size_t)c->p.max_batch * S * c->src_frame_bytes);
            if (rc) return rc;
        }
        const int rc = fm_mjpeg_enqueue(dec, jpegs, sizes, (int)F, B.d_in, rs);
        HIP_TRY(c, hipSetDevice(c->p.device));
        if (rc) return fail(c, rc, "JPEG decode: %s", fm_mjpeg_last_error(dec));
        src = B.d_in;
        on_device = 0;  // (the input stream ran: the pixel stream waits for it below)
    } else if (per_stream) {  // stream s's frames -> rows s, S + s, 2S + s, ... of the [t][s] batch layout
        if (!B.d_in) {
            int rc = dalloc(c, &B.d_in, (size_t)c->p.max_batch * S * c->src_frame_bytes);
            if (rc) return rc;
        }
        const size_t fb = c->src_frame_bytes;
        for (int s = 0; s < S; s++)
            HIP_TRY(c, hipMemcpy2DAsync(B.d_in + (size_t)s * fb, (size_t)S * fb, per_stream[s], fb, fb, (size_t)n,
                                        on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, rs));
        src = B.d_in;
        on_device = 0;
    } else if (!on_device) {
        if (!B.d_in) {
            int rc = dalloc(c, &B.d_in, (size_t)c->p.max_batch * S * c->src_frame_bytes);
            if (rc) return rc;
        }
        HIP_TRY(c, hipMemcpyAsync(B.d_in, frames, F * c->src_frame_bytes, hipMemcpyHostToDevice, rs));
        src = B.d_in;
    }
    const uint8_t* work = src;
    if (c->rmode == ResizeMode::General) {
        uint64_t* ks = c->timer.stamp("resize_area");
        int tok = ks ? -1 : c->timer.begin("resize_area", rs);
        HIP_TRY(c, launch_resize_area(rs, src, B.d_work, (int)F, c->p.src_h, c->p.src_w, c->h, c->w, c->d_xofs, c->d_xcnt,
                                      c->d_xwt, c->ax.max_taps, c->d_yofs, c->d_ycnt, c->d_ywt, c->ay.max_taps, nullptr, ks));
        c->timer.end(tok);
        work = B.d_work;
    } else if (c->rmode == ResizeMode::Fast) {
        uint64_t* ks = c->timer.stamp("resize_area_fast");
        int tok = ks ? -1 : c->timer.begin("resize_area_fast", rs);
        HIP_TRY(c, launch_resize_area_fast(rs, src, B.d_work, (int)F, c->p.src_h, c->p.src_w, c->h, c->w, c->fast_sx,
                                           c->fast_sy, ks));
        c->timer.end(tok);
        work = B.d_work;
    }
    if (rs != ps && (!on_device || c->rmode != ResizeMode::Identity)) {  // something ran on the input stream
        HIP_TRY(c, hipEventRecord(B.ev_rs, rs));
        HIP_TRY(c, hipStreamWaitEvent(ps, B.ev_rs, 0));
    }
    bool any_init = false;
    for (int s = 0; s < S; s++) {
        B.h_init[s] = c->bg_init[s] ? 0 : 1;
        any_init |= B.h_init[s] != 0;
    }
    if (any_init) HIP_TRY(c, hipMemcpyAsync(c->d_init, B.h_init, S, hipMemcpyHostToDevice, ps));

    const long long npx = (long long)c->work_plane;
    // fused path: counters zeroed by k_pix (k_regions on the k_fused path), tile flags cleared by k_counts
    if (!c->use_fused) HIP_TRY(c, hipMemsetAsync(B.d_count, 0, (2 * F + 1) * sizeof(int32_t), ps));
    if (c->use_fused) {
        FusedArgs fa{};
        fa.src = work;
        fa.bg_in = c->d_bg[c->bg_cur];
        fa.bg_out = c->d_bg[c->bg_cur ^ 1];
        fa.keep = c->d_keep;
        fa.has_keep = c->d_has_keep;
        fa.init = any_init ? c->d_init : nullptr;
        fa.mask_out = nullptr;
        fa.planes = B.d_planes;
        fa.bits = B.d_bits;
        fa.dbits = B.d_dbits;
        fa.tiles = B.d_tiles;
        fa.tflag = B.d_tflag;
        fa.tflag_waves = c->use_pix ? 8 : 1;
        fa.candf = B.d_candf;
        fa.clist = B.d_clist;
        fa.rlist = B.d_rlist;
        fa.regrep = B.d_regrep;
        fa.ncr = B.d_ncr;
        fa.nodes = B.d_nodes;
        fa.count = B.d_count;
        fa.heavy = B.d_heavy;
        fa.rec = B.d_rec;
        fa.h_count = B.dh_count;
        fa.h_overflow = B.dh_overflow;
        fa.T = n;
        fa.S = S;
        fa.h = c->h;
        fa.w = c->w;
        fa.ksize = c->p.ksize;
        fa.thresh = c->p.threshold;
        fa.ntx = c->ntx;
        fa.nty = c->nty;
        fa.ntiles = c->ntiles;
        fa.nnodes = c->nnodes;
        fa.nquota = c->nquota;
        fa.h_stats = B.dh_stats;
        fa.cap = c->rec_cap;
        fa.cvt_simd = npx >= 16;
        fa.alpha = c->p.avg;
        fa.beta = 1.0 - c->p.avg;
        fa.acc_vec_end = npx - npx % 16;
        fa.any_keep = std::any_of(c->has_keep.begin(), c->has_keep.end(), [](uint8_t k) { return k != 0; }) ? 1 : 0;
        fa.dbg_skip = c->dbg_skip;
        fa.dbg_ts = c->d_ts;
        fa.dbg_pts = c->d_pts ? c->d_pts + (size_t)(c->pts_launches++ % c->pts_ring) * S * c->ntiles * 36 : nullptr;
        fa.dbg_err = c->dh_err;
        if (c->d_ts) HIP_TRY(c, hipMemsetAsync(c->d_ts, 0, F * c->ntiles * 16 * sizeof(uint64_t), ps));
        for (int i = 0; i < c->p.ksize; i++) fa.coef[i] = c->coef[i];
        fa.t_begin = 0;
        fa.t_end = n;
        if (c->use_pix) {
            const bool planes = B.d_planes != nullptr;
            // each launch reads d_bg[cur] and writes d_bg[cur ^ 1]
            auto run = [&](int t0, int t1, bool init, const char* name) -> int {
                FusedArgs fp = fa;
                fp.t_begin = t0;
                fp.t_end = t1;
                fp.bg_in = c->d_bg[c->bg_cur];
                fp.bg_out = c->d_bg[c->bg_cur ^ 1];
                if (!init) fp.init = nullptr;
                if (c->use_small) {
                    uint64_t* k1 = c->timer.stamp(init ? "small_blur_init" : "small_blur");
                    uint64_t* k2 = c->timer.stamp(init ? "small_scan_init" : "small_scan");
                    // not stamping (FM_FLAG_PROFILE, or the stamp ring full): the pair timed by events
                    int tok = (k1 && k2) ? -1 : c->timer.begin(init ? "small_init" : "small", ps);
                    HIP_TRY(c, launch_small(ps, fp, B.d_sblur, k1, k2));
                    c->timer.end(tok);
                } else {
                    fp.kstamp = c->timer.stamp(name);
                    int tok = fp.kstamp ? -1 : c->timer.begin(name, ps);
                    HIP_TRY(c, launch_pix(ps, fp, planes, init));
                    c->timer.end(tok);
                }
                c->bg_cur ^= 1;
                return FM_OK;
            };
            int rc;
            if (any_init) {  // first frames in their own launch: the steady-state kernel has no init select
                if ((rc = run(0, 1, true, "pix_init"))) return rc;
                if (n > 1 && (rc = run(1, n, false, "pix"))) return rc;
            } else if ((rc = run(0, n, false, "pix"))) {
                return rc;
            }
        } else {
            HIP_TRY(c, launch_fused(ps, fa, &c->timer));
            c->bg_cur ^= 1;
        }
        // contour pass on its own stream, after this batch's pixel kernel
        // consecutive batches on different contour streams: with 4 slots on 3 streams a fixed
        // slot -> stream map put every fourth pair of consecutive chains on one stream, one after
        // the other (the last batch's chain waited ≈130 µs for its predecessor's)
        // (Batches taking the contour streams in turn instead of the fixed slot map: +2 % on one box,
        // equal on another with 8 % longer pixel launches, round 3.)
        hipStream_t cs = c->serial ? ps : B.ccl_stream;
        HIP_TRY(c, hipEventRecord(B.ev_pix, ps));
        HIP_TRY(c, hipStreamWaitEvent(cs, B.ev_pix, 0));
        // the labelling gate: one batch's labelling kernel at a time (the previous batch's, on another contour
        // stream, is waited for), so the labelling of consecutive chains never bunches beside a pixel launch
        // (+1.5 %, 388.1 vs 382.3 k, 4 alternating rounds, round 3)
        if (c->frame_ccl) {  // small work images: the whole pass of a frame in one workgroup (no gate needed)
            FusedArgs fc = fa;
#ifdef FM_DEV_SWITCHES
            fc.kstamp = c->timer.stamp("frame_contours");
#endif
            // FM_FLAG_PROFILE: events around it (a contour stream: never in the pixel-only mode)
            const int tok_fc = fc.kstamp ? -1 : c->timer.begin("frame_contours", cs);
            // the slot-wide words (shared pool, heavy tally, frames done) sit at indices that depend on the batch's
            // frame count; the last workgroup re-arms them for a batch of the same size, so a slot whose batch size
            // changed (a stream's last, partial batch) zeroes them at the new indices first
            if (B.ccl_F != F) {
                HIP_TRY(c, hipMemsetAsync(B.d_count + 2 * F, 0, 2 * sizeof(int32_t), cs));
                HIP_TRY(c, hipMemsetAsync(B.d_count + 3 * F + 2, 0, sizeof(int32_t), cs));
                B.ccl_F = F;
            }
            HIP_TRY(c, launch_frame_contours(cs, fc, c->use_pix));
            c->timer.end(tok_fc);
        } else {
            hipEvent_t gate_wait = nullptr;
            if (!c->serial && c->lab_prev >= 0 && c->lab_prev != si) gate_wait = c->slots[c->lab_prev].ev_lab;
            HIP_TRY(c, launch_tile_ccl(cs, fa, c->use_pix, &c->timer, gate_wait, B.ev_lab));
            c->lab_prev = si;
        }  // counts land in mapped h_count / h_overflow
        B.fa = fa;
        HIP_TRY(c, hipEventRecord(B.ev_done, cs));
    } else {
        PixelArgs a{};
        a.bg = nullptr;
        a.keep = c->d_keep;
        a.has_keep = c->d_has_keep;
        a.S = S;
        a.h = c->h;
        a.w = c->w;
        a.ksize = c->p.ksize;
        a.thresh = c->p.threshold;
        a.alpha = c->p.avg;
        a.beta = 1.0 - c->p.avg;
        a.acc_vec_end = npx - npx % 16;
        a.cvt_simd = npx >= 16;
        for (int i = 0; i < c->p.ksize; i++) a.coef[i] = c->coef[i];
        const size_t step_px = (size_t)S * c->work_plane;
        for (int t = 0; t < n; t++) {
            a.src = work + (size_t)t * step_px * 3;  // work image is [T][S][h][w][3] in every resize mode
            a.init = (t == 0 && any_init) ? c->d_init : nullptr;
            a.mask_out = c->d_mask + (size_t)t * step_px;
            if (B.d_planes) {
                a.gray_out = B.d_planes + (size_t)t * step_px;
                a.blur_out = B.d_planes + F * c->work_plane + (size_t)t * step_px;
                a.delta_out = B.d_planes + 2 * F * c->work_plane + (size_t)t * step_px;
            }
            int tok = c->timer.begin("pixel", ps);
            HIP_TRY(c, launch_pixel_pp(ps, a, c->d_bg[c->bg_cur], c->d_bg[c->bg_cur ^ 1]));
            c->timer.end(tok);
            c->bg_cur ^= 1;
        }
        HIP_TRY(c, hipMemsetAsync(c->d_outer, 0, F * c->work_plane, ps));
        CclArgs ca{c->d_mask, c->d_label, c->d_outer, c->d_cid, B.d_count, c->d_rec_dev, (int)F, c->h, c->w, c->p.max_contours};
        HIP_TRY(c, launch_ccl(ps, ca, &c->timer));
        HIP_TRY(c, hipMemcpyAsync(B.h_rec, c->d_rec_dev, F * c->p.max_contours * 5 * sizeof(int32_t), hipMemcpyDeviceToHost,
                                  ps));
        HIP_TRY(c, hipMemsetAsync(B.d_count + F, 0, F * sizeof(int32_t), ps));
        HIP_TRY(c, hipMemcpyAsync(B.h_overflow, B.d_count + F, F * sizeof(int32_t), hipMemcpyDeviceToHost, ps));
        HIP_TRY(c, hipMemcpyAsync(B.h_count, B.d_count, F * sizeof(int32_t), hipMemcpyDeviceToHost, ps));
        HIP_TRY(c, hipEventRecord(B.ev_done, ps));
    }
    for (int s = 0; s < S; s++) c->bg_init[s] = 1;
    B.n = n;
    B.src = src;
    B.gen++;
    c->inflight.push_back(si);
    c->next_slot = (si + 1) % c->nslots;
    return FM_OK;
}

int fm_submit(fm_ctx* c, const uint8_t* frames, int n, int on_device) {
    return submit_impl(c, frames, n, on_device, nullptr, nullptr, nullptr);
}

int fm_submit_streams(fm_ctx* c, const uint8_t* const* bgr, int n, int on_device) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (!bgr) return fail(c, FM_EINVAL, "null stream pointer array");
    return submit_impl(c, nullptr, n, on_device, nullptr, nullptr, nullptr, bgr);
}

int fm_submit_jpeg(fm_ctx* c, fm_mjpeg* dec, const uint8_t* const* jpegs, const size_t* sizes, int n) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (!dec || !jpegs || !sizes) return fail(c, FM_EINVAL, "null decoder or JPEG arrays");
    // the decoder writes n * S frames of its own size into the batch's input buffer (sized for this
    // context's frames): refuse any mismatch before anything is enqueued
    int dw = 0, dh = 0, ddev = -1, dmax = 0;
    if (fm_mjpeg_geometry(dec, &dw, &dh, &ddev, &dmax)) return fail(c, FM_EINVAL, "bad decoder");
    if (dw != c->p.src_w || dh != c->p.src_h || ddev != c->p.device)
        return fail(c, FM_EINVAL, "decoder for %dx%d frames on device %d, context for %dx%d on device %d", dw, dh, ddev,
                    c->p.src_w, c->p.src_h, c->p.device);
    if (n >= 1 && (long long)n * c->p.n_streams > dmax)
        return fail(c, FM_EINVAL, "decoder takes %d frames per call, the batch has %lld", dmax,
                    (long long)n * c->p.n_streams);
    return submit_impl(c, nullptr, n, 0, dec, jpegs, sizes);
}

int fm_wait(fm_ctx* c) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (c->inflight.empty()) return FM_OK;
    HIP_TRY(c, hipSetDevice(c->p.device));
    const int si = c->inflight.front();
    c->inflight.erase(c->inflight.begin());
    BatchSlot& B = c->slots[si];
#ifdef FM_DEV_SWITCHES  // host time in fm_wait (dev build): blocked on the batch vs the post-pass after it
    const auto hw0 = std::chrono::steady_clock::now();
#endif
    hipError_t e = hipEventSynchronize(B.ev_done);
    if (e != hipSuccess) {
        B.n = 0;
        return fail(c, FM_EHIP, "hipEventSynchronize: %s", hipGetErrorString(e));
    }
#ifdef FM_DEV_SWITCHES
    const auto hw1 = std::chrono::steady_clock::now();
#endif
    const int n = B.n, S = c->p.n_streams, cap = c->rec_cap;
    const size_t F = (size_t)n * S;
    // Frames whose records do not fit the cap are fetched whole, so len(frame.contours)
    // and the records kept never depend on max_contours (fm.py:674-694 counts them all).
    std::vector<std::pair<size_t, std::vector<int32_t>>> whole;
#ifdef FM_BOUNDS_CHECK
    if (*c->h_err) return fail(c, FM_EHIP, "contour-pass bounds check failed: codes 0x%x", *c->h_err);
#endif
    c->fallbacks = 0;
    if (c->use_fused) {
        c->stats[0] = B.h_stats[0];
        c->stats[1] = B.h_stats[1];
    }
    for (size_t f = 0; f < F; f++) {
        const bool ovf = c->use_fused && B.h_overflow[f];
        if (!ovf && B.h_count[f] <= cap) continue;
        std::vector<int32_t> v;
        if (c->use_fused && !ovf) {
            if (int rc = emit_all(c, B, f, B.h_count[f], v)) return rc;
        } else {
            // the contour pass ran out of nodes for this frame (fused path), or the per-frame
            // path kept only cap records: relabel it with the pixel-level CCL, every record
            int cnt = 0;
            if (int rc = relabel_frame(c, B, f, v, cnt)) return rc;
            B.h_count[f] = cnt;
            c->fallbacks += ovf;
        }
        whole.emplace_back(f, std::move(v));
    }
    c->timer.collect();
    if (c->d_ts) {  // profiling: mean cycles between consecutive stamps of each labelled tile
        std::vector<uint64_t> ts(F * c->ntiles * 16);
        HIP_TRY(c, hipMemcpy(ts.data(), c->d_ts, ts.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < F * c->ntiles; i++) {
            const uint64_t* t = &ts[i * 16];
            if (!t[1]) continue;
            uint64_t prev = t[1];
            for (int k = 2; k < 16; k++) {
                if (!t[k]) continue;
                c->ts_sum[k] += (double)(t[k] - prev);
                c->ts_n[k]++;
                prev = t[k];
            }
        }
    }
#ifdef FM_DEV_SWITCHES
    const auto hw2 = std::chrono::steady_clock::now();
#endif
    c->ready_counts.assign(B.h_count, B.h_count + F);
    c->contours.assign(F, {});
    size_t wi = 0;
    for (size_t f = 0; f < F; f++) {
        const int32_t* r = B.h_rec + f * cap * 5;
        int cnt = std::min(B.h_count[f], cap);
        if (wi < whole.size() && whole[wi].first == f) {
            r = whole[wi].second.data();
            cnt = (int)(whole[wi].second.size() / 5);
            wi++;
        }
        auto& v = c->contours[f];
        v.resize(cnt);
        std::vector<std::pair<int32_t, int>> order(cnt);
        for (int i = 0; i < cnt; i++) order[i] = {r[i * 5], i};
        std::sort(order.begin(), order.end());
        for (int i = 0; i < cnt; i++) {
            const int32_t* q = r + order[i].second * 5;
            fm_contour& o = v[i];
            o.x = q[1];
            o.y = q[2];
            o.w = q[3] - q[1] + 1;
            o.h = q[4] - q[2] + 1;
            o.origin_x = q[0] % c->w;
            o.origin_y = q[0] / c->w;
            o.area2 = -1;
            o.reserved1 = 0;
        }
    }
#ifdef FM_DEV_SWITCHES
    if (c->timer.enabled) {
        const auto hw3 = std::chrono::steady_clock::now();
        auto add = [&](const char* name, std::chrono::steady_clock::duration d) {
            const int id = c->timer.id_of(name);
            c->timer.ms[id] += std::chrono::duration<double, std::milli>(d).count();
            c->timer.launches[id] += 1;
        };
        add("host:wait_sync", hw1 - hw0);
        add("host:wait_scan", hw2 - hw1);
        add("host:wait_records", hw3 - hw2);
    }
#endif
    if (c->p.flags & FM_FLAG_CONTOUR_AREA)
        if (int rc = contour_areas(c, B, F)) return rc;
    c->ready = n;
    c->ready_slot = si;
    c->ready_gen = B.gen;
    B.n = 0;
    return FM_OK;
}

int fm_last_fallbacks(const fm_ctx* c) { return c ? c->fallbacks : fail(nullptr, FM_EINVAL, "null context"); }

int fm_last_ccl_stats(const fm_ctx* c, int32_t* shared_nodes, int32_t* heavy_tiles) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (shared_nodes) *shared_nodes = c->stats[0];
    if (heavy_tiles) *heavy_tiles = c->stats[1];
    return FM_OK;
}

int fm_get_counts(fm_ctx* c, int32_t* counts) {
    if (!c || !counts) return fail(c, FM_EINVAL, "null argument");
    std::memcpy(counts, c->ready_counts.data(), c->ready_counts.size() * sizeof(int32_t));
    return FM_OK;
}

int fm_get_contours(fm_ctx* c, int frame, int stream, fm_contour* out, int cap) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (int rc = check_frame(c, frame, stream, false)) return rc;
    const size_t f = (size_t)frame * c->p.n_streams + stream;
    const auto& v = c->contours[f];
    const int m = out ? std::min<int>(cap, (int)v.size()) : 0;
    for (int i = 0; i < m; i++) out[i] = v[i];
    return c->ready_counts[f];
}

int fm_read_mask(fm_ctx* c, int frame, int stream, uint8_t* out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    if (int rc = check_frame(c, frame, stream, true)) return rc;
    HIP_TRY(c, hipSetDevice(c->p.device));
    const size_t f = (size_t)frame * c->p.n_streams + stream;
    hipStream_t st = c->aux_stream;
    if (c->use_fused) {
        const BatchSlot& B = c->slots[c->ready_slot];
        HIP_TRY(c, launch_expand_bits(st, B.d_dbits + f * c->ntiles * 64, B.d_candf + f * c->ntiles, c->d_mask, c->h, c->w,
                                      c->ntx));
        HIP_TRY(c, hipMemcpyAsync(out, c->d_mask, c->work_plane, hipMemcpyDeviceToHost, st));
    } else {
        HIP_TRY(c, hipMemcpyAsync(out, c->d_mask + f * c->work_plane, c->work_plane, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(c, hipStreamSynchronize(st));
    return FM_OK;
}

int fm_read_plane(fm_ctx* c, int plane, int frame, int stream, uint8_t* out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    if (plane < 0 || plane > FM_PLANE_SMALL) return fail(c, FM_EINVAL, "plane %d", plane);
    if (plane == FM_PLANE_SMALL && c->rmode == ResizeMode::Identity)
        return fail(c, FM_ESTATE, "no resize (box_size = frame width): the frame is the work image");
    if (plane != FM_PLANE_SMALL && !(c->p.flags & FM_FLAG_KEEP_PLANES))
        return fail(c, FM_ESTATE, "planes not kept: create with FM_FLAG_KEEP_PLANES");
    if (int rc = check_frame(c, frame, stream, true)) return rc;
    HIP_TRY(c, hipSetDevice(c->p.device));
    const BatchSlot& B = c->slots[c->ready_slot];
    const size_t f = (size_t)frame * c->p.n_streams + stream;
    if (plane == FM_PLANE_SMALL) {  // the INTER_AREA output, [T][S][h][w][3]
        HIP_TRY(c, hipMemcpyAsync(out, B.d_work + f * c->work_plane * 3, c->work_plane * 3, hipMemcpyDeviceToHost,
                                  c->aux_stream));
        HIP_TRY(c, hipStreamSynchronize(c->aux_stream));
        return FM_OK;
    }
    const size_t Fcur = (size_t)c->ready * c->p.n_streams;
    HIP_TRY(c, hipMemcpyAsync(out, B.d_planes + ((size_t)plane * Fcur + f) * c->work_plane, c->work_plane,
                              hipMemcpyDeviceToHost, c->aux_stream));
    HIP_TRY(c, hipStreamSynchronize(c->aux_stream));
    return FM_OK;
}

int fm_read_frame(fm_ctx* c, int frame, int stream, uint8_t* out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    if (int rc = check_frame(c, frame, stream, true)) return rc;
    const BatchSlot& B = c->slots[c->ready_slot];
    if (!B.src) return fail(c, FM_ESTATE, "no source frames for the last waited batch");
    HIP_TRY(c, hipSetDevice(c->p.device));
    HIP_TRY(c, hipMemcpyAsync(out, B.src + ((size_t)frame * c->p.n_streams + stream) * c->src_frame_bytes,
                              c->src_frame_bytes, hipMemcpyDeviceToHost, c->aux_stream));
    HIP_TRY(c, hipStreamSynchronize(c->aux_stream));
    return FM_OK;
}

int fm_frame_device(fm_ctx* c, int frame, int stream, const uint8_t** out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    if (int rc = check_frame(c, frame, stream, true)) return rc;
    const BatchSlot& B = c->slots[c->ready_slot];
    if (!B.src) return fail(c, FM_ESTATE, "no source frames for the last waited batch");
    *out = B.src + ((size_t)frame * c->p.n_streams + stream) * c->src_frame_bytes;
    return FM_OK;
}

int fm_read_background(fm_ctx* c, int stream, double* out) {
    if (!c || !out) return fail(c, FM_EINVAL, "null argument");
    if (int rc = check_idle(c)) return rc;
    if (stream < 0 || stream >= c->p.n_streams) return fail(c, FM_EINVAL, "stream %d out of range", stream);
    if (!c->bg_init[stream]) return fail(c, FM_ESTATE, "stream %d has no background yet", stream);
    HIP_TRY(c, hipSetDevice(c->p.device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpyAsync(out, c->d_bg[c->bg_cur] + (size_t)stream * c->work_plane, c->work_plane * sizeof(double),
                              hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return FM_OK;
}

int fm_write_background(fm_ctx* c, int stream, const double* in) {
    if (!c || !in) return fail(c, FM_EINVAL, "null argument");
    if (int rc = check_idle(c)) return rc;
    if (stream < 0 || stream >= c->p.n_streams) return fail(c, FM_EINVAL, "stream %d out of range", stream);
    HIP_TRY(c, hipSetDevice(c->p.device));
    HIP_TRY(c, hipMemcpyAsync(c->d_bg[c->bg_cur] + (size_t)stream * c->work_plane, in, c->work_plane * sizeof(double),
                              hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->bg_init[stream] = 1;
    return FM_OK;
}

int fm_kernel_times(fm_ctx* c, const char** names, double* ms, int64_t* launches, int cap) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    HIP_TRY(c, hipSetDevice(c->p.device));
    if (c->timer.fold_stamps() != 0) return fail(c, FM_EHIP, "reading the launch stamps failed");
    const int n = (int)c->timer.names.size();
    for (int i = 0; i < std::min(n, cap); i++) {
        if (names) names[i] = c->timer.names[i];
        if (ms) ms[i] = c->timer.ms[i];
        if (launches) launches[i] = c->timer.launches[i];
    }
    return n;
}

int fm_kernel_time_spread(fm_ctx* c, double* ms_sq, int cap) {
    if (!c || !ms_sq) return fail(c, FM_EINVAL, "null argument");
    HIP_TRY(c, hipSetDevice(c->p.device));
    if (c->timer.fold_stamps() != 0) return fail(c, FM_EHIP, "reading the launch stamps failed");
    const int n = (int)c->timer.names.size();
    for (int i = 0; i < std::min(n, cap); i++) ms_sq[i] = c->timer.ms_sq[i];
    return n;
}

int fm_kernel_time_busy(fm_ctx* c, double* busy_ms, int cap) {
    if (!c || !busy_ms) return fail(c, FM_EINVAL, "null argument");
    HIP_TRY(c, hipSetDevice(c->p.device));
    if (c->timer.fold_stamps() != 0) return fail(c, FM_EHIP, "reading the launch stamps failed");
    const int n = (int)c->timer.names.size();
    for (int i = 0; i < std::min(n, cap); i++) {
        const auto& b = c->timer.busy[i];
        busy_ms[i] = b.ms + (b.open ? (double)(b.e - b.s) * 1e-5 : 0.0);
    }
    return n;
}

int fm_kernel_time_stats(fm_ctx* c, const char** names, double* ms, int64_t* launches, double* stamped_ms,
                         int64_t* stamped, double* ms_sq, double* busy_ms, int64_t* unstamped, int cap) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    HIP_TRY(c, hipSetDevice(c->p.device));
    if (c->timer.fold_stamps() != 0) return fail(c, FM_EHIP, "reading the launch stamps failed");
    const auto& T = c->timer;
    const int n = (int)T.names.size();
    for (int i = 0; i < std::min(n, cap); i++) {
        if (names) names[i] = T.names[i];
        if (ms) ms[i] = T.ms[i];
        if (launches) launches[i] = T.launches[i];
        if (ms_sq) ms_sq[i] = T.ms_sq[i];
        if (stamped) stamped[i] = T.stamped[i];
        if (stamped_ms) stamped_ms[i] = T.stamped_ms[i];
        if (busy_ms) busy_ms[i] = T.busy[i].ms + (T.busy[i].open ? (double)(T.busy[i].e - T.busy[i].s) * 1e-5 : 0.0);
    }
    if (unstamped) *unstamped = T.unstamped;
    return n;
}

int fm_reset_kernel_times(fm_ctx* c) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    HIP_TRY(c, hipSetDevice(c->p.device));
    c->timer.reset();
    return FM_OK;
}

}  // extern "C"

int fm_footprint(const fm_ctx* c, size_t* device_bytes, size_t* pinned_bytes) {
    if (!c) return fail(nullptr, FM_EINVAL, "null context");
    if (device_bytes) *device_bytes = c->dev_bytes;
    if (pinned_bytes) *pinned_bytes = c->pinned_bytes;
    return FM_OK;
}
