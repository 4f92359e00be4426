// fm_jpeg.hip — the decode side of the path: MJPEG frames decoded on the GPU.
//
// The reference reads frames with cv2.VideoCapture.read (fm.py:413, 497-506).  For MJPEG video each
// frame is a baseline JPEG; this decoder reproduces libjpeg-turbo's default decode (what OpenCV and
// Pillow call) bit for bit -- pinned against Pillow's libjpeg-turbo by tests/test_jpeg_host.py (CPU
// restatement oracle/jpeg.py) and tests/test_gpu_jpeg.py (this code):
//   host    marker segments (DQT, DHT, SOF0/1, DRI, SOS) parsed per frame; the entropy-coded bytes
//           copied into one pinned buffer with byte stuffing and RSTn markers removed, one segment
//           per restart interval (the whole scan without DRI);
//   k_jpeg_huff   self-synchronizing parallel Huffman decode: each segment cut into chunks of CB bits,
//           one lane per chunk, entry states speculated and fixed up through a chained look-back
//           (see the kernel); 10-bit lookahead tables in LDS that also return the extra bits'
//           value, canonical slow path past 10 bits, DC prediction; non-zero quantized coefficients
//           stored in zigzag order into int16 [frame][comp][block][64] (zeroed by k_jpeg_idct);
//   k_jpeg_idct   8 lanes per block: dequantize + jpeg_idct_islow (jidctint.c: CONST_BITS 13,
//           PASS1_BITS 2, zero-column / zero-row shortcuts, IDCT range-limit table) into component
//           planes;
//   k_jpeg_color  one workgroup per band of 16 output rows (Y and chroma rows staged in LDS), 8 pixels
//           per thread: fancy upsampling (jdsample.c h2v1/h2v2 with the edge-replicated context rows of
//           jdmainct.c) and ycc_rgb_convert (jdcolor.c tables) -> BGR u8 HWC, the cv2.VideoCapture
//           layout, straight into the caller's frame buffer.
// Supported: 8-bit baseline / extended-sequential Huffman, grayscale or 3-component YCbCr with
// Cb, Cr at 1x1 and Y at 1x1, 2x1 or 2x2; restart intervals optional; quantization and Huffman
// tables may change from frame to frame.  Anything else: FM_ENOTSUP.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fm_internal.h"

namespace fm {
namespace jp {

constexpr int kMaxComp = 3;
constexpr int kStreamSlack = 64;          // bytes allocated past the stream buffer's length
constexpr int kSegPad = 16;               // zero bytes after each segment's data (look-ahead reads)
constexpr int kLook = 10;                 // lookahead bits of the fast Huffman table
constexpr uint32_t kFull = 1u << 5;       // fast-table flag: code and extra bits both within kLook bits

struct HuffDev {              // one table as the decoder reads it (LDS image)
    // fast table over the next kLook bits: 0 = a code longer than kLook bits; else bits 0-4 = bits
    // consumed (code + extra bits when kFull, the code alone otherwise), bits 8-15 = the symbol,
    // bits 16-31 = the extended value (HUFF_EXTEND of the extra bits; kFull only)
    uint32_t lut[1 << kLook];
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
    int bpm;                  // blocks per MCU (1 for a one-component scan)
    int8_t ucomp[10], udv[10], udh[10];  // block u of an MCU: component and offset in the MCU's block grid
    // the same per block u as bit fields the Huffman loop reads without a memory access: bit u of
    // udc / uac = the DC / AC table slot, bits 2u..2u+1 of ucomp2 = the component
    uint32_t udc, uac, ucomp2;
};

struct Seg {
    uint32_t off;             // byte offset of the segment's unstuffed data in the stream buffer
    uint32_t len;
    int32_t frame;            // frame of the call (0..n-1)
    int32_t mcu0, nmcu;       // MCUs the segment holds
};

// look-back record of a tile of 64 chunks (published by its last lane)
struct TileState {
    uint32_t flag;            // 1 once the fields below are valid
    uint32_t p;               // exit bit position of the tile's last chunk (segment-relative)
    int32_t uk;               // exit state: block u of the MCU * 64 + coefficient index k
    int32_t cnt;              // blocks started from the segment start through the tile (inclusive)
    int32_t dc[kMaxComp];     // DC predictors after the tile (sums of differences since the segment start)
    int32_t pad;
};

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// MSB-first bit reader that knows its position (bits consumed since the segment start).  The word
// after the accumulator's bits is loaded one refill ahead, so a refill does not wait on memory.
// Reads run at most 16 bytes past the last segment's padding: the stream buffer has kStreamSlack
// bytes beyond its length.
struct BitReader {
    const uint32_t* w;        // next word to fetch
    uint64_t acc;
    int nb;
    uint32_t pos;
    uint32_t nxt;
    __device__ __forceinline__ uint32_t fetch() { return *w++; }
    // start at bit p of the segment whose data begins at byte off of the stream
    __device__ __forceinline__ void init(const uint8_t* stream, uint32_t off, uint32_t p, const uint8_t* end) {
        const uint32_t b = off + (p >> 3);
        w = reinterpret_cast<const uint32_t*>(stream + (b & ~3u));
        (void)end;
        const uint32_t w0 = fetch(), w1 = fetch();
        acc = (uint64_t)bswap32(w0) << 32 | bswap32(w1);
        nxt = fetch();
        const int sk = (int)(b & 3u) * 8 + (int)(p & 7u);
        acc <<= sk;
        nb = 64 - sk;
        pos = p;
    }
    __device__ __forceinline__ void refill() {  // afterwards more than 32 bits are buffered
        if (nb <= 32) {
            acc |= (uint64_t)bswap32(nxt) << (32 - nb);
            nb += 32;
            nxt = fetch();
        }
    }
    __device__ __forceinline__ uint32_t peek(int n) const { return (uint32_t)(acc >> (64 - n)); }
    __device__ __forceinline__ void skip(int n) {
        acc <<= n;
        nb -= n;
        pos += (uint32_t)n;
    }
    __device__ __forceinline__ int get(int n) {  // n in [0, 16]
        const int v = n ? (int)peek(n) : 0;
        skip(n);
        return v;
    }
};

__device__ __forceinline__ int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

// a code longer than kLook bits (jdhuff.c jpeg_huff_decode: canonical codes by length) from the next
// 16 bits: (length << 8) | symbol; length 16 and symbol 0 when no code matches (corrupt data)
__device__ __forceinline__ int huff_slow(uint32_t c16, const HuffDev& t) {
#pragma unroll 1
    for (int l = kLook + 1; l <= 16; l++) {
        const int code = (int)(c16 >> (16 - l));
        if (code <= t.maxcode[l]) return l << 8 | t.vals[(t.valoff[l] + code) & 0xFF];
    }
    return 16 << 8;
}


__device__ __forceinline__ uint64_t pack_state(uint32_t p, int uk) { return (uint64_t)p << 32 | (uint32_t)uk; }

// Decode symbols from state (br.pos, uk) while br.pos < end.  Every symbol is one Huffman code plus
// its extra bits (jdhuff.c decode_mcu): at k == 0 the DC difference of block u, else one AC
// run/size (EOB and ZRL included); uk = u * 64 + k.
// Speculative mode (!WRITE): at the first symbol boundary at or past `mark` the state is recorded as
// the chunk's entry (p_in, uk_in) and the counters restart: cnt counts DC symbols (blocks started),
// dc[] sums the DC differences per component from there.
// WRITE: the entry is exact, cnt = blocks started before it in the segment and dc[] = the DC
// predictors; coefficients go to the lane's LDS block buffer in zigzag order and each block (or the
// part of it inside this chunk) is flushed to its place in the coefficient buffer; decoding stops
// once the segment's `total` blocks are complete.
// the coefficient block (zigzag order) of block n of segment sg
__device__ __forceinline__ int16_t* block_ptr(int16_t* coef, const JpegGeom& g, const Seg& sg, int bpm, int n) {
    const long long a = (long long)sg.mcu0 * bpm + n;
    const int m = (int)(a / bpm), uu = (int)(a - (long long)m * bpm);
    const int my = m / g.mcux, mx = m - my * g.mcux;
    const CompDev& c = g.comp[(g.ucomp2 >> (2 * uu)) & 3];
    const int by = g.interleaved ? my * c.v + g.udv[uu] : my, bx = g.interleaved ? mx * c.h + g.udh[uu] : mx;
    return coef + ((size_t)sg.frame * g.frame_blocks + c.coef0 + (long long)by * c.bw + bx) * 64;
}

// Decode symbols from state (br.pos, uk) while br.pos < end.  Every symbol is one Huffman code plus
// its extra bits (jdhuff.c decode_mcu): at k == 0 the DC difference of block u, else one AC
// run/size (EOB and ZRL included); uk = u * 64 + k.
// Speculative mode (!WRITE): at the first symbol boundary at or past `mark` the state is recorded as
// the chunk's entry (p_in, uk_in) and the counters restart: cnt counts DC symbols (blocks started),
// dc0..dc2 sum the DC differences per component from there.
// WRITE: the entry is exact, cnt = blocks started before it in the segment and dc0..dc2 = the DC
// predictors; each value is stored at its zigzag position of its block in the (zeroed) coefficient
// buffer; decoding stops once the segment's `total` blocks are complete.
// WRITE also records, per block, which 16-B pieces (8 zigzag positions each) hold a non-zero value:
// msk[block] bit r, so that k_jpeg_idct loads only those.  A block decoded whole by this lane gets a
// plain store; the parts of a block split between two chunks are ORed in atomically (k_jpeg_idct
// zeroes every mask it reads, so the OR starts from 0).
template <bool WRITE>
__device__ __forceinline__ void run_symbols(BitReader& br, int& uk, uint32_t mark, uint32_t end, const HuffDev* T, int bpm, int& cnt, int& dc0, int& dc1, int& dc2, uint32_t& p_in,
                                            int& uk_in, int total, const JpegGeom& g, const Seg& sg, int16_t* coef,
                                            uint32_t* msk) {
    int u = uk >> 6, k = uk & 63;
    bool marked = WRITE;
    // (corrupt data can give counts past the segment's blocks: nothing is stored for those)
    bool wr = WRITE && k && cnt >= 1 && cnt <= total;
    int16_t* blk = wr ? block_ptr(coef, g, sg, bpm, cnt - 1) : coef;
    uint32_t bm = 0;      // WRITE: pieces of the current block this lane stored into
    bool whole = false;   // WRITE: the current block started in this lane
    auto flush = [&](bool complete) __attribute__((always_inline)) {
        if (WRITE && wr && bm) {
            uint32_t* mp = msk + ((blk - coef) >> 6);
            if (complete && whole) *mp = bm;
            else atomicOr(mp, bm);
        }
        bm = 0;
    };
    while (true) {
        if (!WRITE && !marked && br.pos >= mark) {
            marked = true;
            p_in = br.pos;
            uk_in = u * 64 + k;
            cnt = 0;
            dc0 = dc1 = dc2 = 0;
        }
        if (br.pos >= end) break;
        if (WRITE && k == 0 && cnt >= total) break;
        br.refill();
        const bool isdc = k == 0;
        const HuffDev& t = T[isdc ? (int)((g.udc >> u) & 1) : 2 + (int)((g.uac >> u) & 1)];
        const uint32_t e = t.lut[br.peek(kLook)];
        int sym, v;
        if (e & kFull) {
            br.skip((int)(e & 31));
            sym = (int)((e >> 8) & 0xFF);
            v = (int)e >> 16;
        } else {
            if (e) {
                br.skip((int)(e & 31));
                sym = (int)((e >> 8) & 0xFF);
            } else {
                const int ls = huff_slow(br.peek(16), t);
                br.skip(ls >> 8);
                sym = ls & 0xFF;
            }
            const int sz = isdc ? min(sym, 16) : (sym & 15);
            v = extend(br.get(sz), sz);
        }
        const int r = isdc ? 0 : sym >> 4;
        const bool val = isdc || (sym & 15);
        if (isdc) {
            // three scalars and selects: an array indexed by ci would live in scratch
            const int ci = (int)((g.ucomp2 >> (2 * u)) & 3);
            const int pred = (ci == 0 ? dc0 : ci == 1 ? dc1 : dc2) + v;
            dc0 = ci == 0 ? pred : dc0;
            dc1 = ci == 1 ? pred : dc1;
            dc2 = ci == 2 ? pred : dc2;
            v = pred;
            if (WRITE) {
                wr = cnt >= 0 && cnt < total;
                blk = wr ? block_ptr(coef, g, sg, bpm, cnt) : coef;
                whole = true;
            }
            cnt++;
        }
        if (WRITE && wr && val && v) {
            const int pos = min(k + r, 63);
            blk[pos] = (int16_t)v;
            bm |= 1u << (pos >> 3);
        }
        k = (!val && r != 15) ? 64 : k + r + 1;
        if (k >= 64) {
            if (WRITE) flush(true);
            k = 0;
            u = u + 1 == bpm ? 0 : u + 1;
        }
    }
    if (WRITE) flush(false);  // a block this chunk ends inside (its rest is the next lane's)
    if (!WRITE && !marked) {  // a symbol jumped over the whole chunk: it starts (and ends) here
        p_in = br.pos;
        uk_in = u * 64 + k;
        cnt = 0;
        dc0 = dc1 = dc2 = 0;
    }
    uk = u * 64 + k;
}

constexpr int kHuffWaves = 4;

// Self-synchronizing parallel Huffman decode (Weissenberger & Schmidt's scheme for JPEG): every
// segment (a restart interval, or the whole scan) is cut into chunks of CB bits, one lane each,
// 64 chunks = one tile per wave (tiles taken in order from a counter).
//   1. speculate: decode from bit start - OV in state (u, k) = (0, 0) up to the chunk start -- Huffman
//      codes resynchronise, so the state reached there is the true one with high probability -- then
//      decode the chunk, counting blocks and summing DC differences;
//   2. fix up: a lane whose entry differs from its predecessor's exit decodes again from that exit
//      (repeated until no lane changes); the wave's first lane gets its predecessor's exit from the
//      previous tile's published record (look-back; the chain is exact from each segment's start,
//      and a tile holding a segment head publishes before it looks back, so waits stay inside one
//      segment);
//   3. a segmented scan over the wave gives each chunk its first block index and DC predictors;
//   4. decode again, storing the non-zero quantized coefficients (zigzag order) into the coefficient
//      buffer, which k_jpeg_idct leaves zeroed behind it.
__global__ __launch_bounds__(64 * kHuffWaves) void k_jpeg_huff(const uint8_t* __restrict__ stream, uint32_t stream_len,
                                                                const Seg* __restrict__ segs, int nseg,
                                                                const uint32_t* __restrict__ seg_chunk0, int chunk0,
                                                                int nchunks,
                                                                const HuffDev* __restrict__ tabs, JpegGeom g, int CB, int OV,
                                                                TileState* __restrict__ ts, uint32_t* __restrict__ tile_ctr,
                                                                int16_t* __restrict__ coef, uint32_t* __restrict__ msk,
                                                                uint64_t* __restrict__ stamps) {
    __shared__ HuffDev T[4];
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(tabs);
        uint32_t* dst = reinterpret_cast<uint32_t*>(T);
        for (int i = threadIdx.x; i < (int)(sizeof(T) / 4); i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int tile = 0;
    if (lane == 0) tile = (int)atomicAdd(tile_ctr, 1u);
    tile = __shfl(tile, 0);
    if (chunk0 + tile * 64 >= nchunks) return;  // the grid's spare waves (whole waves: no barrier follows)
    // profiling only (dev build, FM_JPEG_STAMPS): per tile, realtime at start / phase-0 end / look-back
    // seen / scan done / end, and the hardware id
    uint64_t* stp = (stamps && lane == 0) ? stamps + (size_t)tile * 6 : nullptr;
#define JP_STAMP(k) do { if (stp) stp[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
    JP_STAMP(0);
    if (stp) stp[5] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const int c = chunk0 + tile * 64 + lane;  // chunks [chunk0, nchunks) belong to this launch's segments
    const bool valid = c < nchunks;
    // the chunk's segment: last s with seg_chunk0[s] <= c
    int lo = 0, hi = nseg - 1;
    const int cc = valid ? c : nchunks - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)seg_chunk0[mid] <= cc) lo = mid; else hi = mid - 1;
    }
    const Seg sg = segs[lo];
    const int j = cc - (int)seg_chunk0[lo];
    const bool head = j == 0;
    const uint32_t nbits = sg.len * 8u;
    const uint32_t cb = (uint32_t)j * (uint32_t)CB;
    const uint32_t ce = min(cb + (uint32_t)CB, nbits);
    const uint8_t* send = stream + stream_len;
    const int bpm = g.bpm;

    // 1 + 2: speculate, then fix up until every lane's entry is its predecessor's exit
    uint64_t want = pack_state(head ? 0u : (cb > (uint32_t)OV ? cb - (uint32_t)OV : 0u), 0);
    uint32_t mark = head ? 0u : cb;
    uint64_t st_in = 0, st_out = 0, lb_state = 0;
    int cnt = 0, dc0 = 0, dc1 = 0, dc2 = 0;
    int carry_cnt = 0, cd0 = 0, cd1 = 0, cd2 = 0;
    uint32_t p_in = 0;
    int uk_in = 0;
    BitReader br;
    bool go = true;
    int phase = 0;  // 0: lane 0 as speculated; 1: lane 0 from the previous tile's record
    const bool need_lb = __shfl((int)(!head), 0) != 0;
    int ic, id0, id1, id2, f;
    auto scan = [&]() {  // segmented inclusive scan of (blocks, DC sums); f = a head at or before the lane
        ic = cnt;
        id0 = dc0;
        id1 = dc1;
        id2 = dc2;
        f = head ? 1 : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int pc = __shfl_up(ic, off), p0 = __shfl_up(id0, off), p1 = __shfl_up(id1, off),
                      p2 = __shfl_up(id2, off), pf = __shfl_up(f, off);
            if (lane >= off) {
                if (!f) {
                    ic += pc;
                    id0 += p0;
                    id1 += p1;
                    id2 += p2;
                }
                f |= pf;
            }
        }
    };
    // Publication between XCDs without an agent-scope release / acquire: those write back the
    // whole L2 of the XCD (buffer_wbl2) and invalidate it (buffer_inv) on every poll.  Instead every
    // field is a relaxed agent-scope atomic (written through to / read from the coherence point);
    // the writer waits for the fields' stores to complete before it stores the flag, the reader
    // loads the fields only after it has seen the flag.
    auto publish = [&]() {
        TileState* t = ts + tile;
        __hip_atomic_store(&t->p, (uint32_t)(st_out >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&t->uk, (int)(uint32_t)st_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&t->cnt, ic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&t->dc[0], id0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&t->dc[1], id1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&t->dc[2], id2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores above are done
        __hip_atomic_store(&t->flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    for (int it = 0; it < 256; it++) {  // each pass fixes at least the next lane: <= 2 x 64 passes
        if (go) {
            br.init(stream, sg.off, (uint32_t)(want >> 32), send);
            int uk = (int)(uint32_t)want;
            run_symbols<false>(br, uk, mark, ce, T, bpm, cnt, dc0, dc1, dc2, p_in, uk_in, 0, g, sg, coef, nullptr);
            st_in = pack_state(p_in, uk_in);
            st_out = pack_state(br.pos, uk);
        }
        uint64_t pv = __shfl_up(st_out, 1);
        if (lane == 0) pv = phase ? lb_state : st_in;
        const bool mism = valid && !head && pv != st_in;
        if (__any(mism)) {
            go = mism;
            want = pv;
            mark = (uint32_t)(pv >> 32);
            continue;
        }
        if (phase == 0) JP_STAMP(1);
        if (phase == 1 || !need_lb) break;
        // consistent with lane 0's speculation: a tile holding a segment head publishes now
        scan();
        if (lane == 63 && valid && f) publish();
        if (lane == 0) {
            const TileState* t = ts + tile - 1;
            while (__hip_atomic_load(&t->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) __builtin_amdgcn_s_sleep(1);
            JP_STAMP(2);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the field loads come after the flag's
            lb_state = pack_state(__hip_atomic_load(&t->p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                  __hip_atomic_load(&t->uk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            carry_cnt = __hip_atomic_load(&t->cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cd0 = __hip_atomic_load(&t->dc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cd1 = __hip_atomic_load(&t->dc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cd2 = __hip_atomic_load(&t->dc[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        phase = 1;
        go = false;
    }
    // 3. scan with the previous tile's totals for the lanes of lane 0's segment
    JP_STAMP(3);
    scan();
    if (need_lb) {
        carry_cnt = __shfl(carry_cnt, 0);
        cd0 = __shfl(cd0, 0);
        cd1 = __shfl(cd1, 0);
        cd2 = __shfl(cd2, 0);
        if (!f) {
            ic += carry_cnt;
            id0 += cd0;
            id1 += cd1;
            id2 += cd2;
        }
        if (lane == 63 && valid && !f) publish();
    } else if (lane == 63 && valid) {
        publish();
    }
    if (!valid) return;
    // 4. decode once more from the exact entry, writing the coefficients
    int wcnt = ic - cnt, w0 = id0 - dc0, w1 = id1 - dc1, w2 = id2 - dc2;
    br.init(stream, sg.off, p_in, send);
    int wuk = uk_in;
    run_symbols<true>(br, wuk, 0, ce, T, bpm, wcnt, w0, w1, w2, p_in, uk_in, sg.nmcu * bpm, g, sg, coef, msk);
    JP_STAMP(4);
#undef JP_STAMP
}

// jidctint.c constants (CONST_BITS 13)
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

// products by 24-bit multiplies (full rate): the operands of a valid 8-bit JPEG stay far below 2^23
// (dequantized coefficients < 2^17, pass-1 outputs < 2^21), where they equal the 32-bit products
__device__ __forceinline__ void idct1d(int v0, int v1, int v2, int v3, int v4, int v5, int v6, int v7, int (&o)[8]) {
    int z1 = __mul24(v2 + v6, F0_541);
    const int tmp2 = z1 - __mul24(v6, F1_847), tmp3 = z1 + __mul24(v2, F0_765);
    const int tmp0 = (v0 + v4) * 8192, tmp1 = (v0 - v4) * 8192;
    const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    int a0 = v7, a1 = v5, a2 = v3, a3 = v1;
    z1 = a0 + a3;
    int z2 = a1 + a2, z3 = a0 + a2, z4 = a1 + a3;
    const int z5 = __mul24(z3 + z4, F1_175);
    a0 = __mul24(a0, F0_298);
    a1 = __mul24(a1, F2_053);
    a2 = __mul24(a2, F3_072);
    a3 = __mul24(a3, F1_501);
    z1 = __mul24(z1, -F0_899);
    z2 = __mul24(z2, -F2_562);
    z3 = __mul24(z3, -F1_961) + z5;
    z4 = __mul24(z4, -F0_390) + z5;
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

// zigzag position -> natural index, 8 per lane of a block's 8-lane group (the coefficient buffer holds
// blocks in zigzag order): lane r holds positions 8r .. 8r+7
__constant__ uint2 c_zz8[8] = {{0x10080100u, 0x0A030209u}, {0x19201811u, 0x05040B12u}, {0x211A130Cu, 0x22293028u},
                               {0x060D141Bu, 0x1C150E07u}, {0x38312A23u, 0x242B3239u}, {0x170F161Du, 0x332C251Eu},
                               {0x2D343B3Au, 0x2E271F26u}, {0x363D3C35u, 0x3F3E372Fu}};

// 8 lanes per block: lane r loads zigzag positions 8r..8r+7 (16 B) and scatters them to natural order
// in LDS, runs column r of pass 1, then row r of pass 2
constexpr int kIdctGroups = 4;  // groups of 32 blocks per workgroup (their loads issued together)
// IDCT scratch of a wave's 8 blocks: row-interleaved, element (row, col) of block b at
// row * 65 + 8 * b + col, so that pass 1 (lanes = block x column) and pass 2 (lanes = block x
// row) both hit 64 distinct banks (a [block][65] layout put pass 1 on 8-way conflicts)
constexpr int kWsWave = 8 * 65;
__device__ __forceinline__ int ws_block(int lb) { return (lb >> 3) * kWsWave + (lb & 7) * 8; }

// IDCT_range_limit[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table) with x = DESCALE(v, SH): the 10 bits above the rounding point,
// sign-extended, + CENTERJSAMPLE, clamped to [0, 255] (four VALU ops instead of the table's compare chain)
template <int SH>
__device__ __forceinline__ uint32_t range_limit(int v) {
    const int x = (int)__builtin_amdgcn_sbfe(v + (1 << (SH - 1)), SH, 10) + 128;  // (int: mixed-type min/max go to f64)
    return (uint32_t)(x < 0 ? 0 : x > 255 ? 255 : x);
}

// scratch offsets of lane r's zigzag positions 8r .. 8r+7 in its block's rows
__device__ __forceinline__ void zz_offsets(int r, int (&zo)[8]) {
    const uint2 nat = c_zz8[r];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int n = (int)(((i < 4 ? nat.x : nat.y) >> (8 * (i & 3))) & 63);
        zo[i] = (n >> 3) * 65 + (n & 7);
    }
}

// a wave's LDS accesses complete in order: its 8-lane blocks need no barrier, only that the compiler
// keep the accesses in program order
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// lane r of a block's 8 lanes (one wave's): raw = the block's zigzag coefficients 8r .. 8r+7,
// qc[k] = the dequantization factor of row k, column r -> the 8 samples of row r, packed
// (jpeg_idct_islow: dequantize, columns with the all-zero-AC shortcut, rows with the zero-row shortcut)
__device__ __forceinline__ uint2 idct_lane(int* wb, int r, uint4 raw, const int (&qc)[8], const int (&zo)[8]) {
    const uint32_t w4[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 8; i++) wb[zo[i]] = (int)(int16_t)(w4[i >> 1] >> (16 * (i & 1)));
    wave_lds_order();
    int v[8];
    // |coefficient| < 2^15, factor < 2^16: 24-bit multiplies are exact
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = __mul24(wb[65 * k + r], qc[k]);
    if ((v[1] | v[2] | v[3] | v[4] | v[5] | v[6] | v[7]) == 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) wb[65 * k + r] = v[0] * 4;
    } else {
        int o[8];
        idct1d(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o);
#pragma unroll
        for (int k = 0; k < 8; k++) wb[65 * k + r] = (o[k] + (1 << 10)) >> 11;
    }
    wave_lds_order();
    int w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = wb[65 * r + k];
    wave_lds_order();  // (pass 2's reads before the block's next scatter)
    uint32_t px[8];
    if ((w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0) {
        const uint32_t d = range_limit<5>(w[0]);
#pragma unroll
        for (int k = 0; k < 8; k++) px[k] = d;
    } else {
        int o[8];
        idct1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
#pragma unroll
        for (int k = 0; k < 8; k++) px[k] = range_limit<18>(o[k]);
    }
    return make_uint2(px[0] | px[1] << 8 | px[2] << 16 | px[3] << 24, px[4] | px[5] << 8 | px[6] << 16 | px[7] << 24);
}

// nblocks blocks of the call: of each frame the blocks from number `skip` on (0: all of them; with
// k_jpeg_color<., true> decoding the Y blocks itself, the chroma blocks only)
__global__ __launch_bounds__(256) void k_jpeg_idct(int16_t* __restrict__ coef, uint32_t* __restrict__ msk,
                                                    const uint16_t* __restrict__ qt, JpegGeom g, int skip, int nblocks,
                                                    uint8_t* __restrict__ planes) {
    __shared__ int ws[4 * kWsWave];
    const int r = threadIdx.x & 7, lb = threadIdx.x >> 3;
    int* wb = ws + ws_block(lb);
    const int b0 = blockIdx.x * (32 * kIdctGroups) + lb;
    const int fbk = (int)g.frame_blocks, dbk = fbk - skip;
    int fbs[kIdctGroups];  // the call-wide block numbers
    uint32_t bm[kIdctGroups];
#pragma unroll
    for (int G = 0; G < kIdctGroups; G++) {
        const int b = b0 + 32 * G;
        const int f = b / dbk;
        fbs[G] = b < nblocks ? f * fbk + skip + (b - f * dbk) : 0;
        bm[G] = b < nblocks ? msk[fbs[G]] : 0u;
    }
    // only the 16-B pieces the Huffman pass stored into (the rest of the block is zero)
    uint4 raw[kIdctGroups];
#pragma unroll
    for (int G = 0; G < kIdctGroups; G++) {
        raw[G] = ((bm[G] >> r) & 1) ? reinterpret_cast<const uint4*>(coef + (size_t)fbs[G] * 64)[r] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int G = 0; G < kIdctGroups; G++)
        if (r == 0 && bm[G]) msk[fbs[G]] = 0u;  // for the next call's stores
    int zo[8];
    zz_offsets(r, zo);
#pragma unroll
    for (int G = 0; G < kIdctGroups; G++) {
        const bool live = b0 + 32 * G < nblocks;
        const int fb = fbs[G];
        const int frame = fb / fbk;
        const int rem = fb - frame * fbk;
        int ci = 0;
        while (ci + 1 < g.nc && rem >= (int)g.comp[ci + 1].coef0) ci++;
        const CompDev& c = g.comp[ci];
        const int ib = rem - (int)c.coef0;
        const int by = ib / c.bw, bx = ib - by * c.bw;
        const uint16_t* q = qt + ((size_t)frame * kMaxComp + ci) * 64;
        int qc[8];
#pragma unroll
        for (int k = 0; k < 8; k++) qc[k] = (int)q[8 * k + r];
        // leave the block zeroed for the next call's sparse coefficient stores (only the 16-B
        // pieces that hold something: most of a typical block is zero already)
        if ((bm[G] >> r) & 1) reinterpret_cast<uint4*>(coef + (size_t)fb * 64)[r] = make_uint4(0, 0, 0, 0);
        const uint2 px = idct_lane(wb, r, raw[G], qc, zo);
#ifndef FM_JP_ABL
#define FM_JP_ABL 0  // timing ablations only (results invalid): 1 IDCT without plane stores, 2 colour without plane
                     // loads, 4 colour without its Y blocks' IDCT, 8 colour kernel without the colour rows
#endif
        if (live && !(FM_JP_ABL & 1)) {
            const int pw = c.bw * 8;
            uint8_t* row = planes + (size_t)frame * g.frame_plane + c.plane0 + (size_t)(by * 8 + r) * pw + (size_t)bx * 8;
            reinterpret_cast<uint2*>(row)[0] = px;
        }
    }
}

__device__ __forceinline__ int clamp255(int x) { return x < 0 ? 0 : x > 255 ? 255 : x; }

__device__ __forceinline__ uint32_t ycc_bgr(int Y, int cb, int cr) {  // jdcolor.c ycc_rgb_convert, BGR
    // |cb|, |cr| <= 128 and the constants < 2^17: 24-bit multiplies (full rate, v_mul_lo_u32 is not)
    const int R = clamp255(Y + ((__mul24(91881, cr) + 32768) >> 16));
    const int G = clamp255(Y + ((__mul24(-22554, cb) + 32768 - __mul24(46802, cr)) >> 16));
    const int B = clamp255(Y + ((__mul24(116130, cb) + 32768) >> 16));
    return (uint32_t)B | (uint32_t)G << 8 | (uint32_t)R << 16;
}

// One workgroup per band of `rb` output rows (blockIdx.x) of one frame (blockIdx.y).  The band's Y
// rows and the chroma rows it needs (for h2v2 also the context rows above and below, jdsample.c
// with jdmainct.c's edge replication) are staged in LDS with 8-byte loads, all in flight together;
// then row by row each thread converts 8 consecutive pixels (chroma upsampled from LDS,
// ycc_rgb_convert) into a BGR row in LDS (two of them, alternating), stored with 16-byte stores.
// MODE: 0 grayscale, 1 per-pixel chroma (1x1 chroma, or planes too narrow for the fancy filters),
// 2 h2v1 fancy upsampling, 3 h2v2 fancy upsampling (straight-line code for the common 4:2:2 / 4:2:0).
// FUSEY: the band's Y blocks (rb a multiple of 8) are dequantized and inverse-transformed here, straight
// into the LDS rows, instead of going through the Y plane in HBM (k_jpeg_idct then does the chroma
// blocks only): the plane store and reload were a third of the decoder's device time
// FUSEY: groups of 32 Y blocks with their loads in flight together (8 groups: 96 VGPRs and spills,
// 3.0 vs 1.95 ms; loading whole blocks without the piece masks, 1.91-1.96 ms: unchanged)
constexpr int kYGroups = 4;
#ifndef FM_JP_COLOR_WPE
#define FM_JP_COLOR_WPE 5  // five workgroups per CU: the LDS bound with the scratch over the chroma rows
#endif
// ys_off: LDS bytes before the Y rows (the two BGR rows unless the stores go direct); ws_off: FUSEY's
// IDCT scratch, either in front of the Y rows or over the chroma rows (which are then staged after it)
template <int MODE, bool FUSEY>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FM_JP_COLOR_WPE))) void k_jpeg_color(
    const uint8_t* __restrict__ planes, JpegGeom g, int rb, int ys_off, int ws_off, uint8_t* __restrict__ out, int frame0,
    int16_t* __restrict__ coef, uint32_t* __restrict__ msk, const uint16_t* __restrict__ qt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int y0 = blockIdx.x * rb, frame = frame0 + blockIdx.y;
    const int y1 = min(y0 + rb, g.H);
    const uint8_t* fp = planes + (size_t)frame * g.frame_plane;
    const CompDev& cy = g.comp[0];
    const int ypw = cy.bw * 8;
    const int wr = (g.W + 7) & ~7;           // Y bytes staged per row
    const int orow_sz = (g.W * 3 + 15) & ~15;
    uint8_t* orow = lds;                     // [2][orow_sz] (and the IDCT scratch of FUSEY before them)
    uint8_t* ys = lds + ys_off;              // [rb][wr]
    uint8_t* cs = ys + rb * wr;              // [2 comps][nr][cpw]
    constexpr bool color = MODE != 0;
    int hf = 1, vf = 1, dw = 0, dh = 0, cpw = 0, r_lo = 0, nr = 0;
    if (color) {
        const CompDev& cc = g.comp[1];
        hf = g.hmax / cc.h;
        vf = g.vmax / cc.v;
        dw = (g.W * cc.h + g.hmax - 1) / g.hmax;
        dh = (g.H * cc.v + g.vmax - 1) / g.vmax;
        cpw = cc.bw * 8;
        int r_hi;
        if (vf == 2) {
            r_lo = max((y0 >> 1) - 1, 0);
            r_hi = min(((y1 - 1) >> 1) + 1, dh - 1);
        } else {
            r_lo = y0;
            r_hi = y1 - 1;
        }
        nr = r_hi - r_lo + 1;
    }
    const bool ws_over_cs = FUSEY && ws_off >= ys_off;
    auto stage = [&]() {  // Y rows (unless decoded below), then chroma rows (8-byte words)
        const int yw = wr >> 3, nyw = FUSEY ? 0 : (y1 - y0) * yw;
        const int cw = cpw >> 3, ncw = 2 * nr * cw;
        for (int i = threadIdx.x; i < nyw + ncw; i += 256) {
            uint2 v;
            uint8_t* dst;
            if (i < nyw) {
                const int r = i / yw, x8 = i - r * yw;
                v = (FM_JP_ABL & 2) ? make_uint2(i, r) : reinterpret_cast<const uint2*>(fp + cy.plane0 + (size_t)(y0 + r) * ypw)[x8];
                dst = ys + r * wr + x8 * 8;
            } else {
                const int q = i - nyw, comp = q / (nr * cw), rem = q - comp * nr * cw, r = rem / cw, x8 = rem - r * cw;
                v = (FM_JP_ABL & 2) ? make_uint2(q, r) : reinterpret_cast<const uint2*>(fp + g.comp[1 + comp].plane0 + (size_t)(r_lo + r) * cpw)[x8];
                dst = cs + (comp * nr + r) * cpw + x8 * 8;
            }
            *reinterpret_cast<uint2*>(dst) = v;
        }
    };
    if (!ws_over_cs) stage();
    if constexpr (FUSEY && !(FM_JP_ABL & 4)) {
        // Y block rows y0/8 .. (y1-1)/8, block columns 0 .. wr/8-1, as k_jpeg_idct does them (8 lanes per
        // block), four groups of 32 blocks with their loads in flight together.  The 8 lanes of a block are
        // one wave's: its scratch needs wave-level ordering only (idct_lane).
        int* ws = reinterpret_cast<int*>(lds + ws_off);  // [4][kWsWave], over rows not used yet
        const int r = threadIdx.x & 7, lb = threadIdx.x >> 3;
        const int nbx = wr >> 3, nyb = nbx * (((y1 - 1) >> 3) - (y0 >> 3) + 1);
        const int64_t blk0 = (int64_t)frame * g.frame_blocks + cy.coef0 + (int64_t)(y0 >> 3) * cy.bw;
        const uint16_t* q = qt + (size_t)frame * kMaxComp * 64;
        int qv[8], zo[8];
#pragma unroll
        for (int k = 0; k < 8; k++) qv[k] = (int)q[8 * k + r];
        zz_offsets(r, zo);
        for (int base = 0; base < nyb; base += 32 * kYGroups) {
            int64_t bk[kYGroups];
            uint32_t bm[kYGroups];
            uint4 raw[kYGroups];
#pragma unroll
            for (int G = 0; G < kYGroups; G++) {
                const int j = base + 32 * G + lb, jr = j / nbx;
                bk[G] = blk0 + (int64_t)jr * cy.bw + (j - jr * nbx);
                bm[G] = j < nyb ? msk[bk[G]] : 0u;
            }
#pragma unroll
            for (int G = 0; G < kYGroups; G++)
                raw[G] = ((bm[G] >> r) & 1) ? reinterpret_cast<const uint4*>(coef + bk[G] * 64)[r] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int G = 0; G < kYGroups; G++) {
                if (r == 0 && bm[G]) msk[bk[G]] = 0u;  // for the next call's stores
                if ((bm[G] >> r) & 1) reinterpret_cast<uint4*>(coef + bk[G] * 64)[r] = make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int G = 0; G < kYGroups; G++) {
                const int j = base + 32 * G + lb, jr = j / nbx;
                if (base + 32 * G >= nyb) break;  // uniform over the workgroup
                const uint2 px = idct_lane(ws + ws_block(lb), r, raw[G], qv, zo);
                const int yr = jr * 8 + r;  // band row (y0 is a multiple of 8)
                if (j < nyb && y0 + yr < y1)
                    *reinterpret_cast<uint2*>(ys + yr * wr + (j - jr * nbx) * 8) = px;
            }
        }
    }
    if (ws_over_cs) {
        __syncthreads();  // the scratch is read
        stage();
    }
    __syncthreads();
    const int nbytes = g.W * 3;
    // whole 8-pixel groups and 8-B aligned rows: each thread stores its 24 B itself (no LDS row; as
    // jpeg_color_direct on the host decides)
    const bool direct = (g.W & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0;
    for (int y = y0; y < ((FM_JP_ABL & 8) ? y0 : y1); y++) {
        uint8_t* ob = orow + ((y - y0) & 1) * orow_sz;
        const uint8_t* yrow = ys + (y - y0) * wr;
        const uint8_t *n0 = nullptr, *f0 = nullptr;
        if (color) {
            int rn, rf;
            if (vf == 2) {
                rn = y >> 1;
                rf = (y & 1) ? min(rn + 1, dh - 1) : max(rn - 1, 0);  // the farther context row
            } else {
                rn = rf = y;
            }
            n0 = cs + (rn - r_lo) * cpw;
            f0 = cs + (rf - r_lo) * cpw;
        }
        for (int x0 = threadIdx.x * 8; x0 < g.W; x0 += 256 * 8) {
            const uint2 yy = *reinterpret_cast<const uint2*>(yrow + x0);
            uint32_t bgr[8];
            if constexpr (MODE >= 2) {
                constexpr bool V2 = MODE == 3;
                // fancy h2v1 / h2v2 over chroma columns cx0-1 .. cx0+4, read as three LDS words per row
                const int cx0 = x0 >> 1;
                int up[2][8];
#pragma unroll
                for (int comp = 0; comp < 2; comp++) {
                    int cs[6];
#pragma unroll
                    for (int rr = 0; rr < (V2 ? 2 : 1); rr++) {
                        const uint8_t* row = (rr ? f0 : n0) + comp * nr * cpw;
                        const uint32_t a = cx0 ? *reinterpret_cast<const uint32_t*>(row + cx0 - 4) : 0u;
                        const uint32_t b = *reinterpret_cast<const uint32_t*>(row + cx0);
                        const uint32_t c = *reinterpret_cast<const uint32_t*>(row + cx0 + 4);
                        const int v6[6] = {(int)(a >> 24), (int)(b & 255), (int)((b >> 8) & 255), (int)((b >> 16) & 255),
                                           (int)(b >> 24), (int)(c & 255)};
#pragma unroll
                        for (int q = 0; q < 6; q++) {
                            if (V2) cs[q] = rr ? cs[q] + v6[q] : v6[q] * 3;  // 3 * nearer + farther
                            else if (!rr) cs[q] = v6[q];
                        }
                    }
#pragma unroll
                    for (int m = 0; m < 4; m++) {
                        const int cx = cx0 + m;
                        const int cc = cs[m + 1], cl = cs[m], cr = cs[m + 2];
                        if (V2) {
                            up[comp][2 * m] = cx == 0 ? (cc * 4 + 8) >> 4 : (cc * 3 + cl + 8) >> 4;
                            up[comp][2 * m + 1] = cx == dw - 1 ? (cc * 4 + 7) >> 4 : (cc * 3 + cr + 7) >> 4;
                        } else {
                            up[comp][2 * m] = cx == 0 ? cc : (cc * 3 + cl + 1) >> 2;
                            up[comp][2 * m + 1] = cx == dw - 1 ? cc : (cc * 3 + cr + 2) >> 2;
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int Y = (int)(((i < 4 ? yy.x : yy.y) >> (8 * (i & 3))) & 0xFF);
                    bgr[i] = ycc_bgr(Y, up[0][i] - 128, up[1][i] - 128);
                }
            } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int Y = (int)(((i < 4 ? yy.x : yy.y) >> (8 * (i & 3))) & 0xFF);
                if (!color) {
                    bgr[i] = (uint32_t)Y * 0x010101u;
                    continue;
                }
                const int x = x0 + i;
                int cbv = 0, crv = 0;
#pragma unroll
                for (int comp = 0; comp < 2; comp++) {
                    const uint8_t* n = n0 + comp * nr * cpw;
                    const uint8_t* f = f0 + comp * nr * cpw;
                    int v;
                    if (hf == 1) {
                        v = n[x];
                    } else if (dw <= 2) {
                        v = n[x >> 1];  // narrow planes are replicated (h2v1_upsample / h2v2_upsample)
                    } else if (vf == 2) {  // h2v2_fancy_upsample
                        const int cx = x >> 1;
                        const int c0 = n[cx] * 3 + f[cx];
                        if ((x & 1) == 0)
                            v = cx == 0 ? (c0 * 4 + 8) >> 4 : (c0 * 3 + n[cx - 1] * 3 + f[cx - 1] + 8) >> 4;
                        else
                            v = cx == dw - 1 ? (c0 * 4 + 7) >> 4 : (c0 * 3 + n[cx + 1] * 3 + f[cx + 1] + 7) >> 4;
                    } else {  // h2v1_fancy_upsample
                        const int cx = x >> 1;
                        if ((x & 1) == 0)
                            v = cx == 0 ? n[0] : (n[cx] * 3 + n[cx - 1] + 1) >> 2;
                        else
                            v = cx == dw - 1 ? n[cx] : (n[cx] * 3 + n[cx + 1] + 2) >> 2;
                    }
                    if (comp == 0) cbv = v - 128; else crv = v - 128;
                }
                bgr[i] = ycc_bgr(Y, cbv, crv);
            }
            }
            if (direct) {  // 24 B straight to the frame: three 8-B stores (the L2 merges the wave's 1.5 KB)
                uint2* d64 = reinterpret_cast<uint2*>(out + ((size_t)frame * g.H + y) * nbytes + (size_t)x0 * 3);
                d64[0] = make_uint2(bgr[0] | bgr[1] << 24, bgr[1] >> 8 | bgr[2] << 16);
                d64[1] = make_uint2(bgr[2] >> 16 | bgr[3] << 8, bgr[4] | bgr[5] << 24);
                d64[2] = make_uint2(bgr[5] >> 8 | bgr[6] << 16, bgr[6] >> 16 | bgr[7] << 8);
                continue;
            }
            uint8_t* dst = ob + (size_t)x0 * 3;
            if (x0 + 8 <= g.W) {  // 24 B at a 4-B aligned LDS address
                uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t* b = bgr + 4 * h;
                    d32[3 * h] = b[0] | b[1] << 24;
                    d32[3 * h + 1] = b[1] >> 8 | b[2] << 16;
                    d32[3 * h + 2] = b[2] >> 16 | b[3] << 8;
                }
            } else {
                const int nx = min(8, g.W - x0);
                for (int k = 0; k < nx; k++) {
                    dst[3 * k] = (uint8_t)bgr[k];
                    dst[3 * k + 1] = (uint8_t)(bgr[k] >> 8);
                    dst[3 * k + 2] = (uint8_t)(bgr[k] >> 16);
                }
            }
        }
        if (direct) continue;
        __syncthreads();  // (also: every thread is past its stores of the row two back, from this buffer)
        uint8_t* o = out + ((size_t)frame * g.H + y) * nbytes;
        const uintptr_t al = reinterpret_cast<uintptr_t>(o) | (uintptr_t)nbytes;
        if ((al & 15) == 0) {
            for (int i = threadIdx.x; i < nbytes / 16; i += 256)
                reinterpret_cast<uint4*>(o)[i] = reinterpret_cast<const uint4*>(ob)[i];
        } else if ((al & 3) == 0) {
            for (int i = threadIdx.x; i < nbytes / 4; i += 256)
                reinterpret_cast<uint32_t*>(o)[i] = reinterpret_cast<const uint32_t*>(ob)[i];
        } else {
            for (int i = threadIdx.x; i < nbytes; i += 256) o[i] = ob[i];
        }
    }
}

}  // namespace jp
}  // namespace fm

using namespace fm::jp;

// ---------------------------------------------------------------------------------------------
// host side

// A few persistent host threads for the per-frame parsing and unstuffing (thread start-up per call
// would cost more than the work): run(n, fn) calls fn(i) for i in [0, n), the caller included.
class FramePool {
public:
    explicit FramePool(int nthreads) {
        for (int t = 0; t < nthreads; t++) th_.emplace_back([this]() { loop(); });
    }
    ~FramePool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int n, const std::function<void(int)>& fn) {
        if (th_.empty() || n < 16) {
            for (int i = 0; i < n; i++) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            busy_ = (int)th_.size();
            gen_++;
        }
        cv_.notify_all();
        for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this]() { return busy_ == 0; });
        fn_ = nullptr;
    }

private:
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&]() { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
                n = n_;
            }
            for (int i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
            std::lock_guard<std::mutex> lk(m_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, busy_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct fm_mjpeg {
    int device = 0, W = 0, H = 0, max_frames = 0;
    FramePool* pool = nullptr;  // host threads for parsing / unstuffing
    std::string err;
    bool have_geom = false;
    JpegGeom g{};
    int tsel[kMaxComp][2] = {};      // (td, ta) of each component in the scan
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    // device buffers of one call, two sets used in turn, each with its own stream: a call's Huffman
    // pass (latency-bound, few waves) runs beside the previous call's IDCT and colour kernels
    struct DevSet {
        hipStream_t st = nullptr;
        hipEvent_t done = nullptr;         // the call's kernels are finished (the caller's stream waits for it)
        uint8_t* d_stream = nullptr;
        size_t stream_cap = 0;
        Seg* d_segs = nullptr;
        size_t segs_cap = 0;
        uint32_t* d_chunk0 = nullptr;      // [nseg + 1] first chunk of each segment
        size_t chunk0_cap = 0;
        TileState* d_ts = nullptr;         // look-back records, one per tile of 64 chunks (+ the tile counter)
        size_t ts_cap = 0;
        HuffDev* d_tabs = nullptr;         // [n_sets][4]
        size_t tabs_cap = 0;
        uint16_t* d_qt = nullptr;          // [max_frames][3][64] natural order
        int16_t* d_coef = nullptr;         // [max_frames][frame_blocks][64]
        uint32_t* d_msk = nullptr;         // [max_frames][frame_blocks]: non-zero 16-B pieces of each block
        uint8_t* d_planes = nullptr;       // [max_frames][frame_plane]
    } ds[2];
    int CB = 512, OV = 512;            // chunk and speculation lengths in bits (fm_mjpeg_tune)
    uint64_t* d_stamps = nullptr;      // dev build, FM_JPEG_STAMPS: per-tile phase stamps of k_jpeg_huff
    size_t stamps_cap = 0;
    size_t stamps_n = 0;
    uint8_t* d_out = nullptr;          // device BGR when the caller wants host output
    // pinned host staging, two sets used in turn: a call refills the set whose uploads (two calls
    // back) are done, so host parsing overlaps the previous call's transfers and kernels
    struct HostSet {
        uint8_t* stream = nullptr;
        size_t stream_cap = 0;
        Seg* segs = nullptr;
        size_t segs_cap = 0;
        uint32_t* chunk0 = nullptr;
        size_t chunk0_cap = 0;
        HuffDev* tabs = nullptr;
        size_t tabs_cap = 0;
        uint16_t* qt = nullptr;
        hipEvent_t done = nullptr;  // the set's uploads are finished
        bool used = false;
    } hs[2];
    int cur = 0;  // the next call's host and device sets
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

int pfail(std::string& err, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
}

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

// T.81 Annex K.3 Huffman tables, which libjpeg-turbo's std_huff_tables (jstdhuff.c) installs in
// table slots 0 (luminance) and 1 (chrominance) of each class that the stream leaves undefined:
// Motion-JPEG (AVI1) frames from many cameras carry no DHT at all.  The AC symbol lists are an
// irregular head followed by every remaining (run, size) symbol, size 1..10, in increasing order.
void std_huff(HuffHost& t, const uint8_t (&bits)[16], const uint8_t* head, int nhead, bool ac) {
    for (int l = 1; l <= 16; l++) t.bits[l] = bits[l - 1];
    int n = 0;
    bool used[256] = {};
    for (int k = 0; k < nhead; k++) used[t.vals[n++] = head[k]] = true;
    if (ac)
        for (int rs = 0; rs < 256; rs++)
            if ((rs & 15) >= 1 && (rs & 15) <= 10 && !used[rs]) t.vals[n++] = (uint8_t)rs;
    t.n = n;
    t.present = true;
}

void add_std_huff(ParsedJpeg& J) {
    static const uint8_t dc_bits[2][16] = {{0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0},
                                           {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0}};
    static const uint8_t ac_bits[2][16] = {{0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d},
                                           {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77}};
    static const uint8_t dc_vals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
    static const uint8_t ac_head0[40] = {0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51,
                                         0x61, 0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1,
                                         0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16};
    static const uint8_t ac_head1[43] = {0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
                                         0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
                                         0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1};
    for (int id = 0; id < 2; id++) {
        if (!J.ht[0][id].present) std_huff(J.ht[0][id], dc_bits[id], dc_vals, 12, false);
        if (!J.ht[1][id].present) std_huff(J.ht[1][id], ac_bits[id], id ? ac_head1 : ac_head0, id ? 43 : 40, true);
    }
}

int parse_jpeg(std::string& err, int idx, const uint8_t* p, size_t n, ParsedJpeg& J) {
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return pfail(err, FM_EINVAL, "frame %d: no SOI", idx);
    size_t i = 2;
    bool sof = false;
    while (i + 4 <= n) {
        if (p[i] != 0xFF) return pfail(err, FM_EINVAL, "frame %d: marker expected at byte %zu", idx, i);
        while (i < n && p[i] == 0xFF) i++;
        if (i >= n) break;
        const int m = p[i++];
        if (m == 0xD9) break;
        if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
        if (i + 2 > n) return pfail(err, FM_EINVAL, "frame %d: truncated marker", idx);
        const size_t len = ((size_t)p[i] << 8) | p[i + 1];
        if (len < 2 || i + len > n) return pfail(err, FM_EINVAL, "frame %d: bad segment length", idx);
        const uint8_t* s = p + i + 2;
        const size_t sl = len - 2;
        if (m == 0xDB) {
            size_t q = 0;
            while (q < sl) {
                const int pq = s[q] >> 4, tq = s[q] & 15;
                q++;
                if (tq > 3 || q + (pq ? 128 : 64) > sl) return pfail(err, FM_EINVAL, "frame %d: bad DQT", idx);
                for (int k = 0; k < 64; k++) J.qt[tq][kZig[k]] = pq ? (uint16_t)((s[q + 2 * k] << 8) | s[q + 2 * k + 1]) : s[q + k];
                J.qt_present[tq] = true;
                q += pq ? 128 : 64;
            }
        } else if (m == 0xC4) {
            size_t q = 0;
            while (q < sl) {
                const int tc = s[q] >> 4, th = s[q] & 15;
                if (tc > 1 || th > 3 || q + 17 > sl) return pfail(err, FM_EINVAL, "frame %d: bad DHT", idx);
                HuffHost& t = J.ht[tc][th];
                int cnt = 0;
                for (int l = 1; l <= 16; l++) {
                    t.bits[l] = s[q + l];
                    cnt += s[q + l];
                }
                if (cnt > 256 || q + 17 + cnt > sl) return pfail(err, FM_EINVAL, "frame %d: bad DHT counts", idx);
                memcpy(t.vals, s + q + 17, cnt);
                t.n = cnt;
                t.present = true;
                q += 17 + cnt;
            }
        } else if (m == 0xC0 || m == 0xC1) {
            if (sl < 6 || s[0] != 8) return pfail(err, FM_ENOTSUP, "frame %d: only 8-bit samples", idx);
            J.H = (s[1] << 8) | s[2];
            J.W = (s[3] << 8) | s[4];
            J.nc = s[5];
            if ((J.nc != 1 && J.nc != 3) || sl < 6 + 3 * (size_t)J.nc)
                return pfail(err, FM_ENOTSUP, "frame %d: %d components (1 or 3 supported)", idx, J.nc);
            for (int c = 0; c < J.nc; c++) {
                J.cid[c] = s[6 + 3 * c];
                J.ch[c] = s[7 + 3 * c] >> 4;
                J.cv[c] = s[7 + 3 * c] & 15;
                J.ctq[c] = s[8 + 3 * c] & 3;
            }
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return pfail(err, FM_ENOTSUP, "frame %d: SOF%d (progressive / lossless / arithmetic) not supported", idx,
                         m - 0xC0);
        } else if (m == 0xDD) {
            if (sl < 2) return pfail(err, FM_EINVAL, "frame %d: bad DRI", idx);
            J.dri = (s[0] << 8) | s[1];
        } else if (m == 0xDA) {
            if (!sof) return pfail(err, FM_EINVAL, "frame %d: SOS before SOF", idx);
            J.ns = s[0];
            if (J.ns != J.nc || sl < 1 + 2 * (size_t)J.ns + 3)
                return pfail(err, FM_ENOTSUP, "frame %d: non-interleaved multi-scan JPEG not supported", idx);
            for (int k = 0; k < J.ns; k++) {
                J.sid[k] = s[1 + 2 * k];
                J.std_[k] = s[2 + 2 * k] >> 4;
                J.sta[k] = s[2 + 2 * k] & 15;
            }
            J.scan_begin = i + len;
            // the scan ends at the first marker that is neither stuffing (FF 00) nor RSTn; any run of
            // 0xFF fill bytes may precede a marker (T.81 B.1.1.2) and is skipped, as libjpeg's
            // fill_bit_buffer and next_marker do (FF FF 00 is a stuffed data byte there too)
            J.scan_end = n;
            for (size_t k = J.scan_begin; k < n;) {
                const uint8_t* ff = (const uint8_t*)memchr(p + k, 0xFF, n - k);
                if (!ff) break;
                k = (size_t)(ff - p);
                size_t j = k + 1;
                while (j < n && p[j] == 0xFF) j++;
                if (j >= n) {
                    J.scan_end = k;
                    break;
                }
                if (p[j] >= 0xD0 && p[j] <= 0xD7) {
                    J.nrst++;
                } else if (p[j] != 0x00) {
                    J.scan_end = k;
                    break;
                }
                k = j + 1;
            }
            add_std_huff(J);
            return FM_OK;
        }
        i += len;
    }
    return pfail(err, FM_EINVAL, "frame %d: no scan", idx);
}

void build_table(const HuffHost& h, HuffDev& t, bool dc) {
    memset(&t, 0, sizeof t);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        t.valoff[l] = k - code;
        for (int j = 0; j < h.bits[l]; j++) {
            if (l <= kLook) {
                const int sym = h.vals[k];
                const int s = dc ? std::min(sym, 16) : (sym & 15);
                for (int sfx = 0; sfx < (1 << (kLook - l)); sfx++) {
                    const int idx = (code << (kLook - l)) | sfx;
                    uint32_t e = (uint32_t)l | (uint32_t)sym << 8;
                    if (l + s <= kLook) {
                        const int extra = s ? (sfx >> (kLook - l - s)) & ((1 << s) - 1) : 0;
                        const int v = (s && extra < (1 << (s - 1))) ? extra - (1 << s) + 1 : extra;
                        e = (uint32_t)(l + s) | kFull | (uint32_t)sym << 8 | (uint32_t)(uint16_t)(int16_t)v << 16;
                    }
                    t.lut[idx] = e;
                }
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
    g.bpm = 0;
    if (g.interleaved) {
        for (int c = 0; c < J.nc; c++)
            for (int v = 0; v < J.cv[c]; v++)
                for (int h = 0; h < J.ch[c]; h++) {
                    g.ucomp[g.bpm] = (int8_t)c;
                    g.udv[g.bpm] = (int8_t)v;
                    g.udh[g.bpm] = (int8_t)h;
                    g.bpm++;
                }
    } else {
        g.bpm = 1;
    }
    const size_t nb = (size_t)d->max_frames * blocks * 64;
    for (auto& S : d->ds) {
        JHIP(d, hipMalloc((void**)&S.d_coef, nb * sizeof(int16_t)));
        JHIP(d, hipMemsetAsync(S.d_coef, 0, nb * sizeof(int16_t), d->st));
        JHIP(d, hipMalloc((void**)&S.d_msk, (size_t)d->max_frames * blocks * sizeof(uint32_t)));
        JHIP(d, hipMemsetAsync(S.d_msk, 0, (size_t)d->max_frames * blocks * sizeof(uint32_t), d->st));
        JHIP(d, hipMalloc((void**)&S.d_planes, (size_t)d->max_frames * g.frame_plane));
        JHIP(d, hipMalloc((void**)&S.d_qt, (size_t)d->max_frames * kMaxComp * 64 * sizeof(uint16_t)));
    }
    for (auto& H : d->hs)
        JHIP(d, hipHostMalloc((void**)&H.qt, (size_t)d->max_frames * kMaxComp * 64 * sizeof(uint16_t), hipHostMallocDefault));
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
    for (auto& H : d->hs) {
        JHIP(d, hipHostMalloc((void**)&H.tabs, 4 * sizeof(HuffDev), hipHostMallocDefault));
        H.tabs_cap = 4;
        JHIP(d, hipEventCreateWithFlags(&H.done, hipEventDisableTiming));
    }
    for (auto& S : d->ds) {
        JHIP(d, hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking));
        JHIP(d, hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
    }
    d->pool = new FramePool(std::max(0, std::min(7, (int)std::thread::hardware_concurrency() - 1)));
    return FM_OK;
}

void fm_mjpeg_destroy(fm_mjpeg* d) {
    if (!d) return;
    if (d->st) (void)hipStreamSynchronize(d->st);
    for (auto& S : d->ds) {
        if (S.st) (void)hipStreamSynchronize(S.st);
        for (void* p : {(void*)S.d_stream, (void*)S.d_segs, (void*)S.d_tabs, (void*)S.d_qt, (void*)S.d_coef, (void*)S.d_msk,
                        (void*)S.d_planes, (void*)S.d_chunk0, (void*)S.d_ts})
            if (p) (void)hipFree(p);
        if (S.done) (void)hipEventDestroy(S.done);
        if (S.st) (void)hipStreamDestroy(S.st);
    }
    for (void* p : {(void*)d->d_out, (void*)d->d_stamps})
        if (p) (void)hipFree(p);
    for (auto& H : d->hs) {
        for (void* p : {(void*)H.stream, (void*)H.segs, (void*)H.tabs, (void*)H.qt, (void*)H.chunk0})
            if (p) (void)hipHostFree(p);
        if (H.done) (void)hipEventDestroy(H.done);
    }
    delete d->pool;
    if (d->e0) (void)hipEventDestroy(d->e0);
    if (d->e1) (void)hipEventDestroy(d->e1);
    if (d->st) (void)hipStreamDestroy(d->st);
    delete d;
}

const char* fm_mjpeg_last_error(const fm_mjpeg* d) { return d ? d->err.c_str() : "null decoder"; }

int fm_mjpeg_tune(fm_mjpeg* d, int chunk_bits, int spec_bits) {
    if (!d) return FM_EINVAL;
    if (chunk_bits < 64 || chunk_bits > (1 << 24) || spec_bits < 0 || spec_bits > (1 << 24))
        return jfail(d, FM_EINVAL, "chunk_bits %d / spec_bits %d outside [64, 2^24] / [0, 2^24]", chunk_bits, spec_bits);
    d->CB = chunk_bits;
    d->OV = spec_bits;
    return FM_OK;
}

double fm_mjpeg_last_ms(const fm_mjpeg* d) { return d ? (double)d->last_ms : 0.0; }

int fm_mjpeg_geometry(const fm_mjpeg* d, int* width, int* height, int* device, int* max_frames) {
    if (!d) return FM_EINVAL;
    if (width) *width = d->W;
    if (height) *height = d->H;
    if (device) *device = d->device;
    if (max_frames) *max_frames = d->max_frames;
    return FM_OK;
}

}  // extern "C"

// Queue the decode of n JPEGs into n BGR frames at device address out (pitch W*3, frames
// contiguous) on stream st (the decoder's own when null).  Host work: parse, unstuff, upload.
int fm_mjpeg_enqueue(fm_mjpeg* d, const uint8_t* const* jpegs, const size_t* sizes, int n, uint8_t* out, hipStream_t st) {
    if (!d) return FM_EINVAL;
    if (!jpegs || !sizes || !out || n < 1 || n > d->max_frames)
        return jfail(d, FM_EINVAL, "n %d outside [1, max_frames=%d] or null buffers", n, d->max_frames);
    if (!d->pool) return jfail(d, FM_ESTATE, "decoder not initialised (fm_mjpeg_create failed)");
    JHIP(d, hipSetDevice(d->device));
    // The call runs on its device set's stream (the set of the call before the previous one: stream
    // order reuses its buffers) and the caller's stream waits for it at the end; work queued on the
    // caller's stream before the call is not waited for (the output buffer must be free already).
    // The host staging set's previous uploads must be done before it is refilled.
    const hipStream_t cst = st ? st : d->st;
    auto& H = d->hs[d->cur];
    auto& S = d->ds[d->cur];
    st = S.st;
    if (H.used) JHIP(d, hipEventSynchronize(H.done));
    std::vector<ParsedJpeg> P(n);
    for (int i = 0; i < n; i++)
        if (!jpegs[i]) return jfail(d, FM_EINVAL, "frame %d: null", i);
    {   // marker parsing, frames in parallel (errors reported for the first failing frame)
        std::vector<int> prc(n, FM_OK);
        std::vector<std::string> perr(n);
        d->pool->run(n, [&](int i) { prc[i] = parse_jpeg(perr[i], i, jpegs[i], sizes[i], P[i]); });
        for (int i = 0; i < n; i++)
            if (prc[i]) return jfail(d, prc[i], "%s", perr[i].c_str());
    }
    if (!d->have_geom)
        if (int rc = setup_geometry(d, P[0])) return rc;
    const JpegGeom& g = d->g;
    // Huffman tables: per frame, each class (DC, AC) may use two distinct table ids (slots 0, 1 in
    // order of first use by the components); consecutive frames with the same slots and table
    // contents form a run, decoded by one launch of k_jpeg_huff with that run's four tables
    // (MJPEG streams normally repeat one set: one run).  Quantization tables may differ per frame.
    struct TabSet {
        int slot[kMaxComp][2];
        const HuffHost* t[2][2];
    };
    std::vector<TabSet> fsets(n);
    for (int i = 0; i < n; i++) {
        const ParsedJpeg& J = P[i];
        if (J.W != g.W || J.H != g.H) return jfail(d, FM_EINVAL, "frame %d: geometry differs", i);
        // a later frame coded with other components or sampling than the decoder's layout: FM_ENOTSUP, the
        // status on which the decode-ahead feeder decodes the batch on the host (a stream may switch)
        if (J.nc != g.nc) return jfail(d, FM_ENOTSUP, "frame %d: %d components, the decoder's layout has %d", i, J.nc, g.nc);
        TabSet& ts_ = fsets[i];
        int ids[2][2] = {{-1, -1}, {-1, -1}};
        for (int c = 0; c < g.nc; c++) {
            if (J.ch[c] != g.comp[c].h || J.cv[c] != g.comp[c].v)
                return jfail(d, FM_ENOTSUP, "frame %d: sampling differs from the decoder's layout", i);
            if (!J.qt_present[J.ctq[c]]) return jfail(d, FM_EINVAL, "frame %d: missing DQT %d", i, J.ctq[c]);
            int k = 0;
            while (k < J.ns && J.sid[k] != J.cid[c]) k++;
            if (k == J.ns) return jfail(d, FM_EINVAL, "frame %d: component %d not in the scan", i, J.cid[c]);
            for (int t = 0; t < 2; t++) {
                const int id = (t ? J.sta[k] : J.std_[k]) & 3;
                if (!J.ht[t][id].present) return jfail(d, FM_EINVAL, "frame %d: missing DHT", i);
                int sl = ids[t][0] == id ? 0 : ids[t][1] == id ? 1 : -1;
                if (sl < 0) {
                    sl = ids[t][0] < 0 ? 0 : ids[t][1] < 0 ? 1 : -1;
                    if (sl < 0) return jfail(d, FM_ENOTSUP, "frame %d: more than two %s tables in the scan", i, t ? "AC" : "DC");
                    ids[t][sl] = id;
                }
                ts_.slot[c][t] = sl;
            }
        }
        for (int t = 0; t < 2; t++)
            for (int sl = 0; sl < 2; sl++) ts_.t[t][sl] = ids[t][sl] >= 0 ? &J.ht[t][ids[t][sl]] : nullptr;
    }
    auto same_set = [&](const TabSet& x, const TabSet& y) {
        for (int c = 0; c < g.nc; c++)
            if (x.slot[c][0] != y.slot[c][0] || x.slot[c][1] != y.slot[c][1]) return false;
        for (int t = 0; t < 2; t++)
            for (int sl = 0; sl < 2; sl++) {
                const HuffHost *p = x.t[t][sl], *q = y.t[t][sl];
                if (!p != !q) return false;
                if (p && (p->n != q->n || memcmp(p->bits, q->bits, sizeof p->bits) || memcmp(p->vals, q->vals, p->n)))
                    return false;
            }
        return true;
    };
    std::vector<int> run_first;  // first frame of each run
    for (int i = 0; i < n; i++)
        if (i == 0 || !same_set(fsets[i], fsets[run_first.back()])) run_first.push_back(i);
    const int nruns = (int)run_first.size();
    if (int rc = grow_host(d, &H.tabs, H.tabs_cap, (size_t)nruns * 4)) return rc;
    for (int r = 0; r < nruns; r++) {
        const TabSet& ts_ = fsets[run_first[r]];
        for (int t = 0; t < 2; t++)
            for (int sl = 0; sl < 2; sl++) {
                HuffDev& hd = H.tabs[r * 4 + 2 * t + sl];
                if (ts_.t[t][sl]) build_table(*ts_.t[t][sl], hd, t == 0);
                else memset(&hd, 0, sizeof hd);
            }
    }
    // entropy-coded bytes: stuffing and RSTn removed, one segment per restart interval, each followed
    // by kSegPad zero bytes; frame i writes its own region of the staging buffer (bounded by its scan
    // size), frames in parallel
    std::vector<size_t> base(n + 1, 0);
    for (int i = 0; i < n; i++) base[i + 1] = base[i] + P[i].scan_end - P[i].scan_begin + kSegPad * (P[i].nrst + 1);
    if (int rc = grow_host(d, &H.stream, H.stream_cap, base[n] + 16)) return rc;
    const long long nmcu = (long long)g.mcux * g.mcuy;
    std::vector<std::vector<Seg>> fsegs(n);
    std::vector<int> frc(n, FM_OK);
    d->pool->run(n, [&](int i) {
        const ParsedJpeg& J = P[i];
        const uint8_t* s = jpegs[i];
        std::vector<Seg>& segs = fsegs[i];
        size_t w = base[i];
        const long long per = J.dri > 0 ? J.dri : nmcu;
        Seg cur{(uint32_t)w, 0, i, 0, (int32_t)std::min<long long>(per, nmcu)};
        size_t k = J.scan_begin;
        while (k < J.scan_end) {
            const uint8_t* ff = (const uint8_t*)memchr(s + k, 0xFF, J.scan_end - k);
            const size_t run = ff ? (size_t)(ff - (s + k)) : J.scan_end - k;
            memcpy(H.stream + w, s + k, run);
            w += run;
            k += run;
            if (!ff) break;
            const uint8_t nx = k + 1 < J.scan_end ? s[k + 1] : 0;
            if (nx == 0x00) {
                H.stream[w++] = 0xFF;
                k += 2;
            } else if (nx >= 0xD0 && nx <= 0xD7) {  // restart marker: the next interval starts here
                cur.len = (uint32_t)(w - cur.off);
                segs.push_back(cur);
                memset(H.stream + w, 0, kSegPad);
                w += kSegPad;
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
        memset(H.stream + w, 0, kSegPad);
        if (J.dri > 0 && (segs.empty() || (long long)(segs.back().mcu0 + segs.back().nmcu) != nmcu)) frc[i] = FM_EINVAL;
        for (int c = 0; c < g.nc; c++) memcpy(H.qt + ((size_t)i * kMaxComp + c) * 64, J.qt[J.ctq[c]], 128);
    });
    std::vector<Seg> segs;
    segs.reserve(n);
    for (int i = 0; i < n; i++) {
        if (frc[i]) return jfail(d, FM_EINVAL, "frame %d: restart markers do not cover the %lld MCUs", i, nmcu);
        segs.insert(segs.end(), fsegs[i].begin(), fsegs[i].end());
    }
    size_t w = base[n];
    memset(H.stream + w, 0, 16);
    w += 16;
    if (w >= (size_t)UINT32_MAX) return jfail(d, FM_ENOTSUP, "compressed batch too large");
    if (int rc = grow_host(d, &H.segs, H.segs_cap, segs.size())) return rc;
    memcpy(H.segs, segs.data(), segs.size() * sizeof(Seg));
    // chunks of CB bits per segment (at least one), 64 per tile
    // each run's chunks start on a tile boundary (tiles never span runs: no look-back between them)
    const int nseg = (int)segs.size();
    if (int rc = grow_host(d, &H.chunk0, H.chunk0_cap, (size_t)nseg + 1)) return rc;
    std::vector<int> run_seg(nruns + 1, nseg);        // first segment of each run
    std::vector<size_t> run_chunk(nruns + 1), run_end(nruns), run_tile(nruns + 1);
    {
        int r = 0;
        for (int i = 0; i < nseg && r < nruns; i++)
            while (r < nruns && segs[i].frame >= run_first[r]) run_seg[r++] = i;
    }
    size_t nchunks = 0, ntiles = 0;
    for (int r = 0; r < nruns; r++) {
        nchunks = (nchunks + 63) & ~(size_t)63;
        run_chunk[r] = nchunks;
        run_tile[r] = ntiles;
        for (int i = run_seg[r]; i < run_seg[r + 1]; i++) {
            H.chunk0[i] = (uint32_t)nchunks;
            nchunks += std::max<size_t>(1, ((size_t)segs[i].len * 8 + d->CB - 1) / d->CB);
        }
        run_end[r] = nchunks;
        ntiles += (nchunks - run_chunk[r] + 63) / 64;
    }
    run_chunk[nruns] = nchunks;
    run_tile[nruns] = ntiles;
    H.chunk0[nseg] = (uint32_t)nchunks;
    if (nchunks >= (size_t)INT32_MAX / 2) return jfail(d, FM_ENOTSUP, "compressed batch too large");
    if (int rc = grow_dev(d, &S.d_stream, S.stream_cap, w + kStreamSlack)) return rc;  // look-ahead reads
    if (int rc = grow_dev(d, &S.d_segs, S.segs_cap, segs.size())) return rc;
    if (int rc = grow_dev(d, &S.d_chunk0, S.chunk0_cap, (size_t)nseg + 1)) return rc;
    if (int rc = grow_dev(d, &S.d_ts, S.ts_cap, ntiles + nruns)) return rc;  // + one tile counter per run
#ifdef FM_DEV_SWITCHES
    if (getenv("FM_JPEG_STAMPS")) {
        if (int rc = grow_dev(d, &d->d_stamps, d->stamps_cap, ntiles * 6)) return rc;
        d->stamps_n = ntiles;
        JHIP(d, hipMemsetAsync(d->d_stamps, 0, ntiles * 6 * sizeof(uint64_t), st));
    }
#endif
    if (int rc = grow_dev(d, &S.d_tabs, S.tabs_cap, (size_t)nruns * 4)) return rc;
    JHIP(d, hipMemcpyAsync(S.d_stream, H.stream, w, hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(S.d_segs, H.segs, segs.size() * sizeof(Seg), hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(S.d_chunk0, H.chunk0, ((size_t)nseg + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    JHIP(d, hipMemsetAsync(S.d_ts, 0, (ntiles + nruns) * sizeof(TileState), st));  // flags + the tile counters
    JHIP(d, hipMemcpyAsync(S.d_tabs, H.tabs, (size_t)nruns * 4 * sizeof(HuffDev), hipMemcpyHostToDevice, st));
    JHIP(d, hipMemcpyAsync(S.d_qt, H.qt, (size_t)n * kMaxComp * 64 * sizeof(uint16_t), hipMemcpyHostToDevice, st));
    JHIP(d, hipEventRecord(H.done, st));
    H.used = true;
    d->cur ^= 1;
    if (d->timing) JHIP(d, hipEventRecord(d->e0, st));
    for (int r = 0; r < nruns; r++) {
        const int nt = (int)(run_tile[r + 1] - run_tile[r]);
        if (nt == 0) continue;
        JpegGeom gr = d->g;  // this run's table slots
        for (int c = 0; c < g.nc; c++) {
            gr.comp[c].dc = fsets[run_first[r]].slot[c][0];
            gr.comp[c].ac = 2 + fsets[run_first[r]].slot[c][1];
        }
        gr.udc = gr.uac = gr.ucomp2 = 0;
        for (int u = 0; u < gr.bpm; u++) {
            const int c = gr.ucomp[u];
            gr.udc |= (uint32_t)gr.comp[c].dc << u;
            gr.uac |= (uint32_t)(gr.comp[c].ac - 2) << u;
            gr.ucomp2 |= (uint32_t)c << (2 * u);
        }
        hipLaunchKernelGGL(k_jpeg_huff, dim3((unsigned)((nt + kHuffWaves - 1) / kHuffWaves)), dim3(64 * kHuffWaves), 0, st,
                           S.d_stream, (uint32_t)w, S.d_segs + run_seg[r], run_seg[r + 1] - run_seg[r],
                           S.d_chunk0 + run_seg[r], (int)run_chunk[r], (int)run_end[r], S.d_tabs + 4 * r, gr,
                           d->CB, d->OV, S.d_ts + run_tile[r], reinterpret_cast<uint32_t*>(S.d_ts + ntiles + r),
                           S.d_coef, S.d_msk, d->d_stamps ? d->d_stamps + 6 * run_tile[r] : nullptr);
    }
    JHIP(d, hipGetLastError());
    const long long nb = (long long)n * g.frame_blocks;
    if (nb >= INT32_MAX / 2) return jfail(d, FM_ENOTSUP, "too many coefficient blocks in one call");
    // colour bands: as many rows as keep the staging within 48 KB of LDS
#ifndef FM_JP_FUSEY
#define FM_JP_FUSEY 1
#endif
#ifndef FM_JP_WSCS
#define FM_JP_WSCS 1
#endif
    const bool direct = (g.W & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0;
    int rb = 16;
    size_t lds = 0, ys_off = 0, ws_off = 0;
    for (;; rb >>= 1) {
        const size_t orow = ((size_t)g.W * 3 + 15) & ~(size_t)15, wr = ((size_t)g.W + 7) & ~(size_t)7;
        size_t nr = 0;
        if (g.nc == 3) nr = g.vmax / g.comp[1].v == 2 ? (size_t)rb / 2 + 3 : (size_t)rb;
        const size_t wsz = FM_JP_FUSEY && rb >= 8 ? 4 * kWsWave * 4 : 0, front = direct ? 0 : 2 * orow;
        const size_t csz = g.nc == 3 ? 2 * nr * (size_t)g.comp[1].bw * 8 + 16 : 0;  // + word look-ahead
        if (wsz && FM_JP_WSCS != 0) {  // the scratch over the chroma rows
            ys_off = front;
            ws_off = ys_off + rb * wr;
            lds = ws_off + std::max(csz, wsz);
        } else {
            ys_off = std::max(front, wsz);
            ws_off = 0;
            lds = ys_off + rb * wr + csz;
        }
        if (lds <= 48 * 1024 || rb == 1) break;
    }
    if (lds > 64 * 1024) return jfail(d, FM_ENOTSUP, "frame width %d too large for the colour kernel", g.W);
    int mode = 0;
    if (g.nc == 3) {
        const int hf = g.hmax / g.comp[1].h, vf = g.vmax / g.comp[1].v;
        const int dw = (g.W * g.comp[1].h + g.hmax - 1) / g.hmax;
        mode = (hf == 2 && dw > 2) ? (vf == 2 ? 3 : 2) : 1;
    }
    // the Y blocks decoded inside the colour kernel when its bands are whole block rows
    const bool fuse = FM_JP_FUSEY && rb >= 8 && g.comp[0].coef0 == 0;
    const int skip = fuse ? (g.nc > 1 ? (int)g.comp[1].coef0 : (int)g.frame_blocks) : 0;
    const long long nbi = (long long)n * ((long long)g.frame_blocks - skip);
    if (nbi > 0)
        hipLaunchKernelGGL(k_jpeg_idct, dim3((unsigned)((nbi + 32 * kIdctGroups - 1) / (32 * kIdctGroups))), dim3(256), 0, st,
                           S.d_coef, S.d_msk, S.d_qt, d->g, skip, (int)nbi, S.d_planes);
    {
        const dim3 cgrid((unsigned)((g.H + rb - 1) / rb), (unsigned)n);
#define FM_JP_COLOR(M, F) \
    hipLaunchKernelGGL((k_jpeg_color<M, F>), cgrid, dim3(256), lds, st, S.d_planes, d->g, rb, (int)ys_off, (int)ws_off, out, 0, S.d_coef, S.d_msk, S.d_qt)
        if (fuse) {
            if (mode == 3) FM_JP_COLOR(3, true);
            else if (mode == 2) FM_JP_COLOR(2, true);
            else if (mode == 1) FM_JP_COLOR(1, true);
            else FM_JP_COLOR(0, true);
        } else {
            if (mode == 3) FM_JP_COLOR(3, false);
            else if (mode == 2) FM_JP_COLOR(2, false);
            else if (mode == 1) FM_JP_COLOR(1, false);
            else FM_JP_COLOR(0, false);
        }
#undef FM_JP_COLOR
    }
    JHIP(d, hipGetLastError());
    if (d->timing) JHIP(d, hipEventRecord(d->e1, st));
    JHIP(d, hipEventRecord(S.done, st));
    JHIP(d, hipStreamWaitEvent(cst, S.done, 0));
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
#ifdef FM_DEV_SWITCHES
    if (const char* path = getenv("FM_JPEG_STAMPS")) {
        std::vector<uint64_t> h(d->stamps_n * 6);
        JHIP(d, hipMemcpy(h.data(), d->d_stamps, h.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* fp = fopen(path, "wb")) {
            fwrite(h.data(), 8, h.size(), fp);
            fclose(fp);
        }
    }
#endif
    return FM_OK;
}

}  // extern "C"
