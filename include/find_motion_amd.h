/*
 * find_motion_amd.h — C ABI of the MI355X motion-detection hot path.
 *
 * The reference (dmiruke/find_motion, find_motion/find_motion.py = "fm.py")
 * has no FFI: its hot path is a chain of cv2 calls made from three
 * VideoMotion methods in the frame loop (fm.py:866-868):
 *
 *   blur_frame()      fm.py:487-494  imutils.resize -> cvtColor -> GaussianBlur
 *   mask_off_areas()  fm.py:619-636  rectangle / fillConvexPoly onto frame.blur
 *   find_diff()       fm.py:638-662  convertScaleAbs+absdiff, threshold,
 *                                    accumulateWeighted, dilate, findContours
 *
 * This header is the boundary a binding (ctypes / cffi / pybind11) would bind
 * to replace those three methods; find_motion_amd/motion.py is that binding.
 * Every entry point is a plain C function over plain pointers and sizes.
 * Status codes: 0 = OK, negative = error (see FM_E*); fm_last_error() gives
 * the message.  No C++ exception crosses this boundary.
 *
 * Threading: one fm_ctx per host thread; contexts are independent and bound
 * to one HIP device (one process per GPU in the multi-GPU runner).
 */
#ifndef FIND_MOTION_AMD_H
#define FIND_MOTION_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FM_ABI_VERSION 1

/* status codes */
#define FM_OK 0
#define FM_EINVAL -1   /* bad argument */
#define FM_EHIP -2     /* HIP runtime error */
#define FM_ENOMEM -3   /* allocation failed */
#define FM_ESTATE -4   /* call out of order (e.g. results before fm_wait) */
#define FM_ENOTSUP -5  /* configuration outside the restated OpenCV path */

/* fm_params.flags */
#define FM_FLAG_KEEP_PLANES 0x1u /* keep gray/blur/frame_delta per frame (show/debug, fm.py:907-926) */
#define FM_FLAG_PROFILE 0x2u     /* time every kernel launch with HIP events */
#define FM_FLAG_PROFILE_PIX 0x4u /* time only the pixel-stream kernels (cheap enough for the bench's timed loop) */
#define FM_FLAG_CONTOUR_AREA 0x8u /* trace every external contour's border on the GPU at fm_wait and return
                                     2 x cv2.contourArea (fm.py:679) in fm_contour.area2: needed only where
                                     the area filter of fm.py:684 is live (max_area < min_area) */

/* planes for fm_read_plane */
#define FM_PLANE_GRAY 0  /* VideoFrame.gray        (fm.py:493) */
#define FM_PLANE_BLUR 1  /* VideoFrame.blur, masked (fm.py:494, 619-636) */
#define FM_PLANE_DELTA 2 /* VideoFrame.frame_delta (fm.py:250) */
#define FM_PLANE_SMALL 3 /* the INTER_AREA-resized BGR frame `small` (fm.py:490), h*w*3 bytes; resize modes only,
                            no FM_FLAG_KEEP_PLANES needed */

typedef struct fm_ctx fm_ctx;

/* Construction parameters: the VideoMotion constructor arguments that reach
 * the hot path (fm.py:299-307) plus the batch geometry. */
typedef struct fm_params {
    int device;       /* HIP device ordinal */
    int n_streams;    /* independent videos/cameras, one background model each */
    int src_w, src_h; /* decoded frame size (fm.py:433-435) */
    int box_size;     /* -B / box_size: processing width (fm.py:492, 1474) */
    int ksize;        /* odd Gaussian size from _make_gaussian (fm.py:478-484) */
    int threshold;    /* -t / threshold (fm.py:256, 1476) */
    double avg;       /* -a / avg, accumulateWeighted alpha (fm.py:659, 1479) */
    int max_batch;    /* max frames per stream per fm_submit */
    int max_contours; /* per-frame contour records kept in mapped host memory (a frame
                         with more is fetched whole at fm_wait: no contour is lost) */
    unsigned flags;   /* FM_FLAG_* */
} fm_params;

/* One external contour (an element of VideoFrame.contours, fm.py:269-276). */
typedef struct fm_contour {
    int32_t x, y, w, h;          /* cv2.boundingRect (fm.py:792) */
    int32_t origin_x, origin_y;  /* border start = raster-first pixel of the component */
    int32_t area2;               /* 2 x cv2.contourArea of the CHAIN_APPROX_SIMPLE contour (an integer: the
                                    shoelace sum); -1 unless the context has FM_FLAG_CONTOUR_AREA */
    int32_t reserved1;
} fm_contour;

/* Library version (FM_ABI_VERSION) */
int fm_abi_version(void);

/* Create / destroy a context.  Allocates all device state. */
int fm_create(fm_ctx** out, const fm_params* params);
void fm_destroy(fm_ctx* ctx);

/* Last error message for ctx (or the calling thread's last error if ctx is NULL). */
const char* fm_last_error(const fm_ctx* ctx);

/* Working image size (h = int(src_h * box/src_w), w = box; imutils rule, fm.py:492). */
int fm_work_size(const fm_ctx* ctx, int* h, int* w);

/* Static keep-mask for one stream: h*w bytes, 0 = masked off (mask_off_areas,
 * fm.py:619-636, rasterised once per video).  NULL clears the mask. */
int fm_set_mask(fm_ctx* ctx, int stream, const uint8_t* keep_hw);

/* Forget the background model: the next frame re-initialises it
 * (VideoMotion.ref_frame = None, fm.py:414, 651-652). */
int fm_reset_stream(fm_ctx* ctx, int stream);

/* Batches that may be in flight at once (fm_submit before fm_wait): the contour
 * pass of one batch overlaps the pixel kernel of the next ones. */
int fm_max_inflight(const fm_ctx* ctx);

/* Run the hot path on n_frames consecutive frames of every stream.
 * frames: BGR u8, layout [n_frames][n_streams][src_h][src_w][3], C-contiguous;
 * host memory (on_device = 0, copied with hipMemcpyAsync) or device memory
 * (on_device = 1, read in place).  Asynchronous: host buffers must stay valid
 * until fm_wait returns for this batch.  Up to fm_max_inflight() batches may be
 * submitted before waiting; fm_wait completes them in submission order. */
int fm_submit(fm_ctx* ctx, const uint8_t* frames, int n_frames, int on_device);

/* fm_submit with one frame pointer per stream, SURVEY.md §8(b)'s
 * fm_submit(ctx, const uint8_t* const* bgr, n_frames): bgr[s] holds stream s's
 * n_frames consecutive frames [n_frames][src_h][src_w][3] (e.g. what a
 * per-stream decoder wrote).  Host memory: one strided DMA per stream puts them
 * into the batch's [t][s] layout on the input stream (no gather copy on the
 * host; page-locked buffers make it asynchronous).  Device memory: read in
 * place for one stream, one strided device copy per stream otherwise.
 * Results are identical to fm_submit of the same frames gathered into
 * [n_frames][n_streams] order; the same lifetime rules apply. */
int fm_submit_streams(fm_ctx* ctx, const uint8_t* const* bgr, int n_frames, int on_device);

/* Page-locked host memory for frame batches (a decoder writes frames here): fm_submit
 * of such a buffer is a true asynchronous DMA (hipMemcpyAsync) on the context's input
 * stream, overlapped with the previous batch's kernels (north_star: "frame batches
 * pinned and hipMemcpyAsync-overlapped with compute").  Replaces nothing in the
 * reference (cap.read() returns pageable numpy frames, fm.py:501); optional. */
int fm_host_alloc(fm_ctx* ctx, size_t bytes, void** out);
int fm_host_free(fm_ctx* ctx, void* ptr);

/* Wait for the oldest batch in flight; makes its results readable (device-side
 * results -- masks, planes -- until that batch's slot is reused by a later submit). */
int fm_wait(fm_ctx* ctx);

/* External-contour counts of the last batch, layout [n_frames][n_streams]
 * (len(VideoFrame.contours), the quantity find_movement counts, fm.py:674-695). */
int fm_get_counts(fm_ctx* ctx, int32_t* counts);

/* Contours of one (frame, stream) of the last batch, in raster order of their
 * start pixels.  Returns the count (records written: min(count, cap)).  Every
 * contour is kept whatever fm_params.max_contours is (a frame with more is
 * fetched whole by fm_wait), so a second call with cap = count gets them all. */
int fm_get_contours(fm_ctx* ctx, int frame, int stream, fm_contour* out, int cap);

/* Diagnostics: frames of the last waited batch whose contours came from the
 * pixel-level fallback (the batch exhausted its contour-pass node pool). */
int fm_last_fallbacks(const fm_ctx* ctx);
/* Diagnostics of the last waited batch's contour pass: union-find nodes its frames
 * took from the shared pool (past their own quotas) and tiles labelled by the heavy
 * pass (more than 256 runs: dense speckle). */
int fm_last_ccl_stats(const fm_ctx* ctx, int32_t* shared_nodes, int32_t* heavy_tiles);

/* Dilated threshold mask (VideoFrame.thresh after find_contours, fm.py:266), h*w bytes. */
int fm_read_mask(fm_ctx* ctx, int frame, int stream, uint8_t* out);

/* gray / blur / frame_delta planes (needs FM_FLAG_KEEP_PLANES), h*w bytes; FM_PLANE_SMALL: the
 * resized BGR frame, h*w*3 bytes (FM_ESTATE when box_size = frame width). */
int fm_read_plane(fm_ctx* ctx, int plane, int frame, int stream, uint8_t* out);

/* Background model (VideoMotion.ref_frame, float64, fm.py:652, 659), h*w doubles. */
int fm_read_background(fm_ctx* ctx, int stream, double* out);
int fm_write_background(fm_ctx* ctx, int stream, const double* in);

/* Launch on the caller's HIP stream (hipStream_t) instead of the context's own
 * stream; NULL restores the context stream. */
int fm_set_hip_stream(fm_ctx* ctx, void* hip_stream);

/* Memory the context holds: device bytes (fm_create's buffers, plus input staging allocated on the
 * first host submit) and page-locked host bytes (the mapped contour records and counters).  No
 * reference counterpart (sizing for many streams per GPU). */
int fm_footprint(const fm_ctx* ctx, size_t* device_bytes, size_t* pinned_bytes);

/* FM_FLAG_PROFILE: per-kernel accumulated device time since the last reset.
 * names[i] (static strings), ms[i], launches[i] for i < returned count. */
int fm_kernel_times(fm_ctx* ctx, const char** names, double* ms, int64_t* launches, int cap);
/* The same kernels in the same order, with ms_sq[i] = the sum of the squared launch times (ms^2) of the
 * launches timed by in-kernel stamps (the pixel kernel and the INTER_AREA resize under FM_FLAG_PROFILE_PIX;
 * 0 for event-timed kernels), for the spread of the launch time across a run. */
int fm_kernel_time_spread(fm_ctx* ctx, double* ms_sq, int cap);
/* The same kernels in the same order, with busy_ms[i] = the time during which at least one of the kernel's
 * stamped launches was running (the union of their windows; less than the summed launch times when launches
 * of one kernel overlap, e.g. the resizes of consecutive batches on the two input streams). */
int fm_kernel_time_busy(fm_ctx* ctx, double* busy_ms, int cap);
/* Everything above from ONE fold of the launch stamps (so the sums, the squares and the counts cover the same
 * launches): per kernel ms and launches (stamped + event-timed), stamped_ms / stamped / ms_sq (the stamped
 * launches alone: their sum, count and sum of squares, for the spread), busy_ms; *unstamped = launches that
 * found the stamp ring full between two folds (event-timed on one launch in four, or untimed).  Any array may
 * be NULL. */
int fm_kernel_time_stats(fm_ctx* ctx, const char** names, double* ms, int64_t* launches, double* stamped_ms,
                         int64_t* stamped, double* ms_sq, double* busy_ms, int64_t* unstamped, int cap);
int fm_reset_kernel_times(fm_ctx* ctx);

/* Rasterise mask polygons to a keep-mask (mask_off_areas, fm.py:611-636):
 * each polygon's points are scaled by int(v * scale) (scale_area, fm.py:616);
 * 2 points -> filled rectangle (cv2.rectangle FILLED), >= 3 points ->
 * cv2.fillConvexPoly.  xy: all points (x0,y0,x1,y1,...), npts: points per
 * polygon.  keep (h*w) is set to 1 everywhere, then 0 inside the polygons. */
int fm_rasterize_masks(int h, int w, double scale, const int32_t* xy, const int32_t* npts,
                       int n_polys, uint8_t* keep);

/* ---- Object-ROI stage ----------------------------------
 * Replaces cv2.CascadeClassifier(path) + detectMultiScale(frame.resized,
 * scaleFactor=1.1, minNeighbors=5) at find_motion.py:396 and :722-731 for HAAR
 * cascades (find_motion_amd/cascade.py reads the XML into this description).
 * Independent of fm_ctx: one detector per cascade and device. */
typedef struct fm_haar fm_haar;
typedef struct fm_haar_desc {
    int win_w, win_h;                /* <width>, <height> */
    int n_stages, n_trees, n_nodes, n_leaves, n_features;
    const int32_t* stage_ntrees;     /* [n_stages] weak classifiers per stage */
    const float* stage_threshold;    /* [n_stages] (float)value - 1e-5f, as Data::read */
    const int32_t* tree_nodes;       /* [n_trees] internal nodes per tree */
    const int32_t* node_left;        /* [n_nodes] > 0: node of the same tree, <= 0: leaf -v */
    const int32_t* node_right;       /* [n_nodes] */
    const int32_t* node_feature;     /* [n_nodes] feature index */
    const float* node_threshold;     /* [n_nodes] */
    const float* leaves;             /* [n_leaves] = tree nodes + 1 per tree */
    const int32_t* feat_rects;       /* [n_features][3][4] x y w h */
    const float* feat_weights;       /* [n_features][3], 0 = unused third rect */
    const uint8_t* feat_tilted;      /* [n_features] or NULL */
} fm_haar_desc;

/* Validate and upload a cascade (FM_EINVAL before any HIP call when the
 * description is inconsistent).  *out is set even on failure so that
 * fm_haar_last_error can say why; release it with fm_haar_destroy. */
int fm_haar_create(int device, const fm_haar_desc* desc, fm_haar** out);
void fm_haar_destroy(fm_haar* det);
const char* fm_haar_last_error(const fm_haar* det);
int fm_haar_window(const fm_haar* det, int* w, int* h);

/* detectMultiScale over n images of one size ([n][H][W][channels] u8, BGR or
 * gray; host memory, or device memory when on_device).  max_w/max_h 0 = the
 * image size.  rects: [n][cap][4] (x, y, w, h), counts[n] = detections per
 * image (may exceed cap; only cap are written).  Synchronous. */
int fm_haar_detect(fm_haar* det, const uint8_t* images, int n, int H, int W, int channels, int on_device,
                   double scale_factor, int min_neighbors, int min_w, int min_h, int max_w, int max_h,
                   int32_t* rects, int cap, int32_t* counts);
/* find_objects (find_motion.py:703-731) on raw frames: each [H][W][3] BGR
 * frame is resized to width roi_w with INTER_AREA on the device
 * (imutils.resize: height int(H * roi_w / W), *roi_h_out), then detected as
 * fm_haar_detect with default min/max sizes.  FM_ENOTSUP when W < roi_w. */
int fm_haar_detect_frames(fm_haar* det, const uint8_t* frames, int n, int H, int W, int on_device, int roi_w,
                          double scale_factor, int min_neighbors, int32_t* rects, int cap, int32_t* counts,
                          int* roi_h_out);
/* fm_haar_detect_frames over n frames already in device memory at n separate
 * addresses (frames[i]: [H][W][3] BGR; the frame list find_objects collects
 * over many streams and batches, fm.py:703-731): the INTER_AREA resize reads
 * each frame where it lies (no gather copy) whenever the tap table has at most
 * 32 taps, and gathers the frames on the detector's stream otherwise. */
int fm_haar_detect_frame_list(fm_haar* det, const uint8_t* const* frames, int n, int H, int W, int roi_w,
                              double scale_factor, int min_neighbors, int32_t* rects, int cap, int32_t* counts,
                              int* roi_h_out);
/* fm_haar_detect_frame_list without waiting for it: the detection is queued on the detector's own
 * stream and the call returns; fm_haar_collect waits and returns its results (find_objects' detections
 * feed only the seen-objects set and the display, never the written-frame decision, fm.py:549-575, 703-731,
 * so they may be collected a batch later).  One detection in flight per detector (FM_ESTATE otherwise);
 * the frames must stay where they are until it is collected. */
int fm_haar_detect_frame_list_async(fm_haar* det, const uint8_t* const* frames, int n, int H, int W, int roi_w,
                                    double scale_factor, int min_neighbors, int* roi_h_out);
/* The results of the last detection (waits for a queued one): counts[n] (every rect) and up to cap rects
 * per image in rects[n][cap][4], as fm_haar_detect_frame_list; may be called again with a larger cap. */
int fm_haar_collect(fm_haar* det, int32_t* rects, int cap, int32_t* counts, int n);
/* The ungrouped candidates of image 0 of the last fm_haar_detect (parity
 * tests); returns their number. */
int fm_haar_candidates(const fm_haar* det, int32_t* rects, int cap);
/* Device time of the last fm_haar_detect's kernels (HIP events), ms. */
double fm_haar_last_ms(const fm_haar* det);

/* ---- Decode side: MJPEG frames decoded on the GPU ------
 * Stands in for cv2.VideoCapture.read (find_motion.py:413, :497-506) on MJPEG
 * video, where every frame is one baseline JPEG, when the caller opts in (or
 * OpenCV is absent).  The decode is libjpeg-turbo's default one: jpeg_idct_islow,
 * fancy upsampling, integer YCbCr->RGB tables, BGR u8 HWC -- bit-exact to
 * cv2.imdecode and to OpenCV's built-in MJPEG reader (CAP_OPENCV_MJPEG), NOT to
 * cv2.VideoCapture's default FFmpeg backend (libavcodec IDCT + swscale), whose
 * output can differ by a few levels; that parity is unpinned here.
 * Frames without a DHT segment (AVI1 Motion-JPEG) get the T.81 Annex K tables,
 * as libjpeg-turbo's std_huff_tables installs them.
 * Supported: 8-bit baseline / extended-sequential Huffman JPEG, grayscale or
 * YCbCr with Cb, Cr at 1x1 and Y at 1x1, 2x1 or 2x2, restart intervals
 * optional (each interval is decoded by its own lane; without them one lane
 * decodes one frame).  The host only parses marker segments and copies the
 * entropy-coded bytes (stuffing and RSTn removed); Huffman decoding, IDCT,
 * upsampling and colour conversion run on the device.  Every frame of one
 * call must share frame 0's size, sampling and Huffman tables (an MJPEG
 * stream repeats them); quantization tables may differ per frame. */
typedef struct fm_mjpeg fm_mjpeg;
/* A decoder for width x height frames, up to max_frames per call.  *out is set
 * even on failure (fm_mjpeg_last_error says why); release with fm_mjpeg_destroy. */
int fm_mjpeg_create(int device, int width, int height, int max_frames, fm_mjpeg** out);
void fm_mjpeg_destroy(fm_mjpeg* dec);
const char* fm_mjpeg_last_error(const fm_mjpeg* dec);
/* Decode n JPEGs (host memory: jpegs[i], sizes[i] bytes) into [n][H][W][3] BGR
 * frames at out: device memory when out_on_device, else host memory.
 * Synchronous.  It runs on the decoder's own streams: a device `out` must not be
 * in use by work the caller queued on other streams (as for hipMemcpy). */
int fm_mjpeg_decode(fm_mjpeg* dec, const uint8_t* const* jpegs, const size_t* sizes, int n, uint8_t* out,
                    int out_on_device);
/* Device time of the last fm_mjpeg_decode's kernels (HIP events), ms. */
double fm_mjpeg_last_ms(const fm_mjpeg* dec);
/* The frame size, device and max_frames the decoder was created with. */
int fm_mjpeg_geometry(const fm_mjpeg* dec, int* width, int* height, int* device, int* max_frames);
/* fm_submit from compressed frames: n_frames x n_streams JPEGs in [t][s]
 * order, decoded by dec (created for this context's src_w x src_h) into the
 * batch's device buffer -- on the decoder's own two streams, used in turn, so one
 * batch's Huffman pass overlaps the previous batch's IDCT / colour kernels; the
 * context's input stream waits for the decode -- then processed as
 * fm_submit (frames, n_frames, on_device = 1) would.  The host buffers may be
 * reused when the call returns.  The decode does not wait for work queued earlier on the context's
 * streams: it writes the batch slot's input buffer, which is idle by construction (fm_wait
 * synchronised the slot's previous batch before the slot is handed out again) -- a waited-for-entry
 * event would serialise consecutive calls, whose Huffman pass overlaps the previous call's IDCT and
 * colour kernels.  FM_EINVAL (nothing enqueued) when dec was
 * created for another frame size or device, or for fewer than
 * n_frames x n_streams frames per call. */
int fm_submit_jpeg(fm_ctx* ctx, fm_mjpeg* dec, const uint8_t* const* jpegs, const size_t* sizes, int n_frames);
/* Tuning of the parallel Huffman decode (no reference counterpart): every entropy-coded segment is
 * cut into chunks of chunk_bits bits, one GPU lane each, and each lane speculates its entry state
 * by decoding from spec_bits bits before its chunk (default 512 / 512).  Results are identical
 * for any values; only the speed changes. */
int fm_mjpeg_tune(fm_mjpeg* dec, int chunk_bits, int spec_bits);
/* The source frame (BGR u8 [H][W][3], cap.read()'s frame.raw, fm.py:501) of (frame, stream) of the
 * last waited batch, copied to host memory: what the host needs of a batch submitted with
 * fm_submit_jpeg only for the frames it writes (fm.py:535-546) or shows.  Valid until the next
 * fm_wait; for fm_submit(on_device = 1) the caller's buffer must still hold the frames. */
int fm_read_frame(fm_ctx* ctx, int frame, int stream, uint8_t* out);
/* The device address of that same source frame, left in HBM: what find_objects (fm.py:703-731)
 * hands to fm_haar_detect_frames(on_device = 1) so an MJPEG frame decoded on the GPU reaches the
 * cascade without a round trip through host memory.  Valid until the next fm_wait. */
int fm_frame_device(fm_ctx* ctx, int frame, int stream, const uint8_t** out);

#ifdef __cplusplus
}
#endif

#endif /* FIND_MOTION_AMD_H */
