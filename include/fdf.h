/*
 * fdf.h -- C ABI of the MI355X (gfx950) FAST-9..16 corner detector.
 *
 * Drop-in boundary for the reference's hot path `fast_simd::detector`
 * (iwanders/feature_detector_fast src/fast_simd.rs:847-859), which the crate API calls from
 * `Config::detect` (src/lib.rs:56-58) and `detect` (src/lib.rs:62-64).  Every entry point
 * below names the reference interface it replaces.  A Rust shim that binds these symbols
 * is shown in INTEGRATION.md; the C++ mirror of the crate API is include/fdf.hpp.
 *
 * Semantics are the reference's, bit for bit (SURVEY.md §7 "semantic contract"):
 *   - centres x in [3, w-3), y in [3, h-3); circle order of src/fast_simd.rs:79-98;
 *   - bright <=> p > c + t, dark <=> p < c - t (strict, integer);
 *   - keypoint <=> a cyclic run of >= n bright or >= n dark circle pixels (9 <= n <= 16);
 *   - NMS (MaxThreshold / SumAbsolute): keep iff y not in {3, h-4} and the score is strictly
 *     greater than every 8-neighbour that is itself a keypoint (src/fast_simd.rs:589-616);
 *   - output: points in raster order (y ascending, then x).
 * Where the reference panics, these functions return an error code and never abort.
 *
 * Ownership: the caller owns every input and output buffer.  The library owns device
 * workspace inside an opaque context, reused across calls.  No global mutable state.
 * Threading: a context serialises its own host calls; distinct contexts may be used
 * concurrently from different threads.  One context = one device + one HIP stream.
 */
#ifndef FDF_H
#define FDF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDF_ABI_VERSION 6

/* Status codes.  Shapes the reference maps to an empty Vec return FDF_OK with 0 points. */
enum fdf_status {
    FDF_OK = 0,
    FDF_ERR_COUNT = 1,     /* count n outside [9, 16]: src/fast_simd.rs:302-305 (n<9), :800 (n>16) */
    FDF_ERR_SIZE = 2,      /* h < 3, or h >= 7 with w < 6: the u32 underflows at :342 / :369 */
    FDF_ERR_CAPACITY = 3,  /* output buffer too small; *n_out holds the required point count */
    FDF_ERR_NMS = 4,       /* non_maximal_supression value not 0, 1 or 2 */
    FDF_ERR_DEVICE = 5,    /* HIP runtime failure (no device, launch or copy error) */
    FDF_ERR_ARG = 6,       /* NULL pointer, stride < width, or a size that overflows */
    FDF_ERR_ALLOC = 7,     /* device or pinned host allocation failed */
    FDF_ERR_BUSY = 8,      /* pipeline: the ticket's slot still holds uncollected results */
    FDF_ERR_DROPPED = 9    /* pipeline: a batch found more keypoints than its device capacity */
};

/* src/lib.rs:26-36 NonMaximalSuppression {Off, MaxThreshold, SumAbsolute}. */
enum fdf_nms {
    FDF_NMS_OFF = 0,
    FDF_NMS_MAX_THRESHOLD = 1,
    FDF_NMS_SUM_ABSOLUTE = 2
};

/* src/lib.rs:40-52 Config {threshold: u8, count: u8, non_maximal_supression}. */
typedef struct fdf_config {
    uint8_t threshold;
    uint8_t count;
    uint8_t nms; /* enum fdf_nms */
} fdf_config;

/* src/lib.rs:17-20 Point {x: u32, y: u32}, laid out as #[repr(C)]. */
typedef struct fdf_point {
    uint32_t x;
    uint32_t y;
} fdf_point;

typedef struct fdf_ctx fdf_ctx;

/* Library/ABI identification. */
int fdf_abi_version(void);
const char* fdf_status_string(int status);
/* Number of visible HIP devices (0 when none); never fails. */
int fdf_device_count(void);

/* Validate a configuration and image shape without touching a device.  Returns FDF_OK and
 * sets *empty = 1 for the shapes the reference answers with an empty Vec (3 <= h <= 6, or
 * h >= 7 with w == 6); otherwise the error the reference would panic with. */
int fdf_validate(uint32_t width, uint32_t height, const fdf_config* cfg, int* empty);

/* Context: binds a device and creates a non-blocking HIP stream owned by the context. */
int fdf_ctx_create(int device, fdf_ctx** out_ctx);
void fdf_ctx_destroy(fdf_ctx* ctx);
/* The context's hipStream_t (as void*), for callers that enqueue their own work beside it. */
void* fdf_ctx_stream(fdf_ctx* ctx);

/* Profiling (extension, no reference counterpart): while enabled, each detect call on the
 * context (up to 4096 of them) records the durations of its two kernel launches -- the
 * detector (pre-filter, segment test, NMS, per-band slots) and the raster-order compaction
 * -- with HIP events the dispatches themselves timestamp (no packets between the kernels).
 * A call whose grid writes its points directly has no compaction launch: 0 ms.
 * enable = k > 1 records every k-th call only (the timestamped dispatches cost ~10 us each
 * on the queue, so a timed run samples).  fdf_ctx_timing waits for the recorded calls and
 * returns their number and the summed durations of both launches in ms.  Enabling resets the
 * record. */
int fdf_ctx_set_timing(fdf_ctx* ctx, int enable);
int fdf_ctx_timing(fdf_ctx* ctx, uint32_t* calls, float* detect_ms, float* compact_ms);
/* The same record per call: *n = calls recorded; the first `cap` calls' detector and
 * compaction durations (ms) go to detect_ms[k] / compact_ms[k] (for percentiles). */
int fdf_ctx_timing_samples(fdf_ctx* ctx, float* detect_ms, float* compact_ms, uint32_t cap,
                           uint32_t* n);

/* Geometry (extension; results never depend on it): the band height is chosen so that a
 * launch has at least `min_tasks` workgroups when it can (default 0 = 1024, enough for 4
 * per CU).  min_tasks = 1 makes a small job use the tall bands and long sweep units of
 * large batches -- the parity tests reach those code paths with small inputs this way. */
int fdf_ctx_set_geometry(fdf_ctx* ctx, uint32_t min_tasks);

/* Band height override: every later detection on the context sweeps bands of `rows` centre
 * rows (rounded up to the geometry's sub-band multiple, capped by what the workgroup's LDS
 * holds, 160 KB); 0 restores the automatic choice (LDS budget, grid size, and for NMS the
 * keypoint density of the previous launch).  The keypoints are the same at every height;
 * tests use it to cross the band NMS pass's LDS / spill / dense tiers.  rows > 256 (outside
 * the automatic choice's range): FDF_ERR_ARG. */
int fdf_ctx_set_band_rows(fdf_ctx* ctx, uint32_t rows);

/* How fdf_detect gets a host frame to the device (extension).  chunks = 0 (default): a
 * packed frame (stride = width) in pinned, non-coherent host memory (hipHostMalloc /
 * hipHostRegister without the coherent flag) is read in place by the detector over PCIe, no
 * copy first; any other frame is copied before the launch.  chunks = 1: always one copy.
 * chunks = k in 2..16: a frame of >= 256 KB goes up in k row chunks on a copy stream while
 * the detector already runs, each band waiting (on the device) for the chunk holding the last
 * row it reads -- on ROCm 7 each chunk's ready flag costs a small blit launch, so this
 * measured slower.  The keypoints are the same either way. */
int fdf_ctx_set_upload_chunks(fdf_ctx* ctx, uint32_t chunks);

/* Device bytes the context's workspace holds now (host-API staging and output, per-band
 * slots and counts, compaction sums).  Slots take 1/8 byte per pixel of the largest batch
 * seen; nothing in the workspace scales with more than that. */
int fdf_ctx_workspace_bytes(fdf_ctx* ctx, uint64_t* bytes);

/* Recoveries the host entry points made on their own since the context was created (ABI 6;
 * either pointer may be NULL): `upload_fallbacks` counts fdf_detect calls whose overlapped
 * upload (fdf_ctx_set_upload_chunks k > 1) had a band's chunk wait run out, so the frame was
 * detected again from one copy; `lookback_recoveries` counts host calls whose direct-output
 * look-back ran out and whose output the compaction rebuilt from the band slots.  Both stay
 * 0 in a healthy run -- tests assert it, so a handshake that never works cannot pass by its
 * fallback. */
int fdf_ctx_recoveries(fdf_ctx* ctx, uint64_t* upload_fallbacks, uint64_t* lookback_recoveries);

/* Test hook (no effect on results otherwise): moves the context's host-side count of the
 * direct-output start tickets by `delta`, as if the device counter and the host had fallen
 * out of step (after the context's first launch, which zeroes both).  The next direct-output
 * launch then hands `delta` workgroups tickets past its
 * grid; each one touches no band's memory and sets the context's device error, so that launch
 * is reported: a host call returns FDF_ERR_DEVICE, an asynchronous fdf_detect_device reports
 * it at the context's next device call, once, and the counter is re-zeroed (later calls are
 * correct).  tests/test_gpu_api.py drives it. */
int fdf_ctx_test_skew_tickets(fdf_ctx* ctx, uint32_t delta);

/*
 * Replaces fast_simd::detector(img, config) -> Vec<Point> (src/fast_simd.rs:847).
 * Host image (row-major u8, `stride_bytes` >= width; GrayImage always has stride == width),
 * host output.  Synchronous.  Two-call pattern: if `cap` is too small, returns
 * FDF_ERR_CAPACITY with *n_out = the required count and writes the first `cap` points; the
 * whole result stays on the device, and fdf_fetch_last copies it out without detecting
 * again.
 */
int fdf_detect(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
               size_t stride_bytes, const fdf_config* cfg, fdf_point* out, size_t cap,
               size_t* n_out);

/*
 * Second half of the two-call pattern: the points (frames concatenated, raster order) of
 * the last host-API detection on this context (fdf_detect, fdf_detect_rgb, fdf_detect_batch
 * and the scored variants), and their scores when `out_scores` is not NULL (the score kind
 * of that call's config, as fdf_detect_scored).  Only copies: no detection runs.
 * FDF_ERR_CAPACITY again if `cap` < *n_out; FDF_ERR_ARG if the context holds no result
 * (no host detection yet, or fdf_score_points ran since), or if scores are asked of an
 * unscored fdf_detect that fit its `cap` and read its pinned frame in place (the frame is not
 * kept; fdf_ctx_set_upload_chunks) -- a call that returned FDF_ERR_CAPACITY keeps it.
 */
int fdf_fetch_last(fdf_ctx* ctx, fdf_point* out, uint16_t* out_scores, size_t cap,
                   size_t* n_out);

/*
 * RGB variant of fdf_detect: `data` holds RGB8 pixels (rows of 3 * width bytes at
 * `stride_bytes`), converted on the device exactly as image 0.24.6's to_luma8 -- the
 * reference's callers run `DynamicImage::ImageRgb8(img).to_luma8()` before detect
 * (src/main.rs:58, tests/compare.rs:33) -- then detected as fdf_detect does.
 */
int fdf_detect_rgb(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                   size_t stride_bytes, const fdf_config* cfg, fdf_point* out, size_t cap,
                   size_t* n_out);

/*
 * Device-side RGB8 -> grey (image 0.24.6 to_luma8: (2126 r + 7152 g + 722 b) / 10000).
 * `n_frames` frames of width x height RGB pixels (rows packed, 3 * width bytes) at
 * d_rgb + f * rgb_frame_stride_bytes; grey frames packed (width * height bytes each) at
 * d_grey.  Asynchronous on `stream` (NULL = the HIP null stream).  n_frames <= 65535.
 */
int fdf_rgb_to_luma_device(fdf_ctx* ctx, const uint8_t* d_rgb, uint32_t n_frames,
                           uint32_t width, uint32_t height, uint64_t rgb_frame_stride_bytes,
                           uint8_t* d_grey, void* stream);

/*
 * Batched host variant: `n_frames` frames of width x height, frame f at
 * data + f * frame_stride_bytes (rows packed, stride == width).  Output is every frame's
 * list concatenated in frame order; frame f's points are out[frame_offsets[f] ..
 * frame_offsets[f+1]) (frame_offsets has n_frames + 1 entries; may be NULL).
 * Capacity semantics as fdf_detect.
 */
int fdf_detect_batch(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames, uint32_t width,
                     uint32_t height, size_t frame_stride_bytes, const fdf_config* cfg,
                     fdf_point* out, size_t cap, uint64_t* frame_offsets, size_t* n_out);

/*
 * Multi-device batched variant (frames shard across GPUs with no collective).
 * The batch is cut into n_ctx contiguous shards of (nearly) equal frame counts, shard k is
 * detected on ctxs[k] by its own host thread (contexts may be on different devices, or
 * several on one), and the lists are concatenated in frame order -- the same result as
 * fdf_detect_batch on one context.  The contexts must be distinct.  Capacity semantics as
 * fdf_detect_batch; each context keeps its shard for fdf_fetch_last_multi.  The contexts are
 * locked in one global order, so concurrent calls over the same contexts listed in different
 * orders do not deadlock.
 */
int fdf_detect_batch_multi(fdf_ctx* const* ctxs, uint32_t n_ctx, const uint8_t* data,
                           uint32_t n_frames, uint32_t width, uint32_t height,
                           size_t frame_stride_bytes, const fdf_config* cfg, fdf_point* out,
                           size_t cap, uint64_t* frame_offsets, size_t* n_out);
/* fdf_fetch_last over the contexts of the last fdf_detect_batch_multi, concatenated.  The
 * contexts must hold the shards of ONE such call, passed in that call's order; otherwise (a
 * host call on one of them since, another multi call, a reordered array) FDF_ERR_ARG. */
int fdf_fetch_last_multi(fdf_ctx* const* ctxs, uint32_t n_ctx, fdf_point* out, size_t cap,
                         size_t* n_out);

/*
 * Device-resident batched variant (the throughput path; nothing crosses PCIe).
 * `d_frames`, `d_out` and `d_frame_offsets` are device pointers on the context's device.
 * Asynchronous: enqueued on `stream` (a hipStream_t; NULL = the HIP null stream; pass
 * fdf_ctx_stream(ctx) for the context's own stream).  On
 * completion d_frame_offsets[0..n_frames] holds the exclusive prefix of per-frame counts
 * and d_frame_offsets[n_frames] the total, even when the total exceeds `cap` (points with
 * index >= cap are not written).  Argument and shape errors are returned synchronously.
 * The context's workspace is reused by each call: a call on another stream than the
 * context's previous call first waits (on the device) for that call's work.  Frames may be
 * spaced by any frame_stride_bytes >= width * height (the gap bytes are never centres or
 * circle pixels); frames before the last may be read up to 15 bytes past their end (inside
 * the batch allocation), the last frame is read exactly.  FDF_ERR_DEVICE is also returned,
 * once, by the call after an asynchronous launch whose output could not be completed (a
 * grid small enough to write its points directly, whose look-back wait ran out: the
 * bounded wait that keeps a faulty device from hanging; the host entry points recover such
 * a launch by themselves).
 */
int fdf_detect_device(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
                      uint32_t width, uint32_t height, uint64_t frame_stride_bytes,
                      const fdf_config* cfg, fdf_point* d_out, uint64_t cap,
                      uint64_t* d_frame_offsets, void* stream);

/*
 * fdf_detect_device for RGB8 frames (rows of 3 * width bytes, frame f at
 * d_frames + f * frame_stride_bytes): the detector converts each loaded pixel with image
 * 0.24.6's to_luma8 -- (2126 r + 7152 g + 722 b) / 10000 -- so the keypoints are those of
 * fdf_rgb_to_luma_device followed by fdf_detect_device, with no grey frames written
 * (src/main.rs:58, tests/compare.rs:33).  3 * width * height < 2^31.  It needs no grey
 * buffer but is slower than the two passes, which the host RGB entry
 * points use.
 */
int fdf_detect_device_rgb(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
                          uint32_t width, uint32_t height, uint64_t frame_stride_bytes,
                          const fdf_config* cfg, fdf_point* d_out, uint64_t cap,
                          uint64_t* d_frame_offsets, void* stream);

/*
 * Ring-level helpers, the reference's pub items of src/fast_simd.rs:
 *   FDF_NORTH..FDF_WEST   :69-72   circle indices of the four cardinal pixels
 *   fdf_circle            :79-98   (dx, dy) of the 16 circle pixels, index 0 north, clockwise
 *   fdf_calculate_offsets :104-110 dy * width + dx (i32, as the reference computes it)
 * Either output pointer of fdf_circle may be NULL.  Host-only, no context needed.
 */
#define FDF_NORTH 0
#define FDF_EAST 4
#define FDF_SOUTH 8
#define FDF_WEST 12
void fdf_circle(int32_t dx[16], int32_t dy[16]);
void fdf_calculate_offsets(uint32_t width, int32_t offsets[16]);

/*
 * Ring scores, the reference's keypoint_score_max_threshold(base_v, pixels, consecutive)
 * (src/fast_simd.rs:623) and keypoint_score_sum_abs_difference(pixels, centers, is_above,
 * is_below, threshold) (:722) with the masks its callers build (:282, test :1213-1222:
 * is_above = p > sat(c + t), is_below = p < sat(c - t)).  Ring k is centers[k] and the 16
 * circle pixels rings[16 k .. 16 k + 16) in fdf_circle order.  cfg->nms picks the function:
 * MaxThreshold (consecutive = cfg->count, 9..16) or SumAbsolute (threshold = cfg->threshold).
 * Runs on the GPU through the detector's own score functions (see fdf_kernels.hip), for any
 * ring.  fdf_score_rings: host in/out, synchronous; invalidates fdf_fetch_last's result.
 * fdf_score_rings_device: device pointers, d_rings 16-byte aligned, asynchronous on
 * `stream` (NULL = the HIP null stream, as for fdf_detect_device; round 6 -- NULL meant the
 * context's stream before, which is not ordered with work on the null stream).
 */
int fdf_score_rings(fdf_ctx* ctx, const uint8_t* centers, const uint8_t* rings, size_t n_rings,
                    const fdf_config* cfg, uint16_t* out_scores);
int fdf_score_rings_device(fdf_ctx* ctx, const uint8_t* d_centers, const uint8_t* d_rings,
                           uint64_t n_rings, const fdf_config* cfg, uint16_t* d_scores,
                           void* stream);

/*
 * Scores for given points (extension: the reference's Point carries no score; these are the
 * u16 values its NMS compares, src/fast_simd.rs:623-718 and :722-749).  Host in/out,
 * synchronous.  `nms` selects the score: MaxThreshold (window = cfg->count) or SumAbsolute
 * (uses cfg->threshold).  Points must be centres (3 <= x < w-3, 3 <= y < h-3).
 */
int fdf_score_points(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                     size_t stride_bytes, const fdf_config* cfg, const fdf_point* points,
                     size_t n_points, uint16_t* out_scores);

/*
 * Detection with scores: (x, y, score) per keypoint.  As fdf_detect / fdf_detect_batch,
 * and out_scores[k] (`cap` entries) is point k's u16 score -- the one cfg->nms suppresses
 * with (MaxThreshold: src/fast_simd.rs:623-718; SumAbsolute: :722-749), or the
 * max-threshold score when NMS is off.  Scores are computed on the device from the frame
 * already resident there; capacity semantics as fdf_detect.
 */
int fdf_detect_scored(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                      size_t stride_bytes, const fdf_config* cfg, fdf_point* out,
                      uint16_t* out_scores, size_t cap, size_t* n_out);
int fdf_detect_batch_scored(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames,
                            uint32_t width, uint32_t height, size_t frame_stride_bytes,
                            const fdf_config* cfg, fdf_point* out, uint16_t* out_scores,
                            size_t cap, uint64_t* frame_offsets, size_t* n_out);

/*
 * Device-resident scoring of fdf_detect_device's output: d_points / d_frame_offsets as that
 * call filled them (same frames, shape, config and `cap`), d_scores with `cap` entries.
 * Asynchronous on `stream`; points with index >= cap are skipped.  n_frames <= 65535.
 */
int fdf_score_device(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
                     uint32_t width, uint32_t height, uint64_t frame_stride_bytes,
                     const fdf_config* cfg, const fdf_point* d_points, uint64_t cap,
                     const uint64_t* d_frame_offsets, uint16_t* d_scores, void* stream);

/*
 * Streaming host pipeline (extension; the reference's callers detect on one
 * host image at a time, src/lib.rs:62-64, src/main.rs:58-64).  Host frames in, host
 * keypoints out, with the host->device copy of one batch, the detection of another and the
 * device->host copy of a third in flight together.  `depth` (1..16) batch slots, each with
 * pinned host staging for `max_frames` frames of width x height pixels (3 bytes per pixel
 * with FDF_PIPE_RGB, converted on the device as fdf_detect_rgb does), its own device
 * buffers, context and HIP stream.  Device output per slot holds max_points_per_frame points
 * per frame (0 = (width-6) * (height-6), the most a frame can have).
 *
 * Tickets are issued in order; ticket k uses slot k % depth, which must have been
 * collected: fdf_pipeline_acquire returns FDF_ERR_BUSY otherwise.  A pipeline is not
 * thread-safe beyond one producer and one consumer calling under the pipeline's own lock
 * (every call takes it; fdf_pipeline_collect releases it while waiting on the device).
 */
typedef struct fdf_pipeline fdf_pipeline;
enum fdf_pipe_flags {
    FDF_PIPE_RGB = 1,     /* frames are RGB8 (rows of 3 * width bytes) */
    FDF_PIPE_SCORES = 2   /* also compute each keypoint's score (as fdf_detect_scored) */
};
int fdf_pipeline_create(int device, uint32_t width, uint32_t height, uint32_t max_frames,
                        uint32_t depth, uint64_t max_points_per_frame, uint32_t flags,
                        const fdf_config* cfg, fdf_pipeline** out);
void fdf_pipeline_destroy(fdf_pipeline* p);
/* The pinned staging buffer of the next ticket: frame f at *frames + f * frame bytes. */
int fdf_pipeline_acquire(fdf_pipeline* p, uint8_t** frames, uint64_t* ticket);
/* Enqueue an acquired ticket's first n_frames (1..max_frames) frames; returns at once. */
int fdf_pipeline_submit(fdf_pipeline* p, uint64_t ticket, uint32_t n_frames);
/* acquire + copy n_frames frames (frame f at frames + f * frame_stride_bytes, rows packed)
 * into the staging buffer + submit. */
int fdf_pipeline_push(fdf_pipeline* p, const uint8_t* frames, uint32_t n_frames,
                      size_t frame_stride_bytes, uint64_t* ticket);
/*
 * Wait for a submitted ticket and copy out its keypoints (frames concatenated in order, each
 * in raster order), scores (FDF_PIPE_SCORES; `out_scores` may be NULL) and frame_offsets
 * (n_frames + 1 entries; may be NULL).  FDF_ERR_CAPACITY: `cap` is below *n_out; nothing
 * is released, call again with a larger buffer.  FDF_OK releases the slot.  FDF_ERR_DROPPED:
 * the batch had *n_out points but the slot held only the first max_points_per_frame *
 * n_frames of them (those are copied, frame_offsets are exact); the slot is released.
 */
int fdf_pipeline_collect(fdf_pipeline* p, uint64_t ticket, fdf_point* out,
                         uint16_t* out_scores, size_t cap, uint64_t* frame_offsets,
                         size_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* FDF_H */
