// fdf_api.cpp -- the C ABI of include/fdf.h on top of the HIP kernels.
//
// Replaces fast_simd::detector (iwanders/feature_detector_fast src/fast_simd.rs:847-859):
// validation mirrors the reference's panics (:302-305, :342, :369, :800) as status codes,
// the device work is the fused band kernel (fdf_kernels.hip), and the host side only moves
// bytes and picks the band height.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <new>

#include "../../include/fdf.h"
#include "fdf_kernels.h"

struct fdf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // device workspace, grown on demand
    uint8_t* d_in = nullptr;            size_t in_bytes = 0;       // host-API frame staging
    uint8_t* d_rgb = nullptr;           size_t rgb_bytes = 0;      // host-API RGB staging
    uint2* d_out = nullptr;             size_t out_points = 0;     // host-API output
    uint64_t* d_offsets = nullptr;      size_t offsets_n = 0;      // host-API frame offsets
    uint16_t* d_scores = nullptr;       size_t scores_n = 0;       // host-API scores
    uint8_t* d_slots = nullptr;         size_t slots_bytes = 0;    // per-band output slots
    uint32_t* d_counts = nullptr;       size_t counts_n = 0;       // per-band keypoint counts
    uint8_t* d_map = nullptr;           size_t map_bytes = 0;      // NMS score map
    // optional per-kernel timing (fdf_ctx_set_timing): 3 events around each call's launches
    bool timing = false;
    size_t timed = 0;                     // calls recorded since timing was enabled
    std::vector<hipEvent_t> ev;           // 3 per recorded call, kMaxTimedCalls at most
};

constexpr size_t kMaxTimedCalls = 4096;

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int check_config(const fdf_config* cfg) {
    if (!cfg) return FDF_ERR_ARG;
    if (cfg->count < 9 || cfg->count > 16) return FDF_ERR_COUNT;
    if (cfg->nms > FDF_NMS_SUM_ABSOLUTE) return FDF_ERR_NMS;
    return FDF_OK;
}

// Shape rules derived from the reference's u32 arithmetic (SURVEY.md §7 "Errors").
int check_shape(uint32_t w, uint32_t h, int* empty) {
    *empty = 0;
    if (h < 3) return FDF_ERR_SIZE;        // height - 3 underflows (src/fast_simd.rs:342)
    if (h <= 6) { *empty = 1; return FDF_OK; }
    if (w < 6) return FDF_ERR_SIZE;        // width - 3 - 3 underflows (:369)
    if (w == 6) { *empty = 1; return FDF_OK; }
    return FDF_OK;
}

template <typename T>
int ensure(T** buf, size_t* have, size_t need, bool zero, hipStream_t stream) {
    if (*have >= need) return FDF_OK;
    if (*buf) { (void)hipStreamSynchronize(stream); (void)hipFree(*buf); *buf = nullptr; *have = 0; }
    size_t n = std::max(need, *have * 2);
    if (hipMalloc(reinterpret_cast<void**>(buf), n * sizeof(T)) != hipSuccess) {
        *buf = nullptr;
        return FDF_ERR_ALLOC;
    }
    if (zero && hipMemsetAsync(*buf, 0, n * sizeof(T), stream) != hipSuccess) return FDF_ERR_DEVICE;
    *have = n;
    return FDF_OK;
}

// Band geometry of the sweep kernel.  A band is R full-width centre rows; its 4 waves take
// units = column strips (992 centres) x sub-bands.  Tall bands amortise the 8-row halo of a
// sub-band; short bands give a small job (one frame) enough workgroups.  The LDS footprint
// is kept <= 40 KB so 4 workgroups fit a CU.
struct Geometry {
    uint32_t R, nstrips, nsub;
};


Geometry pick_geometry(uint32_t n_frames, uint32_t w, uint32_t h, uint32_t nms) {
    Geometry g;
    const uint32_t sc = (uint32_t)fdfk::strip_cols(fdfk::kLaneCols);
    g.nstrips = (w - 3 + sc - 1) / sc;
    // >= 4 units per band (one per wave), handed out dynamically; taller units (fewer halo
    // rows) measured faster than more, shorter units for balance
    g.nsub = (4 + g.nstrips - 1) / g.nstrips;
    if (const char* e = std::getenv("FDF_NSUB")) g.nsub = (uint32_t)std::strtoul(e, nullptr, 0);
    const uint32_t centre_rows = h - 6;
    const uint32_t nw = (w + 31) / 32;
    // extra rows a unit tests: NMS bands test one row above and below (first / last unit)
    const uint32_t halo = fdfk::band_halo(nms) * (g.nsub == 1 ? 2u : 1u);
    // LDS per workgroup sets the workgroups per CU: <= 40 KB keeps 4.
    // Without NMS a 35 KB budget (bands of ~122 rows at 1080p) measured faster than the
    // tallest band that fits (more, shorter workgroups: a shorter grid tail).
    uint32_t budget = nms ? 40000u : 35000u;
    if (const char* b = std::getenv("FDF_LDS_BUDGET")) budget = (uint32_t)std::strtoul(b, nullptr, 0);
    // Among band heights whose grid fills the chip (>= 1024 workgroups), take the one with
    // the most owned rows per sweep step; a grid that cannot fill the chip takes the
    // shortest sweep (one 8-step block per unit) for the lowest latency.
    // FDF_MIN_TASKS (tests): the grid size that counts as filling the chip, so that a small
    // job can run the full-size geometry (tall bands, long units)
    uint64_t min_tasks = 1024;
    if (const char* m = std::getenv("FDF_MIN_TASKS")) min_tasks = std::strtoull(m, nullptr, 0);
    double best = -1.0;
    g.R = 0;
    for (uint32_t R = g.nsub; R <= 256 && R < centre_rows + g.nsub; R += g.nsub) {
        if (fdfk::make_sweep_layout(R, nw, nms).total > budget) break;
        const uint64_t tasks = (uint64_t)n_frames * ((centre_rows + R - 1) / R);
        if (tasks < min_tasks) break;
        const uint32_t steps = fdfk::sweep_steps(R / g.nsub, halo);
        const double eff = (double)R / (double)(steps * g.nsub);
        if (eff > best + 1e-9) { best = eff; g.R = R; }
    }
    if (g.R == 0) {
        const uint32_t unit = fdfk::kSweepRing - 3 - halo;
        g.R = g.nsub * unit;
        while (g.R > g.nsub && fdfk::make_sweep_layout(g.R, nw, nms).total > budget)
            g.R -= g.nsub;
    }
    return g;
}

// Enqueue detection + compaction over `n_frames` device frames (w, h >= 7).
int enqueue(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames, uint32_t w, uint32_t h,
            uint64_t frame_stride, const fdf_config* cfg, uint2* d_out, uint64_t cap,
            uint64_t* d_offsets, hipStream_t stream) {
    const uint32_t sb = fdfk::score_bytes_for(cfg->nms);
    const Geometry geo = pick_geometry(n_frames, w, h, cfg->nms);
    const uint32_t R = geo.R;
    const uint32_t nw = (w + 31) / 32;
    if (fdfk::make_sweep_layout(R, nw, cfg->nms).total > fdfk::kSweepMaxLds)
        return FDF_ERR_SIZE;
    const uint32_t bands = (h - 6 + R - 1) / R;
    const uint64_t ntasks = (uint64_t)bands * n_frames;
    if (ntasks == 0 || ntasks > 0x7fffffffull) return FDF_ERR_SIZE;
    const uint32_t slot_bytes = fdfk::slot_bytes_for(R, nw);
    uint32_t tpg = fdfk::compact_tasks_per_group((uint32_t)ntasks);
    if (const char* e = std::getenv("FDF_COMPACT_TPG"))   // ablation runs only
        tpg = std::max(1u, std::min((uint32_t)fdfk::kCompactTasks, (uint32_t)std::strtoul(e, nullptr, 0)));
    int rc;
    if ((rc = ensure(&ctx->d_slots, &ctx->slots_bytes, (size_t)(ntasks * slot_bytes), false, stream))) return rc;
    if ((rc = ensure(&ctx->d_counts, &ctx->counts_n, (size_t)ntasks, false, stream))) return rc;
    // NMS score map: written at keypoints only and read only where the keypoint bitmap
    // marks one, so it is never cleared
    if (sb && (rc = ensure(&ctx->d_map, &ctx->map_bytes, (size_t)n_frames * w * h * sb, false, stream)))
        return rc;
    const char* dbg = std::getenv("FDF_DEBUG_FLAGS");   // ablation runs only, see fdf_kernels.h
    fdfk::BandParams p;
    p.frames = d_frames;
    p.frame_stride = frame_stride;
    p.width = w;
    p.height = h;
    p.rows = R;
    p.bands_per_frame = bands;
    p.ntasks = (uint32_t)ntasks;
    p.words_per_row = nw;
    p.threshold = cfg->threshold;
    p.slot_bytes = slot_bytes;
    p.slots = ctx->d_slots;
    p.counts = ctx->d_counts;
    p.flags = dbg ? (uint32_t)std::strtoul(dbg, nullptr, 0) : 0u;
    p.nstrips = geo.nstrips;
    p.nsub = geo.nsub;
    p.scores = ctx->d_map;
    fdfk::CompactParams c;
    c.width = w;
    c.height = h;
    c.rows = R;
    c.bands_per_frame = bands;
    c.ntasks = (uint32_t)ntasks;
    c.words_per_row = nw;
    c.slot_bytes = slot_bytes;
    c.tasks_per_group = tpg;
    c.slots = ctx->d_slots;
    c.counts = ctx->d_counts;
    c.out = d_out;
    c.cap = cap;
    c.frame_offsets = d_offsets;
    hipEvent_t* ev = nullptr;
    if (ctx->timing && ctx->timed < kMaxTimedCalls) {
        while (ctx->ev.size() < 3 * (ctx->timed + 1)) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return FDF_ERR_DEVICE;
            ctx->ev.push_back(e);
        }
        ev = &ctx->ev[3 * ctx->timed];
    }
    if (ev && hipEventRecord(ev[0], stream) != hipSuccess) return FDF_ERR_DEVICE;
    if (fdfk::launch_sweep(p, cfg->nms, cfg->count, stream) != hipSuccess) return FDF_ERR_DEVICE;
    if (ev && hipEventRecord(ev[1], stream) != hipSuccess) return FDF_ERR_DEVICE;
    if (fdfk::launch_compact(c, stream) != hipSuccess) return FDF_ERR_DEVICE;
    if (ev) {
        if (hipEventRecord(ev[2], stream) != hipSuccess) return FDF_ERR_DEVICE;
        ++ctx->timed;
    }
    return FDF_OK;
}

// Shared body of fdf_detect / fdf_detect_batch: host frames in, host points out.
// `rgb`: the frames are RGB8 (rows of 3 * w bytes at row_stride), converted on the device
// with image 0.24.6's to_luma8 before detection (src/main.rs:58).
// The score reported with a keypoint: the NMS mode's own, max-threshold when NMS is off.
uint32_t score_kind(uint32_t nms) {
    return nms == FDF_NMS_SUM_ABSOLUTE ? FDF_NMS_SUM_ABSOLUTE : FDF_NMS_MAX_THRESHOLD;
}
// ~4 points per thread on average, 1..64 workgroups per frame.
uint32_t score_blocks(uint64_t points, uint32_t n_frames) {
    const uint64_t per_frame = points / std::max<uint32_t>(n_frames, 1u);
    return (uint32_t)std::min<uint64_t>(64, per_frame / 1024 + 1);
}

int detect_host(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames, uint32_t w, uint32_t h,
                size_t row_stride, size_t frame_stride, const fdf_config* cfg, fdf_point* out,
                size_t cap, uint64_t* frame_offsets, size_t* n_out, bool rgb = false,
                uint16_t* out_scores = nullptr, bool scored = false) {
    if (!ctx || !n_out || (cap && !out) || (scored && cap && !out_scores)) return FDF_ERR_ARG;
    int rc = check_config(cfg);
    if (rc) return rc;
    int empty = 0;
    rc = check_shape(w, h, &empty);
    if (rc) return rc;
    if (n_frames == 0) empty = 1;
    if (!data && !empty) return FDF_ERR_ARG;
    if (row_stride < (rgb ? 3ull * w : (size_t)w)) return FDF_ERR_ARG;
    if (empty) {
        *n_out = 0;
        if (frame_offsets) std::memset(frame_offsets, 0, sizeof(uint64_t) * (n_frames + 1ull));
        return FDF_OK;
    }
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    const size_t frame_bytes = (size_t)w * h;
    const size_t max_points = (size_t)(w - 6) * (h - 6) * n_frames;
    if ((rc = ensure(&ctx->d_in, &ctx->in_bytes, frame_bytes * n_frames, false, ctx->stream))) return rc;
    if ((rc = ensure(&ctx->d_out, &ctx->out_points, max_points, false, ctx->stream))) return rc;
    if ((rc = ensure(&ctx->d_offsets, &ctx->offsets_n, n_frames + 1ull, false, ctx->stream))) return rc;
    const size_t px = rgb ? 3 : 1;                 // bytes per pixel of the host frames
    uint8_t* stage = ctx->d_in;
    if (rgb) {
        if ((rc = ensure(&ctx->d_rgb, &ctx->rgb_bytes, 3 * frame_bytes * n_frames, false, ctx->stream)))
            return rc;
        stage = ctx->d_rgb;
    }
    for (uint32_t f = 0; f < n_frames; ++f) {
        const uint8_t* src = data + (size_t)f * frame_stride;
        uint8_t* dst = stage + (size_t)f * frame_bytes * px;
        hipError_t e = row_stride == px * w
                           ? hipMemcpyAsync(dst, src, frame_bytes * px, hipMemcpyHostToDevice,
                                            ctx->stream)
                           : hipMemcpy2DAsync(dst, px * w, src, row_stride, px * w, h,
                                              hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) return FDF_ERR_DEVICE;
    }
    if (rgb && fdfk::launch_rgb_to_luma(ctx->d_rgb, n_frames, (uint32_t)frame_bytes,
                                        3 * frame_bytes, ctx->d_in, ctx->stream) != hipSuccess)
        return FDF_ERR_DEVICE;
    rc = enqueue(ctx, ctx->d_in, n_frames, w, h, frame_bytes, cfg, ctx->d_out, max_points,
                 ctx->d_offsets, ctx->stream);
    if (rc) return rc;
    uint64_t* offs = frame_offsets;
    uint64_t local[2];
    if (!offs) offs = n_frames == 1 ? local : new (std::nothrow) uint64_t[n_frames + 1ull];
    if (!offs) return FDF_ERR_ALLOC;
    hipError_t e = hipMemcpyAsync(offs, ctx->d_offsets, sizeof(uint64_t) * (n_frames + 1ull),
                                  hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    const uint64_t total = offs[n_frames];
    if (offs != frame_offsets && offs != local) delete[] offs;
    if (e != hipSuccess) return FDF_ERR_DEVICE;
    const size_t ncopy = (size_t)std::min<uint64_t>(total, cap);
    if (scored && ncopy) {
        if ((rc = ensure(&ctx->d_scores, &ctx->scores_n, ncopy, false, ctx->stream))) return rc;
        e = fdfk::launch_score_frames(ctx->d_in, w, frame_bytes, n_frames, ctx->d_out,
                                      ctx->d_offsets, ncopy, score_blocks(ncopy, n_frames),
                                      score_kind(cfg->nms), cfg->threshold, cfg->count,
                                      ctx->d_scores, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out_scores, ctx->d_scores, ncopy * sizeof(uint16_t),
                               hipMemcpyDeviceToHost, ctx->stream);
        if (e != hipSuccess) return FDF_ERR_DEVICE;
    }
    if (ncopy) {
        e = hipMemcpyAsync(out, ctx->d_out, ncopy * sizeof(fdf_point), hipMemcpyDeviceToHost,
                           ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return FDF_ERR_DEVICE;
    }
    *n_out = (size_t)total;
    return total > cap ? FDF_ERR_CAPACITY : FDF_OK;
}

}  // namespace

extern "C" {

int fdf_abi_version(void) { return FDF_ABI_VERSION; }

const char* fdf_status_string(int status) {
    switch (status) {
        case FDF_OK: return "ok";
        case FDF_ERR_COUNT: return "count must be in [9, 16]";
        case FDF_ERR_SIZE: return "image size not supported by the reference (h < 3, or w < 6 with h >= 7)";
        case FDF_ERR_CAPACITY: return "output buffer too small";
        case FDF_ERR_NMS: return "unknown non-maximal suppression mode";
        case FDF_ERR_DEVICE: return "HIP device error";
        case FDF_ERR_ARG: return "invalid argument";
        case FDF_ERR_ALLOC: return "allocation failed";
        case FDF_ERR_BUSY: return "pipeline slot still holds uncollected results";
        case FDF_ERR_DROPPED: return "batch found more keypoints than the pipeline's device capacity";
        default: return "unknown status";
    }
}

int fdf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int fdf_validate(uint32_t width, uint32_t height, const fdf_config* cfg, int* empty) {
    if (!empty) return FDF_ERR_ARG;
    int rc = check_config(cfg);
    if (rc) return rc;
    return check_shape(width, height, empty);
}

int fdf_ctx_create(int device, fdf_ctx** out_ctx) {
    if (!out_ctx) return FDF_ERR_ARG;
    *out_ctx = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return FDF_ERR_DEVICE;
    fdf_ctx* ctx = new (std::nothrow) fdf_ctx();
    if (!ctx) return FDF_ERR_ALLOC;
    ctx->device = device;
    DeviceGuard guard(device);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return FDF_ERR_DEVICE;
    }
    *out_ctx = ctx;
    return FDF_OK;
}

void fdf_ctx_destroy(fdf_ctx* ctx) {
    if (!ctx) return;
    {
        DeviceGuard guard(ctx->device);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->d_in);
        (void)hipFree(ctx->d_rgb);
        (void)hipFree(ctx->d_out);
        (void)hipFree(ctx->d_offsets);
        (void)hipFree(ctx->d_scores);
        (void)hipFree(ctx->d_slots);
        (void)hipFree(ctx->d_counts);
        (void)hipFree(ctx->d_map);
        for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

void* fdf_ctx_stream(fdf_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int fdf_ctx_set_timing(fdf_ctx* ctx, int enable) {
    if (!ctx) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->timing = enable != 0;
    ctx->timed = 0;
    return FDF_OK;
}

int fdf_ctx_timing(fdf_ctx* ctx, uint32_t* calls, float* detect_ms, float* compact_ms) {
    if (!ctx || !calls || !detect_ms || !compact_ms) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    *calls = (uint32_t)ctx->timed;
    *detect_ms = *compact_ms = 0.0f;
    for (size_t k = 0; k < ctx->timed; ++k) {
        const hipEvent_t* e = &ctx->ev[3 * k];
        float a = 0.0f, b = 0.0f;
        if (hipEventSynchronize(e[2]) != hipSuccess ||
            hipEventElapsedTime(&a, e[0], e[1]) != hipSuccess ||
            hipEventElapsedTime(&b, e[1], e[2]) != hipSuccess)
            return FDF_ERR_DEVICE;
        *detect_ms += a;
        *compact_ms += b;
    }
    return FDF_OK;
}

int fdf_detect(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
               size_t stride_bytes, const fdf_config* cfg, fdf_point* out, size_t cap,
               size_t* n_out) {
    return detect_host(ctx, data, 1, width, height, stride_bytes, 0, cfg, out, cap, nullptr,
                       n_out);
}

int fdf_detect_rgb(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                   size_t stride_bytes, const fdf_config* cfg, fdf_point* out, size_t cap,
                   size_t* n_out) {
    return detect_host(ctx, data, 1, width, height, stride_bytes, 0, cfg, out, cap, nullptr,
                       n_out, true);
}

int fdf_rgb_to_luma_device(fdf_ctx* ctx, const uint8_t* d_rgb, uint32_t n_frames,
                           uint32_t width, uint32_t height, uint64_t rgb_frame_stride_bytes,
                           uint8_t* d_grey, void* stream) {
    if (!ctx) return FDF_ERR_ARG;
    const uint64_t pixels = (uint64_t)width * height;
    if (n_frames == 0 || pixels == 0) return FDF_OK;
    if (!d_rgb || !d_grey || pixels > 0x7fffffffull / 3 || rgb_frame_stride_bytes < 3 * pixels ||
        n_frames > 65535u)
        return FDF_ERR_ARG;
    DeviceGuard guard(ctx->device);
    if (fdfk::launch_rgb_to_luma(d_rgb, n_frames, (uint32_t)pixels, rgb_frame_stride_bytes, d_grey,
                                 reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
        return FDF_ERR_DEVICE;
    return FDF_OK;
}

int fdf_detect_scored(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                      size_t stride_bytes, const fdf_config* cfg, fdf_point* out,
                      uint16_t* out_scores, size_t cap, size_t* n_out) {
    return detect_host(ctx, data, 1, width, height, stride_bytes, 0, cfg, out, cap, nullptr,
                       n_out, false, out_scores, true);
}

int fdf_detect_batch_scored(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames,
                            uint32_t width, uint32_t height, size_t frame_stride_bytes,
                            const fdf_config* cfg, fdf_point* out, uint16_t* out_scores,
                            size_t cap, uint64_t* frame_offsets, size_t* n_out) {
    if (n_frames > 1 && frame_stride_bytes < (size_t)width * height) return FDF_ERR_ARG;
    if (n_frames > 65535u) return FDF_ERR_ARG;
    return detect_host(ctx, data, n_frames, width, height, width, frame_stride_bytes, cfg, out,
                       cap, frame_offsets, n_out, false, out_scores, true);
}

int fdf_score_device(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
                     uint32_t width, uint32_t height, uint64_t frame_stride_bytes,
                     const fdf_config* cfg, const fdf_point* d_points, uint64_t cap,
                     const uint64_t* d_frame_offsets, uint16_t* d_scores, void* stream) {
    if (!ctx || !d_frame_offsets) return FDF_ERR_ARG;
    int rc = check_config(cfg);
    if (rc) return rc;
    int empty = 0;
    rc = check_shape(width, height, &empty);
    if (rc) return rc;
    if (empty || n_frames == 0 || cap == 0) return FDF_OK;
    if (!d_frames || !d_points || !d_scores || n_frames > 65535u) return FDF_ERR_ARG;
    if (n_frames > 1 && frame_stride_bytes < (uint64_t)width * height) return FDF_ERR_ARG;
    DeviceGuard guard(ctx->device);
    const uint64_t fs = n_frames > 1 ? frame_stride_bytes : (uint64_t)width * height;
    const uint64_t est = std::min<uint64_t>(cap, (uint64_t)width * height / 32 * n_frames);
    return fdfk::launch_score_frames(d_frames, width, fs, n_frames,
                                     reinterpret_cast<const uint2*>(d_points), d_frame_offsets,
                                     cap, score_blocks(est, n_frames), score_kind(cfg->nms),
                                     cfg->threshold, cfg->count, d_scores,
                                     reinterpret_cast<hipStream_t>(stream)) == hipSuccess
               ? FDF_OK
               : FDF_ERR_DEVICE;
}

int fdf_detect_batch(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames, uint32_t width,
                     uint32_t height, size_t frame_stride_bytes, const fdf_config* cfg,
                     fdf_point* out, size_t cap, uint64_t* frame_offsets, size_t* n_out) {
    if (n_frames > 1 && frame_stride_bytes < (size_t)width * height) return FDF_ERR_ARG;
    return detect_host(ctx, data, n_frames, width, height, width, frame_stride_bytes, cfg, out,
                       cap, frame_offsets, n_out);
}

int fdf_detect_device(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
                      uint32_t width, uint32_t height, uint64_t frame_stride_bytes,
                      const fdf_config* cfg, fdf_point* d_out, uint64_t cap,
                      uint64_t* d_frame_offsets, void* stream) {
    if (!ctx || !d_frame_offsets) return FDF_ERR_ARG;
    int rc = check_config(cfg);
    if (rc) return rc;
    int empty = 0;
    rc = check_shape(width, height, &empty);
    if (rc) return rc;
    if (n_frames == 0) empty = 1;
    if (!empty && (!d_frames || (cap && !d_out))) return FDF_ERR_ARG;
    if (n_frames > 1 && frame_stride_bytes < (uint64_t)width * height) return FDF_ERR_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);   // NULL = the HIP null stream
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    if (empty) {
        return hipMemsetAsync(d_frame_offsets, 0, sizeof(uint64_t) * (n_frames + 1ull), s) ==
                       hipSuccess
                   ? FDF_OK
                   : FDF_ERR_DEVICE;
    }
    return enqueue(ctx, d_frames, n_frames, width, height,
                   n_frames > 1 ? frame_stride_bytes : (uint64_t)width * height, cfg,
                   reinterpret_cast<uint2*>(d_out), cap, d_frame_offsets, s);
}

int fdf_score_points(fdf_ctx* ctx, const uint8_t* data, uint32_t width, uint32_t height,
                     size_t stride_bytes, const fdf_config* cfg, const fdf_point* points,
                     size_t n_points, uint16_t* out_scores) {
    if (!ctx || !cfg || (n_points && (!points || !out_scores || !data))) return FDF_ERR_ARG;
    if (cfg->count < 9 || cfg->count > 16) return FDF_ERR_COUNT;
    if (cfg->nms != FDF_NMS_MAX_THRESHOLD && cfg->nms != FDF_NMS_SUM_ABSOLUTE) return FDF_ERR_NMS;
    if (stride_bytes < width || n_points > 0xffffffffull) return FDF_ERR_ARG;
    for (size_t k = 0; k < n_points; ++k) {
        const fdf_point p = points[k];
        if (p.x < 3 || p.y < 3 || (uint64_t)p.x + 3 >= width || (uint64_t)p.y + 3 >= height)
            return FDF_ERR_ARG;
    }
    if (n_points == 0) return FDF_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    const size_t frame_bytes = (size_t)width * height;
    int rc;
    if ((rc = ensure(&ctx->d_in, &ctx->in_bytes, frame_bytes, false, ctx->stream))) return rc;
    if ((rc = ensure(&ctx->d_out, &ctx->out_points, n_points + (n_points + 3) / 4, false,
                     ctx->stream)))
        return rc;
    hipError_t e = stride_bytes == width
                       ? hipMemcpyAsync(ctx->d_in, data, frame_bytes, hipMemcpyHostToDevice, ctx->stream)
                       : hipMemcpy2DAsync(ctx->d_in, width, data, stride_bytes, width, height,
                                          hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->d_out, points, n_points * sizeof(fdf_point), hipMemcpyHostToDevice,
                           ctx->stream);
    uint16_t* d_scores = reinterpret_cast<uint16_t*>(ctx->d_out + n_points);
    if (e == hipSuccess)
        e = fdfk::launch_score_points(ctx->d_in, width, ctx->d_out, (uint32_t)n_points, cfg->nms,
                                      cfg->threshold, cfg->count, d_scores, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(out_scores, d_scores, n_points * sizeof(uint16_t), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
}

}  // extern "C"
