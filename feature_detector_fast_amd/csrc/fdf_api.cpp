// fdf_api.cpp -- the C ABI of include/fdf.h on top of the HIP kernels.
//
// Replaces fast_simd::detector (iwanders/feature_detector_fast src/fast_simd.rs:847-859):
// validation mirrors the reference's panics (:302-305, :342, :369, :800) as status codes,
// the device work is the fused band kernel (fdf_kernels.hip), and the host side only moves
// bytes and picks the band height.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#include <new>

#include "../../include/fdf.h"
#include "fdf_kernels.h"

// Result of the last host-API detection on a context (fdf_fetch_last): its points stay in
// d_out, its offsets in d_offsets and its frames in d_in until the next host call.
struct LastResult {
    bool valid = false;
    bool host_out = false;         // the points / offsets are in the host-mapped h_out / h_offs
    uint64_t total = 0;
    uint32_t n_frames = 0, width = 0, height = 0;
    fdf_config cfg{};
    bool rgb = false;              // frames in d_rgb (RGB8); scores need their luma in d_in
    bool in_place = false;         // the frame was read in place from pinned host memory: not
                                   // in d_in, so the result has no scores (fdf_fetch_last)
    // fdf_detect_batch_multi: the call's generation (0: not a multi-context result) and this
    // context's shard of it, checked by fdf_fetch_last_multi
    uint64_t multi_gen = 0;
    uint32_t shard = 0, nshards = 0;
};

struct fdf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // device workspace, grown on demand
    uint8_t* d_in = nullptr;            size_t in_bytes = 0;       // host-API frame staging
    uint8_t* d_rgb = nullptr;           size_t rgb_bytes = 0;      // host-API RGB staging
    uint2* d_out = nullptr;             size_t out_points = 0;     // host-API output
    uint64_t* d_offsets = nullptr;      size_t offsets_n = 0;      // host-API frame offsets
    // host-API output in pinned, device-mapped host memory: the detector (direct output) or
    // the compaction writes the points and offsets there over PCIe, so a host call needs no
    // copy kernel, no device-to-host copy and one synchronisation (hd_*: device addresses)
    uint2* h_out = nullptr;             uint2* hd_out = nullptr;   size_t h_out_points = 0;
    uint64_t* h_offs = nullptr;         uint64_t* hd_offs = nullptr;   size_t h_offs_n = 0;
    // fdf_detect's overlapped upload: the frame goes up in row chunks on copy_stream, each
    // chunk's flag (pinned, device-mapped) set to the call's epoch after its copy, while the
    // detector already runs and each band waits for the chunk of its last row
    hipStream_t copy_stream = nullptr;
    uint32_t* h_flags = nullptr;        // pinned: the epoch each chunk's flag copy carries
    uint32_t* d_flags = nullptr;        // device: the chunk flags the bands poll
    uint32_t chunk_epoch = 0;
    uint32_t chunks = 0;                // upload chunks (0: kChunksDefault; 1: no overlap)
    // host frames that start in pinned memory but run past its mapping (a hipHostRegister'ed
    // range shorter than the frames) are packed into this pinned buffer by the CPU first: the
    // runtime's DMA copy rejects such a source range
    uint8_t* h_stage = nullptr;         uint8_t* hd_stage = nullptr;   size_t h_stage_bytes = 0;
    // recoveries the host entry points made on their own (fdf_ctx_recoveries): a band's wait
    // for its upload chunk ran out and the frame was detected again from one copy; a
    // direct-output look-back ran out and the compaction rebuilt the output from the slots
    uint64_t upload_fallbacks = 0, lookback_recoveries = 0;
    // an asynchronous device call's look-back ran out and a host call found the error word
    // first: kept here and returned by the next fdf_detect_device(_rgb), as fdf.h promises
    bool pending_device_error = false;
    uint16_t* d_scores = nullptr;       size_t scores_n = 0;       // host-API scores
    uint8_t* d_slots = nullptr;         size_t slots_bytes = 0;    // per-band output slots
    uint32_t* d_counts = nullptr;       size_t counts_n = 0;       // per-band keypoint counts
    // compaction bases: two alternating buffers of per-group sums (kept zero between uses)
    // and the keypoint-statistics word, all zeroed once at context creation
    uint32_t* d_sums = nullptr;         // 2 x fdfk::kMaxGroupSums, then 4 words
    int sums_parity = 0;
    bool sums_dirty = false;            // a launch failed: re-zero before the next use
    // NMS keypoint density feedback (band height): the compaction writes the last finished
    // launch's pre-NMS keypoint total to host-mapped memory, tagged with its launch number
    uint64_t* h_stats = nullptr;        // pinned, mapped; *h_stats = seq << 32 | total;
                                        // h_stats[1]: the direct output's look-back error word
    uint64_t* d_stats = nullptr;        // its device address
    uint32_t stats_seq = 0;
    struct LaunchInfo { uint32_t seq = 0, t = 0, n = 0, nms = 0, w = 0; double pixels = 0; };
    LaunchInfo hist[64];
    // the last density read, kept for its configuration: with more launches in flight than
    // `hist` holds, a read finds its launch's record overwritten (the band height then
    // alternated between launches of one configuration)
    // (one per NMS mode, so that interleaved modes keep theirs)
    LaunchInfo known[3];
    double known_density[3] = {0.0, 0.0, 0.0};
    // cross-stream ordering: the device work of the last enqueue (on any stream) completes
    // at `done`; the next enqueue on another stream waits for it first
    hipEvent_t done = nullptr;
    hipStream_t done_stream = nullptr;
    bool done_valid = false;
    // the last enqueue's work is on done_stream but `done` is not recorded after it yet: on
    // the context's own stream and the null stream (streams that outlive every call) the
    // record waits until something needs it (another stream's call, a host wait), so a
    // stream of back-to-back calls enqueues one packet per call, not two
    bool done_pending = false;
    // the last enqueue's compaction, relaunched when the host output has to grow
    fdfk::CompactParams last_compact{};
    LastResult last;
    // grid size that counts as filling the chip (fdf_ctx_set_geometry; 0 = kDefaultMinTasks)
    uint64_t min_tasks = 0;
    uint32_t band_rows = 0;              // fdf_ctx_set_band_rows (0 = automatic)
    // optional per-kernel timing (fdf_ctx_set_timing): every `timing`-th call (0: off) records
    // its kernels' durations
    uint32_t timing = 0;
    uint64_t timing_calls = 0;            // calls since timing was enabled
    size_t timed = 0;                     // calls recorded since timing was enabled
    std::vector<hipEvent_t> ev;           // 4 per recorded call, kMaxTimedCalls at most
    std::vector<uint8_t> timed_compact;   // per recorded call: 1 if it launched the compaction
    // direct output of small grids (BandParams::direct): look-back descriptors, launch tag
    uint64_t* d_lookback = nullptr;       size_t lookback_n = 0;
    // band tickets: the device counter (a spare word of d_sums, zeroed with it) has handed out
    // ticket_next tickets, ntasks per direct launch
    uint32_t ticket_next = 0;
    uint32_t cus = 0;                     // compute units of the device
    // workgroups per CU of a detector instance (sweep_occupancy), by configuration
    struct Occupancy { uint32_t nms, n, lds; bool rgb; uint32_t wg; };
    std::vector<Occupancy> occupancy;
    // debug builds (FDF_STAMPS set): the last detector launch's workgroup stamps
    uint64_t* d_stamps = nullptr;         size_t stamps_n = 0;
    uint64_t stamps_used = 0;             // words written by the last launch
};

constexpr size_t kMaxTimedCalls = 4096;
constexpr uint64_t kDefaultMinTasks = 1024;   // 4 workgroups on each of 256 CUs
constexpr uint32_t kMaxBandRows = 256;        // fdf_ctx_set_band_rows: the automatic path's range
constexpr uint32_t kMaxChunks = 16;           // overlapped upload: chunks at most
// Default 1 (no overlap): each chunk's ready flag costs a copy on the copy stream, which this
// runtime runs as a blit kernel (~4 us plus ~9 us of queue gap, profiles/r04/t7_*): 1080p
// max-t pinned measured p50 0.0787 / 0.0999 / 0.1406 / 0.2196 ms at 1 / 2 / 4 / 8 chunks.
constexpr uint32_t kChunksDefault = 1;
constexpr size_t kChunkMinBytes = 1u << 18;   // frames below 256 KB upload in one copy

// process-wide counters: fdf_detect_batch_multi call generations, direct-output launch tags
std::atomic<uint64_t> g_multi_gen{0};
std::atomic<uint32_t> g_launch_epoch{0};

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

// `done` covers the last enqueue's work (recorded now if that was deferred).
hipError_t record_done(fdf_ctx* ctx) {
    if (!ctx->done_valid || !ctx->done_pending) return hipSuccess;
    ctx->done_pending = false;
    return hipEventRecord(ctx->done, ctx->done_stream);
}

// After enqueueing the context's work on `stream`: `done` is to follow it, now or (streams
// that outlive every call: the context's own, the null stream) when first needed.
hipError_t note_done(fdf_ctx* ctx, hipStream_t stream) {
    ctx->done_stream = stream;
    ctx->done_valid = true;
    ctx->done_pending = true;
    if (stream == ctx->stream || stream == nullptr) return hipSuccess;
    return record_done(ctx);
}

// The device work of the last enqueue (whatever stream it ran on) has finished.
void wait_done(fdf_ctx* ctx) {
    if (!ctx->done_valid) return;
    const hipError_t e = record_done(ctx) == hipSuccess ? hipEventSynchronize(ctx->done)
                                                        : hipStreamSynchronize(ctx->done_stream);
    if (e == hipSuccess) ctx->done_valid = false;    // nothing of the context is outstanding
}

// hipStreamSynchronize of the context's own stream; when the last enqueue ran there, nothing
// of the context is outstanding afterwards (the next wait_done returns at once: a host call's
// completion event is never recorded and waited on after the fact)
hipError_t sync_own_stream(fdf_ctx* ctx) {
    const hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && ctx->done_valid && ctx->done_stream == ctx->stream) {
        ctx->done_valid = false;
        ctx->done_pending = false;
    }
    return e;
}

// Grow a workspace buffer to `need` elements (+1/8 headroom).  The old buffer may still be
// read by work on another stream, so everything the context enqueued is drained first.
template <typename T>
int ensure(fdf_ctx* ctx, T** buf, size_t* have, size_t need, hipStream_t stream) {
    if (*have >= need) return FDF_OK;
    if (*buf) {
        wait_done(ctx);
        (void)hipStreamSynchronize(stream);
        (void)hipFree(*buf);
        *buf = nullptr;
        *have = 0;
    }
    const size_t n = need + need / 8;
    if (hipMalloc(reinterpret_cast<void**>(buf), n * sizeof(T)) != hipSuccess) {
        *buf = nullptr;
        return FDF_ERR_ALLOC;
    }
    *have = n;
    return FDF_OK;
}

// Grow a pinned, device-mapped host buffer to `need` elements (+1/8 headroom); *dev is its
// device address.  Like ensure(), everything the context enqueued is drained first.
template <typename T>
int ensure_host(fdf_ctx* ctx, T** buf, T** dev, size_t* have, size_t need, hipStream_t stream) {
    if (*have >= need) return FDF_OK;
    if (*buf) {
        wait_done(ctx);
        (void)hipStreamSynchronize(stream);
        (void)hipHostFree(*buf);
        *buf = *dev = nullptr;
        *have = 0;
    }
    const size_t n = need + need / 8;
    void* hp = nullptr;
    void* dp = nullptr;
    if (hipHostMalloc(&hp, n * sizeof(T), hipHostMallocMapped) != hipSuccess) return FDF_ERR_ALLOC;
    if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
        (void)hipHostFree(hp);
        return FDF_ERR_ALLOC;
    }
    *buf = static_cast<T*>(hp);
    *dev = static_cast<T*>(dp);
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


Geometry pick_geometry(uint32_t n_frames, uint32_t w, uint32_t h, uint32_t nms,
                       uint64_t slots, double density, uint32_t forced_rows,
                       bool host_src = false) {
    Geometry g;
    const uint32_t sc = (uint32_t)fdfk::strip_cols(fdfk::kLaneCols);
    g.nstrips = (w - 3 + sc - 1) / sc;
    // >= 4 units per band (one per wave), handed out dynamically; taller units (fewer halo
    // rows) measured faster than more, shorter units for balance
    g.nsub = (4 + g.nstrips - 1) / g.nstrips;
#ifdef FDF_DEBUG_BUILD   // ablation builds only (libfdf_debug.so)
    if (const char* e = std::getenv("FDF_NSUB")) g.nsub = std::max(1ul, std::strtoul(e, nullptr, 0));
#endif
    const uint32_t centre_rows = h - 6;
    const uint32_t nw = fdfk::bitmap_words_per_row(w);
    // extra rows a unit tests: NMS bands test one row above and below (first / last unit)
    const uint32_t halo = fdfk::band_halo(nms) * (g.nsub == 1 ? 2u : 1u);
    // LDS per workgroup sets the workgroups per CU: <= 40 KB keeps 4.
    // Without NMS a 35 KB budget (bands of ~122 rows at 1080p) measured faster than the
    // tallest band that fits (more, shorter workgroups: a shorter grid tail).
    uint32_t budget = (nms ? 40000u : 35000u);
#ifdef FDF_DEBUG_BUILD
    if (const char* b = std::getenv("FDF_LDS_BUDGET"))
        budget = std::min<uint32_t>(fdfk::kSweepMaxLds, (uint32_t)std::strtoul(b, nullptr, 0));
#endif
    // The band height with the shortest modelled launch (in sweep-step units): every unit
    // costs its steps plus kUnitCost (prologue, flush, unit hand-out), every workgroup
    // kBandCost more (LDS clear, NMS pass, emit), and the grid runs on `slots` workgroup
    // slots at once -- time = max(total / slots, one workgroup) + half a workgroup of tail
    // (workgroups of one height differ with their rows' content, up to ~1.5x).  So a grid
    // that cannot fill the chip takes the shortest bands (lowest latency), a large batch
    // the tallest that waste no padding steps, and a grid near one round of the chip neither
    // spills into a second round nor leaves slots idle.  slots = 1 (fdf_ctx_set_geometry,
    // tests) gives a small job the full-size geometry (tall bands, long units); the
    // keypoints are the same either way.
    // NMS: when an earlier launch of this configuration measured the keypoint density, keep
    // a band's expected keypoints (x1.2) within the LDS score list, so that few bands
    // spill (4K t=8 n=12 SAD: 38-row bands; margins 1.5 / 1.2 / 1.0 / 0.8 measured 0.726 /
    // 0.716 / 0.715 / 0.730 ms, profiles/r03/l4_margin_4k.json)
    uint32_t max_rows = 256;
    double margin = 1.2;
#ifdef FDF_DEBUG_BUILD
    if (const char* e = std::getenv("FDF_DENSITY_MARGIN")) margin = std::strtod(e, nullptr);
#endif
    if (nms && density > 0.0 && margin > 0.0) {
        const double rows = (double)fdfk::kScoreListCap / (margin * density * (double)w) - 2.0;
        max_rows = rows < (double)g.nsub ? g.nsub : (rows > 256.0 ? 256u : (uint32_t)rows);
    }
    if (forced_rows) {   // fdf_ctx_set_band_rows: the height asked for, as far as LDS allows
        g.R = (forced_rows + g.nsub - 1) / g.nsub * g.nsub;
        while (g.R > g.nsub && fdfk::make_sweep_layout(g.R, nw, nms).total > fdfk::kSweepMaxLds)
            g.R -= g.nsub;
        return g;
    }
    constexpr double kUnitCost = 3.0;
    const double band_cost = nms ? 4.0 : 2.0;
    const uint32_t units_per_wave = (g.nstrips * g.nsub + fdfk::kWaves - 1) / fdfk::kWaves;
    // A grid that fits one round of the chip (a single frame) is latency-bound, one wave per
    // SIMD: a unit's padding steps past its last row (the sweep runs whole 8-step blocks) load
    // nothing and cost a quarter of a real step, and every band's look-back polls the
    // descriptors of the bands before it, one round per 64.  Measured on one device-resident
    // 1080p frame (profiles/r05/e7_single_frame_rows/, sweep us at 4 / 6 / 8 / 10 / 14 / 20 rows):
    // max-t 19.0 / 17.2 / 17.8 / 18.1 / 19.4 / 22.6, NMS off 15.0 / 13.3 / 13.4 / 13.5 / 13.9 /
    // 17.1 -- this model picks 6 rows for both (14 and 16 before).  A frame read in place over
    // PCIe keeps the full-step model: its halo rows cost PCIe bytes, and 6-10 rows measured
    // within noise of 14 there (r5_e8_host_rows_*.json).
    auto wg_cost = [&](uint32_t rows, bool latency) {
        const uint32_t unit_rows = (rows + g.nsub - 1) / g.nsub;
        const double steps = (double)fdfk::sweep_steps(unit_rows, halo);
        const double real = std::min(steps, (double)(unit_rows + halo));
        return units_per_wave * ((latency ? real + 0.25 * (steps - real) : steps) + kUnitCost) +
               band_cost;
    };
    const uint64_t one_round = std::min<uint64_t>(slots, fdfk::kDirectMaxTasks);
    auto pick = [&](bool latency) {
        double best = 0.0;
        uint32_t best_R = 0;
        for (uint32_t R = g.nsub; R <= max_rows && R < centre_rows + g.nsub; R += g.nsub) {
            if (fdfk::make_sweep_layout(R, nw, nms).total > budget) break;
            const uint32_t bands = (centre_rows + R - 1) / R;
            const uint64_t ntasks = (uint64_t)n_frames * bands;
            if (latency && ntasks > one_round) continue;   // stays one round of the chip
            const double lookback = latency ? (double)((ntasks + 63) / 64) : 0.0;
            const double full = wg_cost(R, latency) + lookback;
            const double last = wg_cost(centre_rows - (bands - 1) * R, latency) + lookback;
            const double total = (double)n_frames * ((bands - 1) * full + last);
            const double t = std::max(total / (double)slots, full) + 0.5 * full;
            if (best_R == 0 || t <= best * 1.001) {  // ties: the taller band (fewer workgroups)
                best = t;
                best_R = R;
            }
        }
        return best_R;
    };
    g.R = pick(false);
    // the grid of that height fits one round of the chip: the latency model picks among the
    // heights that keep it so
    if (!host_src && g.R && (uint64_t)n_frames * ((centre_rows + g.R - 1) / g.R) <= one_round) {
        const uint32_t r = pick(true);
        if (r) g.R = r;
    }
    if (g.R == 0) g.R = g.nsub;
    return g;
}

// Enqueue detection + compaction over `n_frames` device frames (w, h >= 7) on `stream`,
// after the context's previous device work (which may have run on another stream: the
// workspace is shared).
// The direct output's look-back error word (h_stats[1]): set by a band whose wait ran out.
volatile uint32_t* lookback_error_word(fdf_ctx* ctx) {
    return ctx->h_stats ? reinterpret_cast<volatile uint32_t*>(ctx->h_stats + 1) : nullptr;
}

// Takes (reads and clears) the look-back error word: bit 0 a direct-output band's look-back
// ran out, bit 1 a band's wait for its upload chunk, bit 2 a workgroup's start ticket lay
// past its grid (the device counter and ticket_next disagree: both are reset).
uint32_t take_lookback_error(fdf_ctx* ctx) {
    volatile uint32_t* e = lookback_error_word(ctx);
    if (!e || *e == 0) return 0;
    const uint32_t v = *e;
    *e = 0;
    if (v & 4u) ctx->sums_dirty = true;
    return v;
}

// The overlapped upload's copy stream and chunk flags (created on first use).
int ensure_chunk_flags(fdf_ctx* ctx) {
    if (!ctx->copy_stream &&
        hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess) {
        ctx->copy_stream = nullptr;
        return FDF_ERR_DEVICE;
    }
    if (!ctx->h_flags) {
        void* hp = nullptr;
        void* dp = nullptr;
        if (hipHostMalloc(&hp, kMaxChunks * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
            return FDF_ERR_ALLOC;
        if (hipMalloc(&dp, kMaxChunks * sizeof(uint32_t)) != hipSuccess ||
            hipMemset(dp, 0, kMaxChunks * sizeof(uint32_t)) != hipSuccess) {
            (void)hipHostFree(hp);
            if (dp) (void)hipFree(dp);
            return FDF_ERR_ALLOC;
        }
        std::memset(hp, 0, kMaxChunks * sizeof(uint32_t));
        ctx->h_flags = static_cast<uint32_t*>(hp);
        ctx->d_flags = static_cast<uint32_t*>(dp);
    }
    return FDF_OK;
}

// Workgroups one CU holds of the detector instance for (nms, n) with `lds` bytes of LDS, from
// the runtime's occupancy calculator (registers, LDS, waves), cached per configuration.
uint32_t wg_per_cu(fdf_ctx* ctx, uint32_t nms, uint32_t n, uint32_t lds, bool rgb) {
    for (const auto& o : ctx->occupancy)
        if (o.nms == nms && o.n == n && o.lds == lds && o.rgb == rgb) return o.wg;
    int wg = 0;
    if (fdfk::sweep_occupancy(nms, n, lds, rgb, &wg) != hipSuccess || wg <= 0)
        wg = (int)std::min<uint32_t>(4u, fdfk::kSweepMaxLds / std::max(lds, 1u));   // LDS bound only
    ctx->occupancy.push_back({nms, n, lds, rgb, (uint32_t)wg});
    return (uint32_t)wg;
}

struct ChunkedUpload {
    const uint32_t* flags = nullptr;   // device address of the chunk flags (NULL: none)
    uint32_t rows = 0, epoch = 0;
};

int enqueue(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames, uint32_t w, uint32_t h,
            uint64_t frame_stride, const fdf_config* cfg, uint2* d_out, uint64_t cap,
            uint64_t* d_offsets, hipStream_t stream, bool rgb = false,
            const ChunkedUpload& up = ChunkedUpload{}, bool host_src = false) {
    double density = 0.0;
    if (!ctx->h_stats) {
        void* hp = nullptr;
        void* dp = nullptr;
        if (hipHostMalloc(&hp, 64, hipHostMallocMapped) == hipSuccess &&
            hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) {
            ctx->h_stats = static_cast<uint64_t*>(hp);
            ctx->d_stats = static_cast<uint64_t*>(dp);
            std::memset(hp, 0, 64);
        } else if (hp) {
            (void)hipHostFree(hp);
        }
    }
    if (cfg->nms) {
        if (ctx->h_stats) {
            const uint64_t v = *reinterpret_cast<volatile uint64_t*>(ctx->h_stats);
            const uint32_t seq = (uint32_t)(v >> 32);
            const fdf_ctx::LaunchInfo& li = ctx->hist[seq % 64];
            if (seq != 0 && li.seq == seq && li.pixels > 0) {
                ctx->known[li.nms % 3] = li;
                ctx->known_density[li.nms % 3] = (double)(uint32_t)v / li.pixels;
            }
            const fdf_ctx::LaunchInfo& k = ctx->known[cfg->nms % 3];
            if (k.seq != 0 && k.t == cfg->threshold && k.n == cfg->count && k.nms == cfg->nms &&
                k.w == w)
                density = ctx->known_density[cfg->nms % 3];
        }
    }
    // workgroup slots of the device: 4 per CU (4 waves per SIMD); fdf_ctx_set_geometry's
    // min_tasks replaces it (1: the tall bands of a large batch for any job)
    const uint64_t per_cu = 4;
    const uint64_t slots = ctx->min_tasks ? ctx->min_tasks
                                          : (ctx->cus ? per_cu * ctx->cus : kDefaultMinTasks);
    const Geometry geo = pick_geometry(n_frames, w, h, cfg->nms, slots, density, ctx->band_rows,
                                       host_src);
    const uint32_t R = geo.R;
    const uint32_t nw = fdfk::bitmap_words_per_row(w);
#ifdef FDF_DEBUG_BUILD
    if (std::getenv("FDF_GEOMETRY_LOG"))
        std::fprintf(stderr, "fdf geometry: %u x %ux%u nms=%u t=%u n=%u density=%.5f R=%u nsub=%u\n",
                     n_frames, w, h, (unsigned)cfg->nms, (unsigned)cfg->threshold,
                     (unsigned)cfg->count, density, R, geo.nsub);
#endif
    if (fdfk::make_sweep_layout(R, nw, cfg->nms).total > fdfk::kSweepMaxLds)
        return FDF_ERR_SIZE;
    const uint32_t bands = (h - 6 + R - 1) / R;
    const uint64_t ntasks = (uint64_t)bands * n_frames;
    if (ntasks == 0 || ntasks > 0x7fffffffull) return FDF_ERR_SIZE;
    // A grid too small to fill the chip (a single frame) is latency-bound: its slots hold 4x
    // the points (6% of the band's pixels instead of 1.6%), so that dense bands stay point
    // lists and the compaction takes no bitmap expansion (a few hundred KB per frame)
    // (fdf_ctx_set_geometry's forced full-size geometry keeps the full-size slots too)
    const uint64_t fill = ctx->min_tasks ? ctx->min_tasks : kDefaultMinTasks;
    const uint32_t slot_bytes = fdfk::slot_bytes_for(R, nw) * (ntasks < fill ? 4u : 1u);
    uint32_t tpg = fdfk::compact_tasks_per_group((uint32_t)ntasks);
    uint32_t flags = 0;
#ifdef FDF_DEBUG_BUILD   // ablation builds only (libfdf_debug.so), see fdf_kernels.h
    if (const char* e = std::getenv("FDF_COMPACT_TPG"))
        tpg = std::max(1u, std::min((uint32_t)fdfk::kCompactTasks, (uint32_t)std::strtoul(e, nullptr, 0)));
    if (const char* dbg = std::getenv("FDF_DEBUG_FLAGS")) flags = (uint32_t)std::strtoul(dbg, nullptr, 0);
#endif
    if (!ctx->done &&
        hipEventCreateWithFlags(&ctx->done, hipEventDisableTiming) != hipSuccess) {
        ctx->done = nullptr;
        return FDF_ERR_DEVICE;
    }
    if (ctx->done_valid && ctx->done_stream != stream &&
        (record_done(ctx) != hipSuccess || hipStreamWaitEvent(stream, ctx->done, 0) != hipSuccess))
        return FDF_ERR_DEVICE;
    int rc;
    if ((rc = ensure(ctx, &ctx->d_slots, &ctx->slots_bytes, (size_t)(ntasks * slot_bytes), stream))) return rc;
    if ((rc = ensure(ctx, &ctx->d_counts, &ctx->counts_n, (size_t)ntasks, stream))) return rc;
    if (!ctx->d_sums) {
        if (hipMalloc(reinterpret_cast<void**>(&ctx->d_sums),
                      (2 * fdfk::kMaxGroupSums + 4) * sizeof(uint32_t)) != hipSuccess) {
            ctx->d_sums = nullptr;
            return FDF_ERR_ALLOC;
        }
        ctx->sums_dirty = true;
    }
    if (ctx->sums_dirty) {
        if (hipMemsetAsync(ctx->d_sums, 0, (2 * fdfk::kMaxGroupSums + 4) * sizeof(uint32_t),
                           stream) != hipSuccess)
            return FDF_ERR_DEVICE;
        ctx->sums_dirty = false;
        ctx->ticket_next = 0;                       // the ticket counter is zero again
    }
    // detection and compaction are two launches: a compaction fused into the detector's last
    // workgroup measured 87 us for one frame against 13 + 12 us (every workgroup's device-scope
    // release is an L2 writeback on gfx950)
    // Small grids write their points directly (look-back, no compaction launch) when every
    // workgroup is resident at once -- by the occupancy calculator for this instance and LDS
    // size (4 per CU at 4 waves per SIMD) -- so that a band's look-back only waits for bands
    // running beside it.  (Correctness does not depend on it: bands are numbered by their
    // start tickets, band_lookback.)
    const fdfk::SweepLayout lay = fdfk::make_sweep_layout(R, nw, cfg->nms);
    const uint32_t wgs = wg_per_cu(ctx, cfg->nms, cfg->count, lay.total, rgb);
    bool direct = ntasks <= std::min<uint64_t>(fdfk::kDirectMaxTasks, (uint64_t)ctx->cus * wgs);
#ifdef FDF_DEBUG_BUILD
    if (const char* e = std::getenv("FDF_DIRECT")) direct = direct && std::strtoul(e, nullptr, 0) != 0;
#endif
    const uint64_t ngroups = (ntasks + tpg - 1) / tpg;
    const bool grouped = !direct && ngroups <= fdfk::kMaxGroupSums;
    uint32_t* sums_now = ctx->d_sums + (size_t)ctx->sums_parity * fdfk::kMaxGroupSums;
    uint32_t* sums_next = ctx->d_sums + (size_t)(1 - ctx->sums_parity) * fdfk::kMaxGroupSums;
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
    p.flags = flags;
    p.nstrips = geo.nstrips;
    p.nsub = geo.nsub;
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
    c.group_sums = grouped ? sums_now : nullptr;
    c.next_sums = sums_next;
    p.group_sums = grouped ? sums_now : nullptr;
    p.tasks_per_group = tpg;
    p.kp_stats = nullptr;
    p.stamps = nullptr;
    p.direct = direct ? 1u : 0u;
    p.epoch = 0;
    p.lookback = nullptr;
    p.out = d_out;
    p.cap = cap;
    p.frame_offsets = d_offsets;
    p.ticket = ctx->d_sums + 2 * fdfk::kMaxGroupSums + 2;
    p.ticket_base = ctx->ticket_next;
    p.lookback_error = ctx->h_stats ? reinterpret_cast<uint32_t*>(ctx->d_stats + 1) : nullptr;
    p.chunk_flags = up.flags;
    p.chunk_rows = up.rows;
    p.chunk_epoch = up.epoch;
    if (direct) {
        // a (re)allocated buffer is zeroed: recycled device memory can hold descriptors of
        // another context's launches.  Launch tags are unique in the process as well.
        const size_t had = ctx->lookback_n;
        if ((rc = ensure(ctx, &ctx->d_lookback, &ctx->lookback_n, (size_t)ntasks, stream))) return rc;
        if (ctx->lookback_n != had &&
            hipMemsetAsync(ctx->d_lookback, 0, ctx->lookback_n * sizeof(uint64_t), stream) != hipSuccess)
            return FDF_ERR_DEVICE;
        p.lookback = ctx->d_lookback;
        uint32_t e = ++g_launch_epoch;
        if (e == 0) e = ++g_launch_epoch;                          // 0 = a zeroed descriptor
        p.epoch = e;
    }
#ifdef FDF_DEBUG_BUILD
    if (std::getenv("FDF_STAMPS")) {
        const size_t words = (size_t)ntasks * fdfk::kStampWords;
        if ((rc = ensure(ctx, &ctx->d_stamps, &ctx->stamps_n, words, stream))) return rc;
        p.stamps = ctx->d_stamps;
        ctx->stamps_used = words;
    }
#endif
    c.kp_stats = nullptr;
    c.stats_out = nullptr;
    c.stats_seq = 0;
    if (cfg->nms && ctx->h_stats && !direct) {
        const uint32_t seq = ++ctx->stats_seq == 0 ? ++ctx->stats_seq : ctx->stats_seq;
        fdf_ctx::LaunchInfo& li = ctx->hist[seq % 64];
        li.seq = seq;
        li.t = cfg->threshold;
        li.n = cfg->count;
        li.nms = cfg->nms;
        li.w = w;
        li.pixels = (double)n_frames * (double)w * (double)(h - 6);
        p.kp_stats = ctx->d_sums + 2 * fdfk::kMaxGroupSums + 1;
        c.kp_stats = p.kp_stats;
        c.stats_out = ctx->d_stats;
        c.stats_seq = seq;
    }
    // per-kernel timing: 4 events per call, timestamped by the dispatches themselves
    // (hipExtLaunchKernelGGL), so no marker packets sit between the kernels
    hipEvent_t* ev = nullptr;
    if (ctx->timing && ctx->timing_calls++ % ctx->timing == 0 && ctx->timed < kMaxTimedCalls) {
        while (ctx->ev.size() < 4 * (ctx->timed + 1)) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return FDF_ERR_DEVICE;
            ctx->ev.push_back(e);
        }
        ev = &ctx->ev[4 * ctx->timed];
    }
    // a small grid whose units are shorter than one 8-step block (a single frame's latency
    // bands) runs the instances that leave the block at the unit's last row
    // (fdf_sweep_latency.hip; 1080p NMS off 13.5 -> 12.5 us, max-t 17.3 -> 17.0 us per frame).
    // Long units keep whole blocks: the exit tests cost the batch loop more than the padding
    // steps they save (512 x 1080p NMS off, 61-row units: +0.6 %, profiles/r05/e16_*)
    const uint32_t unit_steps = (R + geo.nsub - 1) / geo.nsub +
                                fdfk::band_halo(cfg->nms) * (geo.nsub == 1 ? 2u : 1u);
    const bool exit_in_block = !rgb && direct && unit_steps < fdfk::kSweepRing;
    auto launch = rgb ? fdfk::launch_sweep_rgb
                      : (exit_in_block ? fdfk::launch_sweep_latency : fdfk::launch_sweep);
    if (launch(p, cfg->nms, cfg->count, stream, ev ? ev[0] : nullptr, ev ? ev[1] : nullptr) !=
        hipSuccess) {
        ctx->sums_dirty = true;
        return FDF_ERR_DEVICE;
    }
    if (direct) ctx->ticket_next += (uint32_t)ntasks;   // the launch takes one per workgroup
    if (!direct && fdfk::launch_compact(c, stream, ev ? ev[2] : nullptr, ev ? ev[3] : nullptr) !=
                       hipSuccess) {
        ctx->sums_dirty = true;
        return FDF_ERR_DEVICE;
    }
    if (grouped) ctx->sums_parity ^= 1;
    if (ev) {
        if (ctx->timed_compact.size() <= ctx->timed) ctx->timed_compact.resize(ctx->timed + 1);
        ctx->timed_compact[ctx->timed] = direct ? 0 : 1;
        ++ctx->timed;
    }
    ctx->last_compact = c;
    if (note_done(ctx, stream) != hipSuccess) return FDF_ERR_DEVICE;
    return FDF_OK;
}

// The score reported with a keypoint: the NMS mode's own, max-threshold when NMS is off.
uint32_t score_kind(uint32_t nms) {
    return nms == FDF_NMS_SUM_ABSOLUTE ? FDF_NMS_SUM_ABSOLUTE : FDF_NMS_MAX_THRESHOLD;
}
// ~4 points per thread on average, 1..64 workgroups per frame.
uint32_t score_blocks(uint64_t points, uint32_t n_frames) {
    const uint64_t per_frame = points / std::max<uint32_t>(n_frames, 1u);
    return (uint32_t)std::min<uint64_t>(64, per_frame / 1024 + 1);
}

// Validation shared by the host entry points; *empty = the reference returns no points.
int check_host_args(const uint8_t* data, uint32_t n_frames, uint32_t w, uint32_t h,
                    size_t row_stride, const fdf_config* cfg, bool rgb, int* empty) {
    int rc = check_config(cfg);
    if (rc) return rc;
    rc = check_shape(w, h, empty);
    if (rc) return rc;
    if (n_frames == 0) *empty = 1;
    if (!data && !*empty) return FDF_ERR_ARG;
    if (row_stride < (rgb ? 3ull * w : (size_t)w)) return FDF_ERR_ARG;
    return FDF_OK;
}

// Phase 1 of a host detection (lock held): frames in, detection + compaction into the
// context's output buffer, frame offsets back to the host (`offs`, n_frames + 1 entries).
// The output starts small and grows to the keypoint total; when it has to grow only the
// compaction is run again (the per-band slots still hold the detection).  On success
// ctx->last describes the result, which stays in the context until the next host call.
// `host_out`: the output is the pinned, device-mapped h_out / h_offs (the kernels write the
// points and offsets into host memory: no copy back, one synchronisation); otherwise the
// device buffers d_out / d_offsets (the scored calls, whose score kernel reads the points).
// `rgb`: the frames are RGB8 (rows of 3 * w bytes at row_stride), converted on the device
// with image 0.24.6's to_luma8 before detection (src/main.rs:58).
int run_host(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames, uint32_t w, uint32_t h,
             size_t row_stride, size_t frame_stride, const fdf_config* cfg, bool rgb,
             uint64_t* offs, bool host_out) {
    ctx->last = LastResult{};          // invalid, and not a shard of a multi-context call
    const size_t frame_bytes = (size_t)w * h;
    const size_t max_points = (size_t)(w - 6) * (h - 6) * n_frames;
    // first guess: 1 keypoint per 64 pixels (real images: 0.5-1.5 per 100)
    const size_t guess = std::min(max_points, std::max<size_t>(4096, frame_bytes / 64 * n_frames));
    int rc;
    if ((rc = ensure(ctx, &ctx->d_in, &ctx->in_bytes, frame_bytes * n_frames, ctx->stream))) return rc;
    uint2* out_dev;                    // the output as the kernels address it
    uint64_t* offs_dev;
    size_t* out_cap;
    if (host_out) {
        if ((rc = ensure_host(ctx, &ctx->h_out, &ctx->hd_out, &ctx->h_out_points, guess, ctx->stream)))
            return rc;
        if ((rc = ensure_host(ctx, &ctx->h_offs, &ctx->hd_offs, &ctx->h_offs_n, n_frames + 1ull,
                              ctx->stream)))
            return rc;
        out_dev = ctx->hd_out;
        offs_dev = ctx->hd_offs;
        out_cap = &ctx->h_out_points;
    } else {
        if ((rc = ensure(ctx, &ctx->d_out, &ctx->out_points, guess, ctx->stream))) return rc;
        if ((rc = ensure(ctx, &ctx->d_offsets, &ctx->offsets_n, n_frames + 1ull, ctx->stream)))
            return rc;
        out_dev = ctx->d_out;
        offs_dev = ctx->d_offsets;
        out_cap = &ctx->out_points;
    }
    const size_t px = rgb ? 3 : 1;                 // bytes per pixel of the host frames
    uint8_t* stage = ctx->d_in;
    if (rgb) {
        if ((rc = ensure(ctx, &ctx->d_rgb, &ctx->rgb_bytes, 3 * frame_bytes * n_frames, ctx->stream)))
            return rc;
        stage = ctx->d_rgb;
    }
    // the host frames are read by the copies below: nothing else may still read d_in (nor
    // the host output, which the host reads after this call)
    wait_done(ctx);
    // an error an earlier asynchronous fdf_detect_device left in the error word belongs to
    // that call: keep it for the next device call, so this call's own check sees only its own
    if (take_lookback_error(ctx)) ctx->pending_device_error = true;
    // one grey frame of >= kChunkMinBytes: upload it in row chunks on the copy stream while
    // the detector runs, each band waiting for the chunk of its last row (the H2D of a 1080p
    // frame is ~45 us, the detector ~20 us: DESIGN.md §7.5)
    ChunkedUpload up;
#ifdef FDF_DEBUG_BUILD   // A/B of the overlapped upload (tools/host_latency.py): FDF_CHUNKS=1 disables it
    if (const char* e = std::getenv("FDF_CHUNKS")) ctx->chunks = (uint32_t)std::strtoul(e, nullptr, 0);
#endif
    // (the chunk count in effect must be > 1: one chunk is one copy before the launch, which
    // the plain path below does without the flag copy and the second stream)
    const uint32_t nchunks_eff = std::min<uint32_t>(ctx->chunks ? ctx->chunks : kChunksDefault,
                                                    kMaxChunks);
    const bool chunked = host_out && !rgb && n_frames == 1 && frame_bytes >= kChunkMinBytes &&
                         nchunks_eff > 1 && ctx->h_stats && ensure_chunk_flags(ctx) == FDF_OK;
    // one packed grey frame in pinned (page-locked, non-coherent) host memory, unscored: the
    // detector reads it in place over PCIe, with no copy before the launch -- its row stream
    // is the upload (1080p max-t 72-75 vs 82-83 us end to end).  Host writes
    // to the buffer before the call are visible to the launch (the dispatch's system-scope
    // acquire; a wave-level acquire fence cost ~20 us and changed no result:
    // tests/test_gpu_host_inplace.py reuses one buffer for different frames).  The frame is
    // then not in d_in: a result that does not fit the caller's buffer copies it there for
    // fdf_fetch_last (detect_host).
    const uint8_t* in_place = nullptr;
    if (ctx->chunks == 0 && host_out && !rgb && n_frames == 1 && row_stride == w) {
        // the frame's first and last bytes must both be pinned and map to one contiguous
        // device range: a hipHostRegister'ed sub-range shorter than the frame is copied, not
        // read past its end
        hipPointerAttribute_t a, z;
        if (hipPointerGetAttributes(&a, data) == hipSuccess) {
            if (a.type == hipMemoryTypeHost && a.devicePointer &&
                !(a.allocationFlags & hipHostMallocCoherent)) {
                const uint8_t* last = data + frame_bytes - 1;
                if (hipPointerGetAttributes(&z, last) == hipSuccess) {
                    if (z.type == hipMemoryTypeHost && z.devicePointer &&
                        static_cast<const uint8_t*>(z.devicePointer) ==
                            static_cast<const uint8_t*>(a.devicePointer) + (frame_bytes - 1))
                        in_place = static_cast<const uint8_t*>(a.devicePointer);
                } else {
                    (void)hipGetLastError();   // the frame runs past the pinned range
                }
            }
        } else {
            (void)hipGetLastError();   // pageable memory: not an error here
        }
    }
    // frames that start in pinned host memory must lie inside one pinned mapping for the DMA
    // copies below (the chunked upload's too); a range that runs past it is packed into the
    // pinned staging buffer first
    if (!in_place) {
        const size_t span = (size_t)(n_frames - 1) * frame_stride + (size_t)(h - 1) * row_stride +
                            px * w;
        hipPointerAttribute_t a, z;
        if (hipPointerGetAttributes(&a, data) == hipSuccess) {
            if (a.type == hipMemoryTypeHost && a.devicePointer) {
                const bool inside =
                    hipPointerGetAttributes(&z, data + span - 1) == hipSuccess &&
                    z.type == hipMemoryTypeHost &&
                    static_cast<const uint8_t*>(z.devicePointer) ==
                        static_cast<const uint8_t*>(a.devicePointer) + (span - 1);
                if (!inside) {
                    (void)hipGetLastError();
                    const size_t fb = px * frame_bytes;
                    if ((rc = ensure_host(ctx, &ctx->h_stage, &ctx->hd_stage, &ctx->h_stage_bytes,
                                          fb * n_frames, ctx->stream)))
                        return rc;
                    for (uint32_t f = 0; f < n_frames; ++f)
                        for (uint32_t y = 0; y < h; ++y)
                            std::memcpy(ctx->h_stage + f * fb + (size_t)y * px * w,
                                        data + f * frame_stride + (size_t)y * row_stride, px * w);
                    data = ctx->h_stage;
                    row_stride = px * w;
                    frame_stride = fb;
                }
            }
        } else {
            (void)hipGetLastError();   // pageable memory
        }
    }
    if (in_place) {
    } else if (chunked) {
        up.rows = (h + nchunks_eff - 1) / nchunks_eff;
        up.epoch = ++ctx->chunk_epoch == 0 ? ++ctx->chunk_epoch : ctx->chunk_epoch;
        up.flags = ctx->d_flags;
        for (uint32_t r0 = 0, c = 0; r0 < h; r0 += up.rows, ++c) {
            const uint32_t nr = std::min(up.rows, h - r0);
            const uint8_t* src = data + (size_t)r0 * row_stride;
            uint8_t* dst = ctx->d_in + (size_t)r0 * w;
            hipError_t e = row_stride == w
                               ? hipMemcpyAsync(dst, src, (size_t)nr * w, hipMemcpyHostToDevice,
                                                ctx->copy_stream)
                               : hipMemcpy2DAsync(dst, w, src, row_stride, w, nr,
                                                  hipMemcpyHostToDevice, ctx->copy_stream);
            // the chunk's flag: a 4-byte copy behind it on the same (copy-engine) queue --
            // hipStreamWriteValue32 is a kernel launch per call on this runtime (~20 us each)
            ctx->h_flags[c] = up.epoch;
            if (e == hipSuccess)
                e = hipMemcpyAsync(ctx->d_flags + c, ctx->h_flags + c, sizeof(uint32_t),
                                   hipMemcpyHostToDevice, ctx->copy_stream);
            if (e != hipSuccess) {
                // the runtime cannot do this upload: this call takes one copy before the
                // launch (counted; the caller's chunk setting stays)
                (void)hipStreamSynchronize(ctx->copy_stream);
                (void)hipGetLastError();
                ++ctx->upload_fallbacks;
                const uint32_t saved = ctx->chunks;
                ctx->chunks = 1;
                rc = run_host(ctx, data, n_frames, w, h, row_stride, frame_stride, cfg, rgb,
                              offs, host_out);
                ctx->chunks = saved;
                return rc;
            }
        }
    } else {
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
    }
    // RGB: a luma pass, then the grey detector.  The detector with luma converted in its
    // loads (fdf_detect_device_rgb) is correct but measured 1.6x slower on 256 1080p frames:
    // its 48-byte row loads need 12 registers each until converted, which spills and
    // exposes the row latency
    if (rgb && fdfk::launch_rgb_to_luma(ctx->d_rgb, n_frames, (uint32_t)frame_bytes,
                                        3 * frame_bytes, ctx->d_in, ctx->stream) != hipSuccess)
        return FDF_ERR_DEVICE;
    rc = enqueue(ctx, in_place ? in_place : ctx->d_in, n_frames, w, h, frame_bytes, cfg,
                 out_dev, *out_cap, offs_dev, ctx->stream, false, up, in_place != nullptr);
    if (chunked) {
        // the copies end before the detector does (it waits for the last one), but a failed
        // launch or a timed-out wait would leave them running: drain them before any return
        const hipError_t e = hipStreamSynchronize(ctx->copy_stream);
        if (!rc && e != hipSuccess) rc = FDF_ERR_DEVICE;
    }
    if (rc) return rc;
    // the offsets on the host: read in place (host output) or copied back
    auto fetch_offsets = [&]() -> hipError_t {
        hipError_t e = hipSuccess;
        if (!host_out)
            e = hipMemcpyAsync(offs, offs_dev, sizeof(uint64_t) * (n_frames + 1ull),
                               hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = sync_own_stream(ctx);
        if (e == hipSuccess && host_out)
            std::memcpy(offs, ctx->h_offs, sizeof(uint64_t) * (n_frames + 1ull));
        return e;
    };
    if (fetch_offsets() != hipSuccess) return FDF_ERR_DEVICE;
    if (const uint32_t err = take_lookback_error(ctx)) {
        if (err & 4u) return FDF_ERR_DEVICE;   // a band never ran: nothing to rebuild from
        if (err & 2u) {
            // a band's wait for its upload chunk ran out (the copies are drained now): detect
            // again from the whole frame, uploaded before the launch
            ++ctx->upload_fallbacks;
            const uint32_t saved = ctx->chunks;
            ctx->chunks = 1;
            rc = run_host(ctx, data, n_frames, w, h, row_stride, frame_stride, cfg, rgb, offs,
                          host_out);
            ctx->chunks = saved;
            return rc;
        }
        // a direct-output band's look-back ran out (band_lookback): the offsets and points of
        // its frame on are not written; the slots and counts are, so the compaction rebuilds
        // both from them
        ++ctx->lookback_recoveries;
        fdfk::CompactParams c = ctx->last_compact;
        c.kp_stats = nullptr;
        c.group_sums = nullptr;
        if (fdfk::launch_compact(c, ctx->stream) != hipSuccess || fetch_offsets() != hipSuccess)
            return FDF_ERR_DEVICE;
    }
    const uint64_t total = offs[n_frames];
    if (total > *out_cap) {
        // grow the output and compact again (the offsets do not change)
        fdfk::CompactParams c = ctx->last_compact;
        if (host_out) {
            if ((rc = ensure_host(ctx, &ctx->h_out, &ctx->hd_out, &ctx->h_out_points, (size_t)total,
                                  ctx->stream)))
                return rc;
            c.out = ctx->hd_out;
        } else {
            if ((rc = ensure(ctx, &ctx->d_out, &ctx->out_points, (size_t)total, ctx->stream))) return rc;
            c.out = ctx->d_out;
        }
        c.cap = host_out ? ctx->h_out_points : ctx->out_points;
        c.kp_stats = nullptr;           // already reported (and reset) by the first compaction
        if (fdfk::launch_compact(c, ctx->stream) != hipSuccess ||
            note_done(ctx, ctx->stream) != hipSuccess)
            return FDF_ERR_DEVICE;
        // the host reads h_out next: the compaction must be done
        if (host_out && sync_own_stream(ctx) != hipSuccess) return FDF_ERR_DEVICE;
    }
    ctx->last.valid = true;
    ctx->last.host_out = host_out;
    ctx->last.total = total;
    ctx->last.n_frames = n_frames;
    ctx->last.width = w;
    ctx->last.height = h;
    ctx->last.cfg = *cfg;
    ctx->last.rgb = false;          // the luma frames are in d_in
    ctx->last.in_place = in_place != nullptr;   // ... or were read in place (not in d_in)
    return FDF_OK;
}

// Phase 2 (lock held): copy the first `n` points of the last result, and their scores when
// `out_scores` is given, to the host.
int copy_out(fdf_ctx* ctx, fdf_point* out, uint16_t* out_scores, size_t n) {
    if (!n) return FDF_OK;
    const LastResult& L = ctx->last;
    if (out_scores && L.in_place) return FDF_ERR_ARG;
    hipError_t e = hipSuccess;
    if (out_scores) {
        int rc = ensure(ctx, &ctx->d_scores, &ctx->scores_n, n, ctx->stream);
        if (rc) return rc;
        if (L.rgb) {   // the scores are computed from the luma frames
            const size_t fb = (size_t)L.width * L.height;
            if ((rc = ensure(ctx, &ctx->d_in, &ctx->in_bytes, fb * L.n_frames, ctx->stream))) return rc;
            if (fdfk::launch_rgb_to_luma(ctx->d_rgb, L.n_frames, (uint32_t)fb, 3 * fb, ctx->d_in,
                                         ctx->stream) != hipSuccess)
                return FDF_ERR_DEVICE;
        }
        // (a host-output result's points and offsets are read through their device-mapped
        // addresses)
        e = fdfk::launch_score_frames(ctx->d_in, L.width, (uint64_t)L.width * L.height,
                                      L.n_frames, L.host_out ? ctx->hd_out : ctx->d_out,
                                      L.host_out ? ctx->hd_offs : ctx->d_offsets, n,
                                      score_blocks(n, L.n_frames), score_kind(L.cfg.nms),
                                      L.cfg.threshold, L.cfg.count, ctx->d_scores, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out_scores, ctx->d_scores, n * sizeof(uint16_t),
                               hipMemcpyDeviceToHost, ctx->stream);
    }
    if (L.host_out) {
        if (e == hipSuccess && out_scores) e = sync_own_stream(ctx);
        if (e == hipSuccess) std::memcpy(out, ctx->h_out, n * sizeof(fdf_point));
        return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
    }
    if (e == hipSuccess)
        e = hipMemcpyAsync(out, ctx->d_out, n * sizeof(fdf_point), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = sync_own_stream(ctx);
    return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
}

// Shared body of fdf_detect / fdf_detect_batch / the scored and RGB variants: host frames
// in, host points out.  With `cap` below the total, the first `cap` points are written,
// FDF_ERR_CAPACITY is returned and the whole result stays on the device for fdf_fetch_last.
int detect_host(fdf_ctx* ctx, const uint8_t* data, uint32_t n_frames, uint32_t w, uint32_t h,
                size_t row_stride, size_t frame_stride, const fdf_config* cfg, fdf_point* out,
                size_t cap, uint64_t* frame_offsets, size_t* n_out, bool rgb = false,
                uint16_t* out_scores = nullptr, bool scored = false) {
    if (!ctx || !n_out || (cap && !out) || (scored && cap && !out_scores)) return FDF_ERR_ARG;
    int empty = 0;
    int rc = check_host_args(data, n_frames, w, h, row_stride, cfg, rgb, &empty);
    if (rc) return rc;
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (empty) {
        ctx->last = LastResult{};
        ctx->last.valid = true;
        ctx->last.cfg = *cfg;
        *n_out = 0;
        if (frame_offsets) std::memset(frame_offsets, 0, sizeof(uint64_t) * (n_frames + 1ull));
        return FDF_OK;
    }
    DeviceGuard guard(ctx->device);
    std::vector<uint64_t> local;
    uint64_t* offs = frame_offsets;
    if (!offs) {
        local.resize(n_frames + 1ull);
        offs = local.data();
    }
    // unscored calls take the host-mapped output (no copy back); the scored ones keep the
    // points on the device for the score kernel.  (Points written straight into a caller's
    // pinned output buffer, round 5 and again in round 6, came with an asynchronous device
    // error in a later test in 3 of 5 full GPU-suite runs: DESIGN.md §7.7.)
    rc = run_host(ctx, data, n_frames, w, h, row_stride, frame_stride, cfg, rgb, offs, !scored);
    if (rc) return rc;
    const uint64_t total = offs[n_frames];
    if (total > cap && ctx->last.in_place) {
        // the two-call pattern follows: keep the frame for fdf_fetch_last's scores
        if (hipMemcpyAsync(ctx->d_in, data, (size_t)w * h, hipMemcpyHostToDevice, ctx->stream) !=
                hipSuccess ||
            sync_own_stream(ctx) != hipSuccess)
            return FDF_ERR_DEVICE;
        ctx->last.in_place = false;
    }
    rc = copy_out(ctx, out, scored ? out_scores : nullptr, (size_t)std::min<uint64_t>(total, cap));
    if (rc) return rc;
    *n_out = (size_t)total;
    return total > cap ? FDF_ERR_CAPACITY : FDF_OK;
}

// Locks the contexts of a multi-context call in one global order (by address), whatever
// order the caller lists them in: two calls over the same contexts cannot deadlock.
std::vector<std::unique_lock<std::mutex>> lock_all(fdf_ctx* const* ctxs, uint32_t n) {
    std::vector<fdf_ctx*> order(ctxs, ctxs + n);
    std::sort(order.begin(), order.end(), std::less<fdf_ctx*>());
    std::vector<std::unique_lock<std::mutex>> locks;
    locks.reserve(n);
    for (fdf_ctx* c : order) locks.emplace_back(c->mu);
    return locks;
}


// Copy of the last host result (fdf_fetch_last), lock held.
int fetch_last(fdf_ctx* ctx, fdf_point* out, uint16_t* out_scores, size_t cap, size_t* n_out) {
    if (!ctx->last.valid) return FDF_ERR_ARG;
    DeviceGuard guard(ctx->device);
    const uint64_t total = ctx->last.total;
    *n_out = (size_t)total;
    const int rc = copy_out(ctx, out, out_scores, (size_t)std::min<uint64_t>(total, cap));
    if (rc) return rc;
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
    hipDeviceProp_t prop;
    ctx->cus = hipGetDeviceProperties(&prop, device) == hipSuccess ? (uint32_t)prop.multiProcessorCount : 0u;
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
        wait_done(ctx);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->d_in);
        (void)hipFree(ctx->d_rgb);
        (void)hipFree(ctx->d_out);
        (void)hipFree(ctx->d_offsets);
        if (ctx->h_out) (void)hipHostFree(ctx->h_out);
        if (ctx->h_offs) (void)hipHostFree(ctx->h_offs);
        if (ctx->h_flags) (void)hipHostFree(ctx->h_flags);
        if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
        (void)hipFree(ctx->d_flags);
        if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
        (void)hipFree(ctx->d_scores);
        (void)hipFree(ctx->d_slots);
        (void)hipFree(ctx->d_counts);
        (void)hipFree(ctx->d_sums);
        (void)hipFree(ctx->d_stamps);
        (void)hipFree(ctx->d_lookback);
        for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
        if (ctx->done) (void)hipEventDestroy(ctx->done);
        if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
        (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

void* fdf_ctx_stream(fdf_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int fdf_ctx_set_timing(fdf_ctx* ctx, int enable) {
    if (!ctx) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->timing = enable > 0 ? (uint32_t)enable : 0u;
    ctx->timed = 0;
    ctx->timing_calls = 0;
    return FDF_OK;
}

int fdf_ctx_workspace_bytes(fdf_ctx* ctx, uint64_t* bytes) {
    if (!ctx || !bytes) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    *bytes = ctx->in_bytes + ctx->rgb_bytes + ctx->out_points * sizeof(uint2) +
             ctx->offsets_n * sizeof(uint64_t) + ctx->scores_n * sizeof(uint16_t) +
             ctx->slots_bytes + ctx->counts_n * sizeof(uint32_t) +
             (ctx->d_sums ? (2 * fdfk::kMaxGroupSums + 4) * sizeof(uint32_t) : 0);
    return FDF_OK;
}

int fdf_ctx_recoveries(fdf_ctx* ctx, uint64_t* upload_fallbacks, uint64_t* lookback_recoveries) {
    if (!ctx) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (upload_fallbacks) *upload_fallbacks = ctx->upload_fallbacks;
    if (lookback_recoveries) *lookback_recoveries = ctx->lookback_recoveries;
    return FDF_OK;
}

int fdf_ctx_test_skew_tickets(fdf_ctx* ctx, uint32_t delta) {
    if (!ctx) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->ticket_next += delta;
    return FDF_OK;
}

int fdf_ctx_set_geometry(fdf_ctx* ctx, uint32_t min_tasks) {
    if (!ctx) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->min_tasks = min_tasks;
    return FDF_OK;
}

int fdf_ctx_set_upload_chunks(fdf_ctx* ctx, uint32_t chunks) {
    if (!ctx || chunks > kMaxChunks) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->chunks = chunks;
    return FDF_OK;
}

int fdf_ctx_set_band_rows(fdf_ctx* ctx, uint32_t rows) {
    if (!ctx || rows > kMaxBandRows) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->band_rows = rows;
    return FDF_OK;
}

// Kernel durations of recorded call k (0 for a compaction the call did not launch).
static int timed_call(fdf_ctx* ctx, size_t k, float* detect_ms, float* compact_ms) {
    const hipEvent_t* e = &ctx->ev[4 * k];
    const bool compact = k < ctx->timed_compact.size() && ctx->timed_compact[k];
    *compact_ms = 0.0f;
    if (hipEventSynchronize(e[1]) != hipSuccess ||
        hipEventElapsedTime(detect_ms, e[0], e[1]) != hipSuccess)
        return FDF_ERR_DEVICE;
    if (compact && (hipEventSynchronize(e[3]) != hipSuccess ||
                    hipEventElapsedTime(compact_ms, e[2], e[3]) != hipSuccess))
        return FDF_ERR_DEVICE;
    return FDF_OK;
}

int fdf_ctx_timing_samples(fdf_ctx* ctx, float* detect_ms, float* compact_ms, uint32_t cap,
                           uint32_t* n) {
    if (!ctx || !n || (cap && (!detect_ms || !compact_ms))) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    *n = (uint32_t)ctx->timed;
    for (size_t k = 0; k < ctx->timed && k < cap; ++k)
        if (timed_call(ctx, k, &detect_ms[k], &compact_ms[k]) != FDF_OK) return FDF_ERR_DEVICE;
    return FDF_OK;
}

int fdf_ctx_timing(fdf_ctx* ctx, uint32_t* calls, float* detect_ms, float* compact_ms) {
    if (!ctx || !calls || !detect_ms || !compact_ms) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    *calls = (uint32_t)ctx->timed;
    *detect_ms = *compact_ms = 0.0f;
    for (size_t k = 0; k < ctx->timed; ++k) {
        float a = 0.0f, b = 0.0f;
        if (timed_call(ctx, k, &a, &b) != FDF_OK) return FDF_ERR_DEVICE;
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

int fdf_fetch_last(fdf_ctx* ctx, fdf_point* out, uint16_t* out_scores, size_t cap,
                   size_t* n_out) {
    if (!ctx || !n_out || (cap && !out)) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    return fetch_last(ctx, out, out_scores, cap, n_out);
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
    // an earlier asynchronous direct-output launch of this context had a look-back wait run
    // out (band_lookback; never seen in practice): its output was incomplete -- reported once
    // (also when a host call in between found the error word first: pending_device_error)
    if (take_lookback_error(ctx) || ctx->pending_device_error) {
        ctx->pending_device_error = false;
        return FDF_ERR_DEVICE;
    }
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

int fdf_detect_device_rgb(fdf_ctx* ctx, const uint8_t* d_frames, uint32_t n_frames,
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
    const uint64_t fb = 3ull * width * height;
    if (fb > 0x7fffffffull) return FDF_ERR_SIZE;
    if (n_frames > 1 && frame_stride_bytes < fb) return FDF_ERR_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    // an earlier asynchronous direct-output launch of this context had a look-back wait run
    // out (band_lookback; never seen in practice): its output was incomplete -- reported once
    // (also when a host call in between found the error word first: pending_device_error)
    if (take_lookback_error(ctx) || ctx->pending_device_error) {
        ctx->pending_device_error = false;
        return FDF_ERR_DEVICE;
    }
    if (empty) {
        return hipMemsetAsync(d_frame_offsets, 0, sizeof(uint64_t) * (n_frames + 1ull), s) ==
                       hipSuccess
                   ? FDF_OK
                   : FDF_ERR_DEVICE;
    }
    return enqueue(ctx, d_frames, n_frames, width, height, n_frames > 1 ? frame_stride_bytes : fb,
                   cfg, reinterpret_cast<uint2*>(d_out), cap, d_frame_offsets, s, true);
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
    ctx->last.valid = false;              // d_in / d_out are reused below
    wait_done(ctx);
    int rc;
    if ((rc = ensure(ctx, &ctx->d_in, &ctx->in_bytes, frame_bytes, ctx->stream))) return rc;
    if ((rc = ensure(ctx, &ctx->d_out, &ctx->out_points, n_points + (n_points + 3) / 4,
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
    if (e == hipSuccess) e = sync_own_stream(ctx);
    return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
}

// ---- ring-level helpers (src/fast_simd.rs:69-110, :623, :722) ---------------------------

static constexpr int32_t kCircleDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
static constexpr int32_t kCircleDy[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};

void fdf_circle(int32_t dx[16], int32_t dy[16]) {
    for (int i = 0; i < 16; ++i) {
        if (dx) dx[i] = kCircleDx[i];
        if (dy) dy[i] = kCircleDy[i];
    }
}

void fdf_calculate_offsets(uint32_t width, int32_t offsets[16]) {
    if (!offsets) return;
    for (int i = 0; i < 16; ++i)   // same i32 arithmetic as the reference (wraps like it)
        offsets[i] = (int32_t)((uint32_t)kCircleDy[i] * width + (uint32_t)kCircleDx[i]);
}

static int check_ring_args(const fdf_config* cfg) {
    if (!cfg) return FDF_ERR_ARG;
    if (cfg->nms != FDF_NMS_MAX_THRESHOLD && cfg->nms != FDF_NMS_SUM_ABSOLUTE) return FDF_ERR_NMS;
    if (cfg->nms == FDF_NMS_MAX_THRESHOLD && (cfg->count < 9 || cfg->count > 16))
        return FDF_ERR_COUNT;
    return FDF_OK;
}

static inline uint8_t ring_count(const fdf_config* cfg) {
    return cfg->nms == FDF_NMS_MAX_THRESHOLD ? cfg->count : 9;   // SAD ignores the count
}

int fdf_score_rings_device(fdf_ctx* ctx, const uint8_t* d_centers, const uint8_t* d_rings,
                           uint64_t n_rings, const fdf_config* cfg, uint16_t* d_scores,
                           void* stream) {
    if (!ctx || n_rings > 0xffffffffull) return FDF_ERR_ARG;
    int rc = check_ring_args(cfg);
    if (rc) return rc;
    if (n_rings == 0) return FDF_OK;
    if (!d_centers || !d_rings || !d_scores || ((uintptr_t)d_rings & 15u)) return FDF_ERR_ARG;
    DeviceGuard guard(ctx->device);
    // NULL = the HIP null stream, as for every device-pointer call (torch's default stream is
    // NULL: the context's own stream would not be ordered with it)
    const hipError_t e = fdfk::launch_score_rings(d_centers, d_rings, (uint32_t)n_rings, cfg->nms,
                                                  cfg->threshold, ring_count(cfg), d_scores,
                                                  reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
}

int fdf_score_rings(fdf_ctx* ctx, const uint8_t* centers, const uint8_t* rings, size_t n_rings,
                    const fdf_config* cfg, uint16_t* out_scores) {
    if (!ctx || n_rings > 0xffffffffull) return FDF_ERR_ARG;
    int rc = check_ring_args(cfg);
    if (rc) return rc;
    if (n_rings == 0) return FDF_OK;
    if (!centers || !rings || !out_scores) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    ctx->last.valid = false;              // d_in / d_out are reused below
    wait_done(ctx);
    const size_t ring_bytes = n_rings * 16;
    if ((rc = ensure(ctx, &ctx->d_in, &ctx->in_bytes, ring_bytes + n_rings, ctx->stream))) return rc;
    if ((rc = ensure(ctx, &ctx->d_out, &ctx->out_points, (n_rings + 3) / 4, ctx->stream))) return rc;
    uint16_t* d_scores = reinterpret_cast<uint16_t*>(ctx->d_out);
    hipError_t e = hipMemcpyAsync(ctx->d_in, rings, ring_bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->d_in + ring_bytes, centers, n_rings, hipMemcpyHostToDevice,
                           ctx->stream);
    if (e == hipSuccess)
        e = fdfk::launch_score_rings(ctx->d_in + ring_bytes, ctx->d_in, (uint32_t)n_rings,
                                     cfg->nms, cfg->threshold, ring_count(cfg), d_scores,
                                     ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(out_scores, d_scores, n_rings * sizeof(uint16_t), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = sync_own_stream(ctx);
    return e == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
}

// ---- multi-device batch: contiguous frame shards, one host thread per context ----------

int fdf_detect_batch_multi(fdf_ctx* const* ctxs, uint32_t n_ctx, const uint8_t* data,
                           uint32_t n_frames, uint32_t width, uint32_t height,
                           size_t frame_stride_bytes, const fdf_config* cfg, fdf_point* out,
                           size_t cap, uint64_t* frame_offsets, size_t* n_out) {
    if (!ctxs || n_ctx == 0 || n_ctx > 1024 || !n_out || (cap && !out)) return FDF_ERR_ARG;
    for (uint32_t k = 0; k < n_ctx; ++k) {
        if (!ctxs[k]) return FDF_ERR_ARG;
        for (uint32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return FDF_ERR_ARG;   // each shard needs its own workspace
    }
    if (n_frames > 1 && frame_stride_bytes < (size_t)width * height) return FDF_ERR_ARG;
    int empty = 0;
    int rc = check_host_args(data, n_frames, width, height, width, cfg, false, &empty);
    if (rc) return rc;
    std::vector<uint64_t> offs(n_frames + 1ull, 0);
    const auto locks = lock_all(ctxs, n_ctx);                     // held throughout
    const uint64_t gen = ++g_multi_gen;
    auto tag = [&](uint32_t k) {
        ctxs[k]->last.multi_gen = gen;
        ctxs[k]->last.shard = k;
        ctxs[k]->last.nshards = n_ctx;
    };
    if (empty) {
        for (uint32_t k = 0; k < n_ctx; ++k) {
            ctxs[k]->last = LastResult{};
            ctxs[k]->last.valid = true;
            ctxs[k]->last.cfg = *cfg;
            tag(k);
        }
        *n_out = 0;
        if (frame_offsets) std::memset(frame_offsets, 0, sizeof(uint64_t) * (n_frames + 1ull));
        return FDF_OK;
    }
    // shard k: frames [first[k], first[k+1]) (contiguous, sizes differ by at most one)
    std::vector<uint32_t> first(n_ctx + 1);
    for (uint32_t k = 0; k <= n_ctx; ++k) first[k] = (uint32_t)((uint64_t)n_frames * k / n_ctx);
    std::vector<std::vector<uint64_t>> local(n_ctx);
    std::vector<int> status(n_ctx, FDF_OK);
    auto detect_shard = [&](uint32_t k) {
        fdf_ctx* ctx = ctxs[k];
        const uint32_t nf = first[k + 1] - first[k];
        ctx->last = LastResult{};
        if (nf == 0) {
            ctx->last.valid = true;
            ctx->last.cfg = *cfg;
            return;
        }
        DeviceGuard guard(ctx->device);
        local[k].assign(nf + 1ull, 0);
        status[k] = run_host(ctx, data + (size_t)first[k] * frame_stride_bytes, nf, width, height,
                             width, frame_stride_bytes, cfg, false, local[k].data(), true);
    };
    auto run_all = [&](auto&& fn) {
        std::vector<std::thread> pool;
        for (uint32_t k = 1; k < n_ctx; ++k) pool.emplace_back(fn, k);
        fn(0u);
        for (auto& t : pool) t.join();
    };
    run_all(detect_shard);
    for (uint32_t k = 0; k < n_ctx; ++k)
        if (status[k]) return status[k];
    for (uint32_t k = 0; k < n_ctx; ++k) tag(k);
    // global offsets: shard k's points follow shards 0 .. k-1
    std::vector<uint64_t> base(n_ctx + 1, 0);
    for (uint32_t k = 0; k < n_ctx; ++k) {
        const uint32_t nf = first[k + 1] - first[k];
        for (uint32_t f = 0; f < nf; ++f) offs[first[k] + f] = base[k] + local[k][f];
        base[k + 1] = base[k] + (nf ? local[k][nf] : 0);
    }
    const uint64_t total = base[n_ctx];
    offs[n_frames] = total;
    if (frame_offsets) std::memcpy(frame_offsets, offs.data(), sizeof(uint64_t) * (n_frames + 1ull));
    auto copy_shard = [&](uint32_t k) {
        const uint64_t b = std::min<uint64_t>(base[k], cap), e = std::min<uint64_t>(base[k + 1], cap);
        if (e <= b) return;
        DeviceGuard guard(ctxs[k]->device);
        status[k] = copy_out(ctxs[k], out + b, nullptr, (size_t)(e - b));
    };
    run_all(copy_shard);
    for (uint32_t k = 0; k < n_ctx; ++k)
        if (status[k]) return status[k];
    *n_out = (size_t)total;
    return total > cap ? FDF_ERR_CAPACITY : FDF_OK;
}

int fdf_fetch_last_multi(fdf_ctx* const* ctxs, uint32_t n_ctx, fdf_point* out, size_t cap,
                         size_t* n_out) {
    if (!ctxs || n_ctx == 0 || n_ctx > 1024 || !n_out || (cap && !out)) return FDF_ERR_ARG;
    for (uint32_t k = 0; k < n_ctx; ++k) {
        if (!ctxs[k]) return FDF_ERR_ARG;
        for (uint32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return FDF_ERR_ARG;
    }
    const auto locks = lock_all(ctxs, n_ctx);
    // the results must be the shards of ONE fdf_detect_batch_multi call, in its order (a
    // host call on one of the contexts since then, or a reordered array, is an error)
    const uint64_t gen = ctxs[0]->last.multi_gen;
    for (uint32_t k = 0; k < n_ctx; ++k) {
        const LastResult& L = ctxs[k]->last;
        if (!L.valid || gen == 0 || L.multi_gen != gen || L.shard != k || L.nshards != n_ctx)
            return FDF_ERR_ARG;
    }
    uint64_t b = 0;
    for (uint32_t k = 0; k < n_ctx; ++k) {
        const uint64_t n = ctxs[k]->last.total;
        const uint64_t lo = std::min<uint64_t>(b, cap), hi = std::min<uint64_t>(b + n, cap);
        if (hi > lo) {
            DeviceGuard guard(ctxs[k]->device);
            const int rc = copy_out(ctxs[k], out + lo, nullptr, (size_t)(hi - lo));
            if (rc) return rc;
        }
        b += n;
    }
    *n_out = (size_t)b;
    return b > cap ? FDF_ERR_CAPACITY : FDF_OK;
}

#ifdef FDF_DEBUG_BUILD
// Debug builds only (not in include/fdf.h): the last detector launch's workgroup stamps,
// fdfk::kStampWords words per workgroup in blockIdx order (tools/stamps.py).
int fdf_debug_stamps(fdf_ctx* ctx, uint64_t* out, uint64_t cap_words, uint64_t* n_words) {
    if (!ctx || !n_words) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(ctx->mu);
    DeviceGuard guard(ctx->device);
    *n_words = ctx->stamps_used;
    if (!ctx->d_stamps || !out) return FDF_OK;
    wait_done(ctx);
    const size_t n = (size_t)std::min<uint64_t>(cap_words, ctx->stamps_used);
    return hipMemcpy(out, ctx->d_stamps, n * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess
               ? FDF_OK
               : FDF_ERR_DEVICE;
}
#endif

}  // extern "C"
