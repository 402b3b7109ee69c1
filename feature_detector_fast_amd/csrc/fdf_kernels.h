// fdf_kernels.h -- shared between the HIP kernels (fdf_sweep.hip, fdf_kernels.hip) and the
// C-ABI host layer (fdf_api.cpp): geometry constants, LDS layout and launch parameters.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdfk {

constexpr int kNmsOff = 0;
constexpr int kNmsMaxThreshold = 1;
constexpr int kNmsSumAbsolute = 2;

constexpr int kThreads = 256;                 // 4 waves of 64 lanes
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kMaxLds = 64 * 1024;       // default dynamic-LDS limit per workgroup
constexpr int kCompactTasks = 256;            // tasks per workgroup of the compaction kernel

// Internal ablation switches (BandParams::flags), set from the FDF_DEBUG_FLAGS environment
// variable by the host layer of the debug build only (make debug -> libfdf_debug.so, built
// with -DFDF_DEBUG_BUILD); never part of the C ABI.  Results are wrong when set.  In the
// production build the kernels see the constant 0 and the ablation branches compile away.
constexpr uint32_t kFlagNoFullTest = 1;   // candidates are never tested (no keypoints)
constexpr uint32_t kFlagNoEmit = 2;       // bands write no slot contents (counts only)
constexpr uint32_t kFlagNoPrefilter = 4;  // no units are swept (slots and compaction only)
constexpr uint32_t kFlagNoLoad = 8;       // rows are streamed and compared, no candidates
constexpr uint32_t kFlagNoNms = 16;       // NMS modes: every keypoint is kept (no band NMS pass)
constexpr uint32_t kFlagNmsPrefixOnly = 32;  // band NMS pass: rank prefixes only (timing)
constexpr uint32_t kFlagNoEval = 64;       // batches are issued (FIFO, staging, loads), never tested
#ifdef FDF_DEBUG_BUILD
__host__ __device__ inline uint32_t ablation_flags(uint32_t f) { return f; }
constexpr bool kDebugBuild = true;
#else
__host__ __device__ inline uint32_t ablation_flags(uint32_t) { return 0u; }
constexpr bool kDebugBuild = false;
#endif
// Debug builds: per-workgroup stamps of the detector (BandParams::stamps, kStampWords words per
// workgroup): shader clock and 100 MHz real time at the workgroup's start and end, its XCD
// and hardware id, its band, and the shader clock at the end of its phases as wave 0 sees
// them (setup, its sweep, NMS, look-back), and the low 32 bits of the shader clock at each
// wave's sweep end.  Written only to that buffer; no output depends on them.
constexpr uint32_t kStampWords = 12;

// Column-sweep kernel (fdf_sweep.hip).  Lane l of a wave owns kLaneCols columns; a strip is
// 62 lanes wide (lanes 0 and 63 are halo lanes).
constexpr int kLaneCols = 16;
__host__ __device__ constexpr int strip_cols(int lc) { return 62 * lc; }
constexpr int kSweepPixelQ = 256;             // candidate pixel FIFO per wave (power of two)
constexpr uint32_t kSweepMaxLds = 160 * 1024; // gfx950 LDS per CU (and per workgroup)

// A full-test batch is issued every kSweepIssue rows once 64 candidates are queued and is
// evaluated the same number of rows later.
#ifndef FDF_ISSUE
#define FDF_ISSUE 3
#endif
constexpr int kSweepIssue = FDF_ISSUE;
// Full-test batches in flight (each evaluated kSweepBatchSlots issue points after its issue).
#ifndef FDF_BATCH_SLOTS
#define FDF_BATCH_SLOTS 1
#endif
constexpr int kSweepBatchSlots = FDF_BATCH_SLOTS;
// Pixel-row register ring of the sweep (rows in flight = kSweepRing - 4); unit sweeps are
// whole multiples of kSweepRing steps.
#ifndef FDF_RING
#define FDF_RING 8
#endif
constexpr int kSweepRing = FDF_RING;
// Waves per SIMD of the sweep kernel (register budget 512 / kSweepWavesPerEU VGPRs).
#ifndef FDF_WAVES_PER_EU
#define FDF_WAVES_PER_EU 4
#endif
constexpr int kSweepWavesPerEU = FDF_WAVES_PER_EU;

// Rows of keypoint bitmap above and below a band: NMS compares a band's edge rows with the
// neighbouring bands' rows, so the band also tests one row each side (scores only).
__host__ __device__ inline uint32_t band_halo(uint32_t nms) { return nms ? 1u : 0u; }

// LDS of one workgroup: the keypoint bitmap of the band's R rows plus the NMS halo rows (NMS
// then clears the suppressed keypoints in place; one pad word after the bitmap lets bit
// look-ups read two words unconditionally), 4 candidate FIFOs (+ batch staging), and for NMS
// the band's keypoint scores: a list of kScoreListCap (position, score) entries and per-row /
// per-4-word-block keypoint counts that turn a bitmap position into its raster rank.  The
// FIFOs, staging and score list are contiguous: once the sweep is done they hold the scores
// in rank order (`nms_area`, u16 entries; the FIFO part alone for band_nms_lds).
#ifndef FDF_SLIST_CAP
#define FDF_SLIST_CAP 2048
#endif
constexpr uint32_t kScoreListCap = FDF_SLIST_CAP;
constexpr uint32_t kRankBlock = 4;            // bitmap words per rank-prefix block
// band_nms_lds ranks the list's scores as u16 into the 4 candidate FIFOs
static_assert(kScoreListCap * 2 <= 4 * kSweepPixelQ * 4, "ranked scores must fit the FIFO area");
static_assert(kScoreListCap % 256 == 0, "the spill NMS pass holds the list 1/256 per thread");
static_assert(kScoreListCap < 4096, "the LDS NMS pass keeps rank + 1 in a list entry's 12 score bits");
struct SweepLayout {
    uint32_t pq, wave_bytes, stage, bitmap, slist, bprefix, rprefix, misc, total;
    uint32_t seltab;             // during the sweep: the 256-entry set-bit table (1 KB) in
                                 // the rank-prefix area, which NMS uses only after the sweep
    uint32_t nms_area_entries;   // u16 ranked scores that fit [pq, bprefix) after the sweep
};

__host__ __device__ inline uint32_t align16(uint32_t v);

__host__ __device__ inline SweepLayout make_sweep_layout(uint32_t R, uint32_t nw, uint32_t nms) {
    SweepLayout L;
    const uint32_t rows = R + 2 * band_halo(nms);
    const uint32_t nb = (nw + kRankBlock - 1) / kRankBlock;
    L.bitmap = 0;
    L.pq = align16(rows * nw * 4 + 4);
    L.wave_bytes = kSweepPixelQ * 4;              // 4 FIFOs = kScoreListCap u16 ranked scores
    L.stage = L.pq + 4 * L.wave_bytes;            // 4 x 64 staged batch pixels
    L.slist = L.stage + 4 * 64 * 4;
    const uint32_t cap = nms ? kScoreListCap : 0u;
    L.bprefix = L.slist + cap * 4;
    L.nms_area_entries = (L.bprefix - L.pq) / 2;
    L.rprefix = L.bprefix + (nms ? align16(rows * nb * 2) : 0u);
    L.seltab = L.bprefix;
    const uint32_t prefix_end = L.rprefix + (nms ? align16(rows * 4) : 0u);
    L.misc = prefix_end > L.seltab + 1024u ? prefix_end : L.seltab + 1024u;
    L.total = L.misc + 64;
    return L;
}

// Words per bitmap row: ceil(W / 32) rounded up to a multiple of 4, so that every row of a
// band's bitmap (LDS, and a slot holding it) starts 16-byte aligned and the emit reads 4
// words of one row per lane (the pad words stay zero).
__host__ __device__ inline uint32_t bitmap_words_per_row(uint32_t W) {
    return ((W + 31) / 32 + 3) & ~3u;
}

// Sweep steps of a unit of `rows` owned rows plus `halo` extra tested rows, in whole
// kSweepRing-step blocks (the 3 rows of vertical look-ahead are a prologue, not steps).
__host__ __device__ inline uint32_t sweep_steps(uint32_t rows, uint32_t halo) {
    return (rows + halo + kSweepRing - 1) / kSweepRing * kSweepRing;
}

__host__ __device__ inline uint32_t align16(uint32_t v) { return (v + 15u) & ~15u; }

__host__ __device__ inline uint32_t score_bytes_for(uint32_t nms) {
    return nms == kNmsOff ? 0u : (nms == kNmsMaxThreshold ? 1u : 2u);
}

// Per-band output slot: the band's points (8 B each) when they fit, else its keep-bitmap.
__host__ __device__ inline uint32_t slot_bytes_for(uint32_t R, uint32_t nw) {
    const uint32_t b = align16(R * nw * 4);
    return b < 256 ? 256 : b;
}

// Bands per compaction workgroup: enough groups (~1024) to spread the copy over the chip.
__host__ __device__ inline uint32_t compact_tasks_per_group(uint32_t ntasks) {
    const uint32_t t = ntasks / 1024;
    return t < 1 ? 1u : (t > (uint32_t)kCompactTasks ? (uint32_t)kCompactTasks : t);
}
// Per-group keypoint sums the detector accumulates (one atomic add per band) so that a
// compaction group finds its output base by summing the groups before it, O(groups) instead
// of O(tasks).  Two buffers alternate between launches: a launch reads one and its
// compaction zeroes the other for the next launch.
constexpr uint32_t kMaxGroupSums = 2048;
struct CompactParams {
    uint32_t width, height, rows, bands_per_frame, ntasks, words_per_row, slot_bytes;
    uint32_t tasks_per_group;        // compact_tasks_per_group(ntasks)
    const uint8_t* slots;
    const uint32_t* counts;
    uint2* out;
    uint64_t cap;
    uint64_t* frame_offsets;         // frames + 1 entries
    const uint32_t* group_sums;      // per-group sums of this launch (NULL: sum the counts)
    uint32_t* next_sums;             // zeroed here for the next launch (kMaxGroupSums entries)
    uint32_t* kp_stats;              // NMS: the detector's keypoint total (read and reset here)
    uint64_t* stats_out;             // host-mapped: stats_seq << 32 | that total
    uint32_t stats_seq;
};

struct BandParams {
    const uint8_t* frames;       // frame f at frames + f * frame_stride, rows packed (stride = width)
    uint64_t frame_stride;
    uint32_t width, height;
    uint32_t rows;               // centre rows per band (R)
    uint32_t bands_per_frame;
    uint32_t ntasks;             // frames * bands_per_frame == grid size
    uint32_t words_per_row;      // bitmap_words_per_row(width)
    uint32_t threshold;
    uint32_t slot_bytes;
    uint8_t* slots;              // ntasks * slot_bytes
    uint32_t* counts;            // ntasks keypoint counts (band order = raster order)
    uint32_t flags;              // kFlag* ablation switches, 0 in production
    uint32_t nstrips, nsub;      // sweep kernel: column strips x sub-bands per band
    uint32_t* group_sums;        // += band count at [task / tasks_per_group] (NULL: none)
    uint32_t tasks_per_group;
    uint32_t* kp_stats;          // NMS: += each band's keypoints before suppression (NULL: off)
    uint64_t* stamps;            // debug builds: kStampWords per workgroup (NULL: off)
    // Direct output (small grids, every workgroup resident at once): each band finds its
    // output position by a decoupled look-back over the bands before it and writes its points
    // to `out` itself; no compaction launch.  The band slots are still written (a host call
    // whose output has to grow runs compact_kernel from them).
    uint32_t direct;             // 1: direct output
    uint32_t epoch;              // this launch's tag in the look-back descriptors
    uint64_t* lookback;          // ntasks descriptors: epoch << 32 | kLbAggregate / kLbPrefix | value
    uint2* out;                  // direct: the caller's points, `cap` of them
    uint64_t cap;
    uint64_t* frame_offsets;     // direct: frames + 1 entries
    // Direct output: a workgroup's band is its ticket (a device counter taken when it starts,
    // less this launch's first ticket), so bands are swept in the order workgroups start and
    // a band's look-back only ever waits on bands that started before it -- no residency
    // assumption.  Each launch takes exactly ntasks tickets; the host keeps the running base.
    uint32_t* ticket;
    uint32_t ticket_base;
    // Direct output: set when a look-back wait ran out (host-mapped; the band then publishes
    // no prefix and writes no points, and the host recovers from the slots: fdf_api.cpp)
    uint32_t* lookback_error;
    // Host frames arriving in row chunks while the kernel runs (fdf_detect's overlapped
    // upload; NULL: the frames are in place): chunk c = rows [c * chunk_rows, (c+1) *
    // chunk_rows) has landed once chunk_flags[c] == chunk_epoch (device words a 4-byte copy
    // on the copy stream writes after each chunk's copy, in order).  A band waits for the
    // chunk of the last row it reads before its first load; a wait that runs out sets
    // lookback_error.
    const uint32_t* chunk_flags;
    uint32_t chunk_rows;
    uint32_t chunk_epoch;
};
constexpr uint64_t kLbAggregate = 1ull << 30;   // value = the band's own keypoint count
constexpr uint64_t kLbPrefix = 1ull << 31;      // value = keypoints of bands 0 .. this one
constexpr uint64_t kLbValue = kLbAggregate - 1;
constexpr uint64_t kLbNoBase = ~0ull;           // band_lookback's result after a timeout
// Direct output pays off when the whole grid is resident at once (a band's look-back then
// waits only for bands running beside it): up to this many workgroups, within the CU count
// times the workgroups one CU holds by the kernel's occupancy (host side, fdf_api.cpp).
constexpr uint32_t kDirectMaxTasks = 1024;

// start / stop (optional): events the dispatch itself timestamps (hipExtLaunchKernelGGL), so
// per-kernel timing adds no packets between the kernels
hipError_t launch_compact(const CompactParams& c, hipStream_t stream, hipEvent_t start = nullptr,
                          hipEvent_t stop = nullptr);
hipError_t launch_sweep(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                        hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
// The same detector whose units leave their last 8-step block at their last row
// (fdf_sweep_latency.hip): for grids of short units (a single frame's latency bands)
hipError_t launch_sweep_latency(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                                hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
// Workgroups of the detector instance (nms, n; grey or RGB) one CU holds at once with
// `lds_bytes` of dynamic LDS (the runtime's occupancy calculator: registers, LDS, waves).
hipError_t sweep_occupancy(uint32_t nms, uint32_t n, uint32_t lds_bytes, bool rgb, int* wg_per_cu);
hipError_t sweep_occupancy_rgb(uint32_t nms, uint32_t n, uint32_t lds_bytes, int* wg_per_cu);
// RGB8 frames (3 bytes per pixel, frame_stride in bytes), luma converted on load
hipError_t launch_sweep_rgb(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                            hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_rgb_to_luma(const uint8_t* rgb, uint32_t n_frames, uint32_t pixels,
                              uint64_t rgb_frame_stride, uint8_t* grey, hipStream_t stream);
hipError_t launch_score_rings(const uint8_t* centers, const uint8_t* rings, uint32_t nrings,
                              uint32_t nms, uint32_t t, uint32_t n, uint16_t* out,
                              hipStream_t stream);
hipError_t launch_score_points(const uint8_t* img, uint32_t width, const uint2* pts,
                               uint32_t npts, uint32_t nms, uint32_t t, uint32_t n,
                               uint16_t* out, hipStream_t stream);
hipError_t launch_score_frames(const uint8_t* frames, uint32_t width, uint64_t frame_stride,
                               uint32_t n_frames, const uint2* pts, const uint64_t* offsets,
                               uint64_t cap, uint32_t blocks_per_frame, uint32_t nms,
                               uint32_t t, uint32_t n, uint16_t* out, hipStream_t stream);

}  // namespace fdfk
