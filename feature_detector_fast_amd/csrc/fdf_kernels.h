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
// variable by the host layer; never part of the C ABI.  Results are wrong when set.
constexpr uint32_t kFlagNoFullTest = 1;   // candidates are never tested (no keypoints)
constexpr uint32_t kFlagNoEmit = 2;       // bands write no slot contents (counts only)
constexpr uint32_t kFlagNoPrefilter = 4;  // no units are swept (slots and compaction only)
constexpr uint32_t kFlagNoLoad = 8;       // rows are streamed and compared, never pre-filtered

// Column-sweep kernel (fdf_sweep.hip): per-wave LDS region + the band bitmap.
// Columns per lane (16; FDF_LC_NMS = 8 halves the NMS score ring for A/B runs).  A strip is
// 62 lanes wide (lanes 0 and 63 are halo lanes).
#ifndef FDF_LC_NMS
#define FDF_LC_NMS 16
#endif
__host__ __device__ constexpr int lane_cols_for(uint32_t nms) { return nms == 0 ? 16 : FDF_LC_NMS; }
__host__ __device__ constexpr int strip_cols(int lc) { return 62 * lc; }
constexpr int kSweepPixelQ = 256;             // candidate pixel FIFO per wave (power of two)
// NMS score ring rows per wave (power of two): deep enough that testing can lag the sweep
// while a 64-pixel batch fills; SAD's 16-bit scores make its ring twice as big per row.
// (4 rows of 16-column lanes measured fastest: 8 or 16 rows, or 8-column lanes, cost a
// workgroup per CU; batches are issued partially full once their oldest pixel would
// outrun the ring.  tools/build_variant.sh rebuilds with other values for A/B runs.)
#ifndef FDF_RING_MAXT
#define FDF_RING_MAXT 4
#endif
#ifndef FDF_RING_SAD
#define FDF_RING_SAD 4
#endif
__host__ __device__ constexpr int sweep_ring_rows(uint32_t nms) {
    return nms == 0 ? 0 : (nms == 1 ? FDF_RING_MAXT : FDF_RING_SAD);
}
constexpr int kSweepKpCap = 256;              // unfinalized NMS keypoints per wave
constexpr uint32_t kSweepMaxLds = 160 * 1024; // gfx950 LDS per CU (and per workgroup)

// A full-test batch is issued every kSweepIssue(nms) rows once 64 candidates are queued and
// is evaluated the same number of rows later.
#ifndef FDF_ISSUE_NMS
#define FDF_ISSUE_NMS 4
#endif
__host__ __device__ constexpr int sweep_issue_every(uint32_t nms) { return nms == 0 ? 2 : FDF_ISSUE_NMS; }

struct SweepLayout {
    uint32_t pq, ring, kp, wave_bytes, bitmap, total;
};

__host__ __device__ inline uint32_t align16(uint32_t v);

__host__ __device__ inline SweepLayout make_sweep_layout(uint32_t R, uint32_t nw,
                                                         uint32_t score_bytes, uint32_t lc) {
    SweepLayout L;
    uint32_t o = 0;
    L.pq = o;       o += kSweepPixelQ * 4;
    L.ring = o;     o += sweep_ring_rows(score_bytes) * 64 * lc * score_bytes;
    L.kp = o;       o += score_bytes ? kSweepKpCap * 4 : 0;
    L.wave_bytes = align16(o);
    L.bitmap = 4 * L.wave_bytes;
    L.total = L.bitmap + align16(R * nw * 4) + 64;
    return L;
}

// Sweep steps a unit of `rows` owned rows takes: the pre-filtered rows (owned rows plus, with
// NMS, one score row each side) and 3 rows of vertical look-ahead, in whole 8-step blocks.
__host__ __device__ inline uint32_t sweep_steps(uint32_t rows, uint32_t score_bytes) {
    return (rows + 3 + (score_bytes ? 2 : 0) + 7) & ~7u;
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

struct BandParams {
    const uint8_t* frames;       // frame f at frames + f * frame_stride, rows packed (stride = width)
    uint64_t frame_stride;
    uint32_t width, height;
    uint32_t rows;               // centre rows per band (R)
    uint32_t bands_per_frame;
    uint32_t ntasks;             // frames * bands_per_frame == grid size
    uint32_t words_per_row;      // ceil(width / 32)
    uint32_t threshold;
    uint32_t slot_bytes;
    uint8_t* slots;              // ntasks * slot_bytes
    uint32_t* counts;            // ntasks keypoint counts (band order = raster order)
    uint32_t flags;              // kFlag* ablation switches, 0 in production
    uint32_t nstrips, nsub;      // sweep kernel: column strips x sub-bands per band
};

// Bands per compaction workgroup: enough groups (~1024) to spread the copy over the chip.
__host__ __device__ inline uint32_t compact_tasks_per_group(uint32_t ntasks) {
    const uint32_t t = ntasks / 1024;
    return t < 1 ? 1u : (t > (uint32_t)kCompactTasks ? (uint32_t)kCompactTasks : t);
}

struct CompactParams {
    uint32_t width, height, rows, bands_per_frame, ntasks, words_per_row, slot_bytes;
    uint32_t tasks_per_group;        // compact_tasks_per_group(ntasks)
    uint32_t epoch;                  // look-back generation tag, 1..65535
    const uint8_t* slots;
    const uint32_t* counts;
    uint2* out;
    uint64_t cap;
    uint64_t* frame_offsets;         // frames + 1 entries
    unsigned long long* state;       // >= ceil(ntasks / tasks_per_group) look-back words
    uint32_t* ticket;                // zero between launches (self-resetting)
};

hipError_t launch_compact(const CompactParams& c, hipStream_t stream);
hipError_t launch_sweep(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream);
hipError_t launch_rgb_to_luma(const uint8_t* rgb, uint32_t n_frames, uint32_t pixels,
                              uint64_t rgb_frame_stride, uint8_t* grey, hipStream_t stream);
hipError_t launch_score_points(const uint8_t* img, uint32_t width, const uint2* pts,
                               uint32_t npts, uint32_t nms, uint32_t t, uint32_t n,
                               uint16_t* out, hipStream_t stream);
hipError_t launch_score_frames(const uint8_t* frames, uint32_t width, uint64_t frame_stride,
                               uint32_t n_frames, const uint2* pts, const uint64_t* offsets,
                               uint64_t cap, uint32_t blocks_per_frame, uint32_t nms,
                               uint32_t t, uint32_t n, uint16_t* out, hipStream_t stream);

}  // namespace fdfk
