// fdf_kernels.h -- shared between the HIP kernels (fdf_kernels.hip) and the C-ABI host
// layer (fdf_api.cpp): tiling constants, the LDS layout and the launch parameters.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdfk {

constexpr int kNmsOff = 0;
constexpr int kNmsMaxThreshold = 1;
constexpr int kNmsSumAbsolute = 2;

constexpr int kThreads = 256;                 // 4 waves of 64 lanes
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = 1024;                  // centre columns per chunk (256 lanes x 4 px)
constexpr int kGroups = kChunk / 4 + 2;       // 4-pixel groups incl. a 1-group ring each side
constexpr int kPitch = kChunk + 32;           // input tile row pitch in bytes (16-B aligned)
constexpr int kScorePitch = kChunk + 8;       // score row pitch in u16
constexpr int kQueueCap = 80;                 // per-wave candidate queue (15 + 64 fit)
constexpr int kKpCap = 2048;                  // per-chunk NMS keypoint list
constexpr int kMaxRows = 16;                  // largest band height the host may pick
constexpr uint32_t kMaxLds = 64 * 1024;       // default dynamic-LDS limit per workgroup

// Internal ablation switches (BandParams::flags), set from the FDF_DEBUG_FLAGS environment
// variable by the host layer; never part of the C ABI.  Results are wrong when set.
constexpr uint32_t kFlagNoLookback = 1;   // skip the cross-task prefix (offsets start at 0)
constexpr uint32_t kFlagNoEmit = 2;       // skip writing points

struct LdsLayout {
    uint32_t tile, scores, bitmap, q_item, q_cand, kp_list, misc, total;
};

__host__ __device__ inline uint32_t align16(uint32_t v) { return (v + 15u) & ~15u; }

// R = centre rows per band, nw = bitmap words per image row.
__host__ __device__ inline LdsLayout make_layout(uint32_t R, uint32_t nw, bool nms) {
    LdsLayout L;
    uint32_t o = 0;
    L.tile = o;    o += align16((R + 8) * kPitch);
    L.scores = o;  o += nms ? align16((R + 2) * kScorePitch * 2) : 0;
    L.bitmap = o;  o += align16(R * nw * 4);
    L.q_item = o;  o += align16(kWaves * kQueueCap * 4);
    L.q_cand = o;  o += align16(kWaves * kQueueCap * 4);
    L.kp_list = o; o += nms ? align16(kKpCap * 4) : 0;
    L.misc = o;    o += 64;
    L.total = o;
    return L;
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
    uint32_t epoch;              // look-back generation tag, 1..65535
    uint2* out;                  // (x, y) points
    uint64_t cap;                // points that fit in `out`
    uint64_t* frame_offsets;     // frames + 1 entries
    unsigned long long* band_state;  // >= ntasks look-back words
    uint32_t* task_counter;      // zero between launches (self-resetting)
    uint32_t flags;              // kFlag* ablation switches, 0 in production
};

hipError_t launch_band_kernel(const BandParams& p, uint32_t nms, uint32_t n,
                              hipStream_t stream);
hipError_t launch_score_points(const uint8_t* img, uint32_t width, const uint2* pts,
                               uint32_t npts, uint32_t nms, uint32_t t, uint32_t n,
                               uint16_t* out, hipStream_t stream);

}  // namespace fdfk
