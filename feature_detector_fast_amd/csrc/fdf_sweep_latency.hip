// fdf_sweep_latency.hip -- the grey detector for grids whose units end inside an 8-step block
// (a single frame's short bands, fdf_api.cpp enqueue): fdf_sweep_impl.h with
// FDF_SWEEP_TU_EXIT, so a unit stops at its last row instead of sweeping padding rows.
#define FDF_SWEEP_RGB 0
#define FDF_SWEEP_NS grey_lat
#define FDF_SWEEP_TU_EXIT 1
#include "fdf_sweep_impl.h"

namespace fdfk {
hipError_t launch_sweep_latency(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                                hipEvent_t start, hipEvent_t stop) {
    return grey_lat::launch(p, nms, n, stream, start, stop);
}
}  // namespace fdfk
