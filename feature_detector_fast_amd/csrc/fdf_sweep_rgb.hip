// fdf_sweep_rgb.hip -- the detector on RGB8 frames (fdf_sweep_impl.h instantiated for 3-byte
// pixels): each row and window load converts its pixels to luma exactly as image 0.24.6's
// to_luma8 (src/main.rs:58, tests/compare.rs:33), so colour frames need no separate pass.
#define FDF_SWEEP_RGB 1
#define FDF_SWEEP_NS rgb
#include "fdf_sweep_impl.h"

namespace fdfk {
hipError_t launch_sweep_rgb(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop) {
    return rgb::launch(p, nms, n, stream, start, stop);
}
hipError_t sweep_occupancy_rgb(uint32_t nms, uint32_t n, uint32_t lds_bytes, int* wg_per_cu) {
    return rgb::occupancy(nms, n, lds_bytes, wg_per_cu);
}
}  // namespace fdfk
