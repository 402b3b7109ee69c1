// fdf_sweep.hip -- the detector on grey frames (fdf_sweep_impl.h instantiated for u8 pixels).
#define FDF_SWEEP_RGB 0
#define FDF_SWEEP_NS grey
#include "fdf_sweep_impl.h"

namespace fdfk {
hipError_t launch_sweep(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop) {
    return grey::launch(p, nms, n, stream, start, stop);
}
hipError_t sweep_occupancy(uint32_t nms, uint32_t n, uint32_t lds_bytes, bool rgb, int* wg_per_cu) {
    return rgb ? sweep_occupancy_rgb(nms, n, lds_bytes, wg_per_cu)
               : grey::occupancy(nms, n, lds_bytes, wg_per_cu);
}
}  // namespace fdfk
