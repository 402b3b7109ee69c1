// fdf_kernels.hip -- the kernels around the detector (fdf_sweep.hip) on MI355X (gfx950).
//
// compact_kernel -- turns the detector's per-band slots into the reference's output: one
//   list of points per frame, in raster order (src/fast_simd.rs:589-616 pushes keypoints in
//   scan order).  Each group of bands sums the counts of the bands before it (all final
//   when the kernel starts), then copies its bands' points to their final positions.
// score_points_kernel -- the reference's two NMS score functions on given points
//   (extension: fdf_score_points).
// score_rings_kernel -- the same on (centre, 16 circle pixels) tuples through the detector's
//   own score functions (fdf_score_rings; src/fast_simd.rs:623, :722).
// rgb_to_luma_kernel -- RGB8 -> grey exactly as image 0.24.6's to_luma8, which the
//   reference's callers apply before detect (src/main.rs:58, tests/compare.rs:33).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdf_common.h"
#include "fdf_compact.h"
#include "fdf_kernels.h"

namespace fdfk {

// ---------------------------------------------------------------------------------------
// Compaction: raster-order prefix over band counts, then slot -> final position copy.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kCompactTasks) void compact_kernel(CompactParams P) {
    __shared__ CompactShared sm;
    compact_group(P, blockIdx.x, sm);
}

// ---------------------------------------------------------------------------------------
// Point scoring (extension, fdf_score_points): literal formulas of the reference's score
// functions, valid for any point, one thread per point.
// ---------------------------------------------------------------------------------------
// Literal reference formulas on a ring (d_i = c - p_i), valid for any ring.
__device__ __forceinline__ uint32_t score_ring_literal(int c, const int (&p)[16], uint32_t nms,
                                                       uint32_t t, uint32_t n) {
    int d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = c - p[i];
    if (nms == kNmsSumAbsolute) {    // src/fast_simd.rs:722-749
        uint32_t sb = 0, sd = 0;
        for (int i = 0; i < 16; ++i) {
            sb += (uint32_t)max(d[i] - (int)t, 0);
            sd += (uint32_t)max(-d[i] - (int)t, 0);
        }
        return max(sb, sd);
    }
    int hi = -32768, lo = 32767;      // src/fast_simd.rs:623-718
    for (int kk = 0; kk < 16; ++kk) {
        int mn = 32767, mx = -32768;
        for (uint32_t i = 0; i < n; ++i) {
            mn = min(mn, d[(kk + i) & 15]);
            mx = max(mx, d[(kk + i) & 15]);
        }
        hi = max(hi, mn);
        lo = min(lo, mx);
    }
    return (uint32_t)min(abs(hi), abs(lo));
}

__device__ __forceinline__ uint16_t score_point(const uint8_t* img, uint32_t W, uint2 pt,
                                                uint32_t nms, uint32_t t, uint32_t n) {
    const int c = img[(uint64_t)pt.y * W + pt.x];
    int p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        p[i] = img[(uint64_t)((int)pt.y + circle_dy(i)) * W + (int)pt.x + circle_dx(i)];
    return (uint16_t)score_ring_literal(c, p, nms, t, n);
}

__global__ __launch_bounds__(256) void score_points_kernel(const uint8_t* img, uint32_t W,
                                                           const uint2* pts, uint32_t npts,
                                                           uint32_t nms, uint32_t t,
                                                           uint32_t n, uint16_t* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npts) return;
    out[k] = score_point(img, W, pts[k], nms, t, n);
}

// Batched form for detect output: frame f (blockIdx.y) scores points
// [offsets[f], offsets[f+1]) against its own frame; offsets are read on the device, so the
// launch needs no host round trip after detection.
__global__ __launch_bounds__(256) void score_frames_kernel(const uint8_t* frames, uint32_t W,
                                                           uint64_t frame_stride,
                                                           const uint2* pts,
                                                           const uint64_t* offsets,
                                                           uint64_t cap, uint32_t nms,
                                                           uint32_t t, uint32_t n,
                                                           uint16_t* out) {
    const uint32_t f = blockIdx.y;
    const uint64_t b = offsets[f], e = min(offsets[f + 1], cap);
    const uint8_t* img = frames + (uint64_t)f * frame_stride;
    for (uint64_t k = b + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < e;
         k += (uint64_t)gridDim.x * blockDim.x)
        out[k] = score_point(img, W, pts[k], nms, t, n);
}

// ---------------------------------------------------------------------------------------
// Ring scoring (fdf_score_rings; the reference's pub ring functions src/fast_simd.rs:623
// and :722, which take a centre and the 16 circle pixels).  SumAbsolute goes through the
// detector's own score_sum_abs_packed; MaxThreshold through the detector's segment test
// (t = 0: the polarity of an arc of N pixels brighter / darker than the centre) and its
// score_max_threshold<N>, and the literal formula for rings with no such arc (the detector
// never scores those).  Ring k is 16 bytes at rings + 16 k (16-byte aligned).
// ---------------------------------------------------------------------------------------
template <int N>
__global__ __launch_bounds__(256) void score_rings_kernel(const uint8_t* centers,
                                                          const uint4* rings, uint32_t nrings,
                                                          uint32_t nms, uint32_t t,
                                                          uint16_t* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrings) return;
    const uint4 r = rings[k];
    const uint32_t c = centers[k];
    const uint32_t wd[4] = {r.x, r.y, r.z, r.w};   // byte j of wd[q] = pixel 4q + j
    uint32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = (wd[i >> 2] >> (8 * (i & 3))) & 0xffu;
    uint32_t score;
    if (nms == kNmsSumAbsolute) {
        uint32_t w[4];   // byte j of w[m] = pixel 4j + m (the detector's packed ring)
#pragma unroll
        for (int m = 0; m < 4; ++m)
            w[m] = p[m] | (p[m + 4] << 8) | (p[m + 8] << 16) | (p[m + 12] << 24);
        score = score_sum_abs_packed(c, w, t);
    } else {
        bool bright, dark;
        lane_segment_test<N>(c, p, lerp_consts(0), bright, dark);
        if (bright || dark) {
            score = score_max_threshold<N>(c, p, dark);
        } else {
            int q[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) q[i] = (int)p[i];
            score = score_ring_literal((int)c, q, nms, t, N);
        }
    }
    out[k] = (uint16_t)score;
}

hipError_t launch_score_rings(const uint8_t* centers, const uint8_t* rings, uint32_t nrings,
                              uint32_t nms, uint32_t t, uint32_t n, uint16_t* out,
                              hipStream_t stream) {
    if (nrings == 0) return hipSuccess;
    if (((uintptr_t)rings & 15u) != 0 || n < 9 || n > 16) return hipErrorInvalidValue;
    const dim3 grid((nrings + 255) / 256), block(256);
    const uint4* r = reinterpret_cast<const uint4*>(rings);
    switch (n) {
#define FDF_RING_CASE(NN)                                                                     \
    case NN:                                                                                 \
        hipLaunchKernelGGL(score_rings_kernel<NN>, grid, block, 0, stream, centers, r, nrings, \
                           nms, t, out);                                                     \
        break;
        FDF_RING_CASE(9) FDF_RING_CASE(10) FDF_RING_CASE(11) FDF_RING_CASE(12)
        FDF_RING_CASE(13) FDF_RING_CASE(14) FDF_RING_CASE(15) FDF_RING_CASE(16)
#undef FDF_RING_CASE
    }
    return hipGetLastError();
}

hipError_t launch_compact(const CompactParams& c, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop) {
    if (c.tasks_per_group == 0 || c.tasks_per_group > (uint32_t)kCompactTasks)
        return hipErrorInvalidValue;
    const uint32_t ngroups = (c.ntasks + c.tasks_per_group - 1) / c.tasks_per_group;
    if (start || stop)
        hipExtLaunchKernelGGL(compact_kernel, dim3(ngroups), dim3(kCompactTasks), 0, stream, start,
                              stop, 0, c);
    else
        hipLaunchKernelGGL(compact_kernel, dim3(ngroups), dim3(kCompactTasks), 0, stream, c);
    return hipGetLastError();
}

hipError_t launch_score_points(const uint8_t* img, uint32_t W, const uint2* pts,
                               uint32_t npts, uint32_t nms, uint32_t t, uint32_t n,
                               uint16_t* out, hipStream_t stream) {
    if (npts == 0) return hipSuccess;
    hipLaunchKernelGGL(score_points_kernel, dim3((npts + 255) / 256), dim3(256), 0, stream,
                       img, W, pts, npts, nms, t, n, out);
    return hipGetLastError();
}

hipError_t launch_score_frames(const uint8_t* frames, uint32_t W, uint64_t frame_stride,
                               uint32_t n_frames, const uint2* pts, const uint64_t* offsets,
                               uint64_t cap, uint32_t blocks_per_frame, uint32_t nms,
                               uint32_t t, uint32_t n, uint16_t* out, hipStream_t stream) {
    if (n_frames == 0 || cap == 0) return hipSuccess;
    if (n_frames > 65535u || blocks_per_frame == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(score_frames_kernel, dim3(blocks_per_frame, n_frames), dim3(256), 0,
                       stream, frames, W, frame_stride, pts, offsets, cap, nms, t, n, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// RGB8 -> grey: image 0.24.6 color.rs rgb_to_luma for u8 (not vendored in the reference;
// its published formula): l = 2126 r + 7152 g + 722 b, luma = l / 10000 (truncating).
// 16 pixels per thread: three 16-byte loads, one 16-byte store; only a frame's last,
// partial group goes byte by byte, so nothing outside the frame is read or written.
// ---------------------------------------------------------------------------------------
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t luma_of(uint32_t r, uint32_t g, uint32_t b) {
    return (2126u * r + 7152u * g + 722u * b) / 10000u;
}

__global__ __launch_bounds__(256) void rgb_to_luma_kernel(const uint8_t* rgb,
                                                          uint64_t rgb_frame_stride,
                                                          uint32_t pixels, uint8_t* grey) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;        // 16-pixel group
    const uint32_t first = g * 16u;
    if (first >= pixels) return;
    const uint8_t* src = rgb + (uint64_t)blockIdx.y * rgb_frame_stride;
    uint8_t* dst = grey + (uint64_t)blockIdx.y * pixels;
    if (first + 16u > pixels) {
        for (uint32_t i = first; i < pixels; ++i)
            dst[i] = (uint8_t)luma_of(src[3 * i], src[3 * i + 1], src[3 * i + 2]);
        return;
    }
    const __amdgpu_buffer_rsrc_t in = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(src), 0, (int)(3u * pixels), 0x00020000);
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)pixels,
                                                                          0x00020000);
    uint32_t w[12];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const u32x4_t v = __builtin_bit_cast(
            u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(in, (int)(3u * first) + 16 * k, 0, 0));
#pragma unroll
        for (int m = 0; m < 4; ++m) w[4 * k + m] = v[m];
    }
    u32x4_t o = (u32x4_t)(0u);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t r = (w[(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 0xffu;
        const uint32_t gg = (w[(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 0xffu;
        const uint32_t b = (w[(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 0xffu;
        o[j >> 2] |= luma_of(r, gg, b) << (8 * (j & 3));
    }
    __builtin_amdgcn_raw_buffer_store_b128(o, out, (int)first, 0, 0);
}

hipError_t launch_rgb_to_luma(const uint8_t* rgb, uint32_t n_frames, uint32_t pixels,
                              uint64_t rgb_frame_stride, uint8_t* grey, hipStream_t stream) {
    if (n_frames == 0 || pixels == 0) return hipSuccess;
    const uint32_t groups = (pixels + 15u) / 16u;
    const dim3 grid((groups + 255u) / 256u, n_frames);
    if (n_frames > 65535u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rgb_to_luma_kernel, grid, dim3(256), 0, stream, rgb, rgb_frame_stride,
                       pixels, grey);
    return hipGetLastError();
}

}  // namespace fdfk
