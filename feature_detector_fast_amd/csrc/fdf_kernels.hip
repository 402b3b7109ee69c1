// fdf_kernels.hip -- the kernels around the detector (fdf_sweep.hip) on MI355X (gfx950).
//
// compact_kernel -- turns the detector's per-band slots into the reference's output: one
//   list of points per frame, in raster order (src/fast_simd.rs:589-616 pushes keypoints in
//   scan order).  Each group of bands sums the counts of the bands before it (all final
//   when the kernel starts), then copies its bands' points to their final positions.
// score_points_kernel -- the reference's two NMS score functions on given points
//   (extension: fdf_score_points).
// rgb_to_luma_kernel -- RGB8 -> grey exactly as image 0.24.6's to_luma8, which the
//   reference's callers apply before detect (src/main.rs:58, tests/compare.rs:33).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdf_common.h"
#include "fdf_kernels.h"

namespace fdfk {

// ---------------------------------------------------------------------------------------
// Compaction: raster-order prefix over band counts, then slot -> final position copy.
// ---------------------------------------------------------------------------------------
// Group g covers tasks [g*T, g*T + T) (T = P.tasks_per_group <= kCompactTasks, chosen by
// the host so that ~1024 groups share the copy).  The points of the group's slot-list bands
// are copied cooperatively by all threads (output index -> band by binary search over an
// in-group prefix), so the writes are coalesced whatever the per-band counts; bitmap bands
// are expanded by one wave each.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave_sum,
                                                         uint32_t& total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
    if (lane == 63) s_wave_sum[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kCompactTasks / 64; ++w) {
        const uint32_t x = s_wave_sum[w];
        before += (uint32_t)w < wave ? x : 0u;
        total += x;
    }
    __syncthreads();
    return before + incl - v;
}

__global__ __launch_bounds__(kCompactTasks) void compact_kernel(CompactParams P) {
    __shared__ uint32_t s_task_off[kCompactTasks + 1];
    __shared__ uint32_t s_list_off[kCompactTasks + 1];
    __shared__ uint32_t s_wave_sum[kCompactTasks / 64];
    __shared__ unsigned long long s_part[kCompactTasks / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t T = P.tasks_per_group;
    const uint32_t g = blockIdx.x;
    const uint32_t first = g * T;
    const uint32_t ntask_here = min(T, P.ntasks - first);
    const uint32_t task = first + tid;
    const bool mine = tid < ntask_here;
    const uint32_t cnt = mine ? P.counts[task] : 0u;
    const uint32_t slot_pts = P.slot_bytes / 8;
    const bool listed = cnt <= slot_pts;             // slot holds points (else its bitmap)
    uint32_t total, list_total;
    const uint32_t toff = block_exclusive_scan(cnt, s_wave_sum, total);
    const uint32_t loff = block_exclusive_scan(listed ? cnt : 0u, s_wave_sum, list_total);
    s_task_off[tid] = toff;
    s_list_off[tid] = loff;
    if (tid == 0) {
        s_task_off[kCompactTasks] = total;
        s_list_off[kCompactTasks] = list_total;
    }

    // the group's base: every band count is final when this kernel starts (the detector
    // kernel wrote them), so each group sums its predecessors' counts itself -- a few KB of
    // L2-resident reads, no cross-group hand-off
    unsigned long long part = 0;
    {   // 16-byte loads, several in flight per thread (P.counts is 16-byte aligned)
        const uint4* c4 = reinterpret_cast<const uint4*>(P.counts);
        const uint32_t n4 = first / 4;
#pragma unroll 4
        for (uint32_t i = tid; i < n4; i += kCompactTasks) {
            const uint4 v = c4[i];
            part += (unsigned long long)v.x + v.y + v.z + v.w;
        }
        for (uint32_t i = 4 * n4 + tid; i < first; i += kCompactTasks) part += P.counts[i];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d, 64);
    if (lane == 0) s_part[wave] = part;
    __syncthreads();
    unsigned long long base = 0;
#pragma unroll
    for (int w = 0; w < kCompactTasks / 64; ++w) base += s_part[w];
    if (mine) {
        const uint32_t frame = task / P.bands_per_frame;
        const uint32_t band = task - frame * P.bands_per_frame;
        if (band == 0) P.frame_offsets[frame] = base + toff;
        if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = base + toff + cnt;
    }

    // slot lists: output k of the group's listed points -> band i with
    // s_list_off[i] <= k < s_list_off[i + 1] (bands with bitmaps add nothing to that prefix)
    // (kCopyUnroll points per thread per round, their loads in flight together)
    constexpr int kCopyUnroll = 4;
    for (uint32_t k0 = tid; k0 < list_total; k0 += kCopyUnroll * kCompactTasks) {
        uint2 v[kCopyUnroll];
        unsigned long long o[kCopyUnroll];
#pragma unroll
        for (int q = 0; q < kCopyUnroll; ++q) {
            const uint32_t k = k0 + q * kCompactTasks;
            o[q] = ~0ull;
            v[q] = make_uint2(0u, 0u);
            if (k < list_total) {
                uint32_t lo = 0, hi = ntask_here;            // invariant: off[lo] <= k < off[hi]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_list_off[mid] <= k) lo = mid; else hi = mid;
                }
                const uint32_t j = k - s_list_off[lo];
                o[q] = base + s_task_off[lo] + j;
                v[q] = reinterpret_cast<const uint2*>(P.slots + (uint64_t)(first + lo) * P.slot_bytes)[j];
            }
        }
#pragma unroll
        for (int q = 0; q < kCopyUnroll; ++q)
            if (o[q] < P.cap) P.out[o[q]] = v[q];
    }

    // bitmap bands (more points than their slot holds): the whole group expands each one,
    // kExpandWords consecutive words per thread per round (16-byte loads, all in flight), a
    // block scan of the threads' point counts giving every thread its output position
    constexpr uint32_t kExpandWords = 8;
    for (uint32_t i = 0; i < ntask_here; ++i) {          // uniform over the group
        const uint32_t n = s_task_off[i + 1 < ntask_here ? i + 1 : kCompactTasks] - s_task_off[i];
        if (n <= slot_pts) continue;
        const uint32_t tk = first + i;
        const uint8_t* slot = P.slots + (uint64_t)tk * P.slot_bytes;
        const uint32_t frame = tk / P.bands_per_frame;
        const uint32_t band = tk - frame * P.bands_per_frame;
        const uint32_t y0 = 3 + band * P.rows;
        const uint32_t rows = min(P.rows, P.height - 3 - y0);
        const uint32_t nwords = rows * P.words_per_row;
        // the slot is 16-byte aligned and a multiple of 16 bytes long, so a 16-byte load
        // starting below nwords stays inside it; words from nwords on are masked
        const uint4* words4 = reinterpret_cast<const uint4*>(slot);
        unsigned long long o = base + s_task_off[i];
        for (uint32_t w0 = 0; w0 < nwords; w0 += kExpandWords * kCompactTasks) {
            const uint32_t wt = w0 + tid * kExpandWords;   // this thread's first word
            uint32_t bits[kExpandWords];
#pragma unroll
            for (uint32_t q = 0; q < kExpandWords / 4; ++q) {
                const uint32_t w = wt + 4 * q;
                const uint4 v = w < nwords ? words4[w / 4] : make_uint4(0u, 0u, 0u, 0u);
                bits[4 * q] = v.x; bits[4 * q + 1] = v.y; bits[4 * q + 2] = v.z; bits[4 * q + 3] = v.w;
            }
            uint32_t c = 0;
#pragma unroll
            for (uint32_t q = 0; q < kExpandWords; ++q) {
                if (wt + q >= nwords) bits[q] = 0u;
                c += __popc(bits[q]);
            }
            uint32_t round_total;
            unsigned long long k = o + block_exclusive_scan(c, s_wave_sum, round_total);
#pragma unroll
            for (uint32_t q = 0; q < kExpandWords; ++q) {
                const uint32_t w = wt + q;
                const uint32_t r = w / P.words_per_row;
                const uint32_t xb = (w - r * P.words_per_row) * 32;
                uint32_t bq = bits[q];
                while (bq) {
                    const uint32_t bit = __builtin_ctz(bq);
                    bq &= bq - 1;
                    if (k < P.cap) P.out[k] = make_uint2(xb + bit, y0 + r);
                    ++k;
                }
            }
            o += round_total;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Point scoring (extension, fdf_score_points): literal formulas of the reference's score
// functions, valid for any point, one thread per point.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint16_t score_point(const uint8_t* img, uint32_t W, uint2 pt,
                                                uint32_t nms, uint32_t t, uint32_t n) {
    const int c = img[(uint64_t)pt.y * W + pt.x];
    int d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        d[i] = c - (int)img[(uint64_t)((int)pt.y + circle_dy(i)) * W + (int)pt.x + circle_dx(i)];
    uint32_t score;
    if (nms == kNmsSumAbsolute) {    // src/fast_simd.rs:722-749
        uint32_t sb = 0, sd = 0;
        for (int i = 0; i < 16; ++i) {
            sb += (uint32_t)max(d[i] - (int)t, 0);
            sd += (uint32_t)max(-d[i] - (int)t, 0);
        }
        score = max(sb, sd);
    } else {                          // src/fast_simd.rs:623-718
        int hi = -32768, lo = 32767;
        for (int kk = 0; kk < 16; ++kk) {
            int mn = 32767, mx = -32768;
            for (uint32_t i = 0; i < n; ++i) {
                mn = min(mn, d[(kk + i) & 15]);
                mx = max(mx, d[(kk + i) & 15]);
            }
            hi = max(hi, mn);
            lo = min(lo, mx);
        }
        score = (uint32_t)min(abs(hi), abs(lo));
    }
    return (uint16_t)score;
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

hipError_t launch_compact(const CompactParams& c, hipStream_t stream) {
    if (c.tasks_per_group == 0 || c.tasks_per_group > (uint32_t)kCompactTasks)
        return hipErrorInvalidValue;
    const uint32_t ngroups = (c.ntasks + c.tasks_per_group - 1) / c.tasks_per_group;
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
