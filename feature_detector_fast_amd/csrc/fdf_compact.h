// fdf_compact.h -- raster-order compaction of the detector's per-band slots (the body of
// compact_kernel in fdf_kernels.hip).
//
// Turns the per-band slots into the reference's output: one list of points per frame, in
// raster order (src/fast_simd.rs:589-616 pushes keypoints in scan order).  Group g covers
// tasks [g*T, g*T + T) (T = P.tasks_per_group <= kCompactTasks).  Its output base is the sum
// of the counts before it: from the per-group sums the detector accumulated (O(groups)), or
// from the counts themselves.  The points of the group's slot-list bands are copied
// cooperatively by all threads (output index -> band by binary search over an in-group
// prefix), so the writes are coalesced whatever the per-band counts; bitmap bands are
// expanded by the whole group.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdf_kernels.h"

namespace fdfk {

struct CompactShared {
    uint32_t task_off[kCompactTasks + 1];
    uint32_t list_off[kCompactTasks + 1];
    uint32_t wave_sum[kCompactTasks / 64];
    unsigned long long part[kCompactTasks / 64];
};

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

// One compaction group (all kCompactTasks threads of the workgroup take part).
__device__ __forceinline__ void compact_group(const CompactParams& P, uint32_t g, CompactShared& sm) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t T = P.tasks_per_group;
    if (g == 0 && tid == 0 && P.kp_stats) {
        // the launch's keypoint density for the host's next band-height choice
        const uint32_t v = *P.kp_stats;
        *P.kp_stats = 0u;
        *P.stats_out = ((uint64_t)P.stats_seq << 32) | v;
    }
    const uint32_t first = g * T;
    const uint32_t ntask_here = min(T, P.ntasks - first);
    const uint32_t task = first + tid;
    const bool mine = tid < ntask_here;
    const uint32_t cnt = mine ? P.counts[task] : 0u;
    const uint32_t slot_pts = P.slot_bytes / 8;
    const bool listed = cnt <= slot_pts;             // slot holds points (else its bitmap)

    // the group's base: every band count is final when this runs (the detector wrote them),
    // so each group sums its predecessors itself -- the per-group sums when the detector
    // accumulated them, else the counts (16-byte loads, several in flight per thread).
    // Loaded before the scans below: their barriers would otherwise order these loads
    // after the counts' round trip (one memory latency more per group; a single frame's
    // compaction is a chain of such latencies)
    unsigned long long part = 0;
    if (P.group_sums) {
        for (uint32_t i = tid; i < g; i += kCompactTasks) part += P.group_sums[i];
        // and clear the other buffer for the next launch
        const uint32_t ngroups = (P.ntasks + T - 1) / T;
        for (uint32_t i = g * kCompactTasks + tid; i < kMaxGroupSums; i += ngroups * kCompactTasks)
            P.next_sums[i] = 0u;
    } else {
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
    if (lane == 0) sm.part[wave] = part;

    uint32_t total, list_total;
    const uint32_t toff = block_exclusive_scan(cnt, sm.wave_sum, total);
    const uint32_t loff = block_exclusive_scan(listed ? cnt : 0u, sm.wave_sum, list_total);
    sm.task_off[tid] = toff;
    sm.list_off[tid] = loff;
    if (tid == 0) {
        sm.task_off[kCompactTasks] = total;
        sm.list_off[kCompactTasks] = list_total;
    }
    __syncthreads();
    unsigned long long base = 0;
#pragma unroll
    for (int w = 0; w < kCompactTasks / 64; ++w) base += sm.part[w];
    if (mine) {
        const uint32_t frame = task / P.bands_per_frame;
        const uint32_t band = task - frame * P.bands_per_frame;
        if (band == 0) P.frame_offsets[frame] = base + toff;
        if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = base + toff + cnt;
    }

    // slot lists: output k of the group's listed points -> band i with
    // list_off[i] <= k < list_off[i + 1] (bands with bitmaps add nothing to that prefix)
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
                    if (sm.list_off[mid] <= k) lo = mid; else hi = mid;
                }
                const uint32_t j = k - sm.list_off[lo];
                o[q] = base + sm.task_off[lo] + j;
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
        const uint32_t n = sm.task_off[i + 1 < ntask_here ? i + 1 : kCompactTasks] - sm.task_off[i];
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
        unsigned long long o = base + sm.task_off[i];
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
            unsigned long long k = o + block_exclusive_scan(c, sm.wave_sum, round_total);
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

}  // namespace fdfk
