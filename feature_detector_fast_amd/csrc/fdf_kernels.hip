// fdf_kernels.hip -- FAST-9..16 corner detection for MI355X (gfx950, CDNA4).
//
// Two kernels replace the reference's hot path below the host/device boundary:
// detect<NONMAX>() (iwanders/feature_detector_fast src/fast_simd.rs:301-620) with
// determine_keypoint (:115-297) and the NMS score functions (:623-718, :722-749).
//
// fast_band_kernel -- one workgroup per band of R full-width centre rows of one frame
// (DESIGN.md §3).  The band is swept in 1024-column chunks staged into LDS; per chunk:
//   * pre-filter: a lane takes a 4-pixel group (one LDS dword) and runs the cardinal test
//     on all 4 bytes at once.  v_lerp_u8 gives exact per-byte comparisons: with
//     v = lerp(X, ~c, r) = (X - c + 255 + r) >> 1, "X - c > t" is bit 7 of lerp(v, Kb, 0)
//     for r = t & 1, Kb = 128 - ceil(t/2); "X - c < -t" is the complement of bit 7 of
//     lerp(lerp(X, ~c, 1 - (t & 1)), Kd, 0), Kd = 255 - ((254 - t + (1 - (t & 1))) >> 1).
//     2-of-4 adjacent cardinals (src/fast_simd.rs:441-472) and 3-of-4 (:473-506) are then
//     bitwise logic on the flags.  The pre-filter is only a necessary condition.
//   * candidate queues: groups with candidates go to a per-wave LDS queue; 16 groups at a
//     time are expanded into a per-wave queue of candidate pixels.
//   * full test, 64 candidate pixels per wave: the 16 circle bytes come from LDS with
//     immediate offsets; the 32 bright/dark classifications are wave ballots (bit-sliced
//     masks over the 64 lanes) and the cyclic run test is scalar 64-bit AND/OR.
//   * NMS: scores go to an LDS score map with a 1-pixel ring (u8 for max-threshold, whose
//     score is <= 255; u16 for SAD); keypoints of the chunk's own pixels go to a list and
//     the 3x3 strict-max test (:589-616) runs over that list into an LDS band bitmap.
//   * output: the band's points in raster order go to its fixed-size slot (or, if they do
//     not fit, its bitmap) with the count in counts[task]; no inter-workgroup waiting.
// compact_kernel -- scans the band counts in raster order (decoupled look-back over
//   workgroups of 256 bands) and copies each band's slot to its final position.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fdf_common.h"
#include "fdf_kernels.h"

namespace fdfk {

// Cardinal pre-filter of the 4 centres at `px` (tile address of the group's first byte).
// Returns bit 7 of byte j set iff centre j passes (a necessary condition for a keypoint).
template <int N>
__device__ __forceinline__ uint32_t prefilter_group(const uint8_t* px, const LerpConsts& k) {
    const uint32_t c = *reinterpret_cast<const uint32_t*>(px);
    const uint32_t l = *reinterpret_cast<const uint32_t*>(px - 4);
    const uint32_t r = *reinterpret_cast<const uint32_t*>(px + 4);
    const uint32_t n = *reinterpret_cast<const uint32_t*>(px - 3 * kPitch);
    const uint32_t s = *reinterpret_cast<const uint32_t*>(px + 3 * kPitch);
    const uint32_t nc = ~c;
    const uint32_t e = alignbyte(r, c, 3);   // x+3 .. x+6
    const uint32_t w = alignbyte(c, l, 1);   // x-3 .. x
    // bright: bit 7 <=> X - c > t ; ndark: bit 7 <=> NOT(X - c < -t)
    const uint32_t bn = lerp_u8(lerp_u8(n, nc, k.rb), k.kb, 0);
    const uint32_t be = lerp_u8(lerp_u8(e, nc, k.rb), k.kb, 0);
    const uint32_t bs = lerp_u8(lerp_u8(s, nc, k.rb), k.kb, 0);
    const uint32_t bw = lerp_u8(lerp_u8(w, nc, k.rb), k.kb, 0);
    const uint32_t dn = lerp_u8(lerp_u8(n, nc, k.rd), k.kd, 0);
    const uint32_t de = lerp_u8(lerp_u8(e, nc, k.rd), k.kd, 0);
    const uint32_t ds = lerp_u8(lerp_u8(s, nc, k.rd), k.kd, 0);
    const uint32_t dw = lerp_u8(lerp_u8(w, nc, k.rd), k.kd, 0);
    uint32_t bright, not_dark;
    if constexpr (N < 12) {
        // 2 adjacent of 4 <=> (N|S) & (E|W)  (every N/S-E/W pair is adjacent)
        bright = (bn | bs) & (be | bw);
        not_dark = (dn & ds) | (de & dw);                       // NOT((dN|dS) & (dE|dW))
    } else {
        // 3 of 4 (any three cardinals are consecutive)
        bright = (bn & bs & (be | bw)) | (be & bw & (bn | bs));
        not_dark = (dn & ds) | (de & dw) | ((dn | ds) & (de | dw));   // >= 2 not dark
    }
    return (bright | ~not_dark) & kHigh;
}

template <typename ScoreT>
struct Smem {
    uint8_t* tile;       // (R+8) x kPitch input bytes; tile (r, c) = image (y0-4+r, X0-16+c)
    ScoreT* scores;      // (R+2) x kScorePitch; score (s, col) = image (y0-1+s, X0-4+col)
    uint32_t* bitmap;    // R x words_per_row keep-bits of the band
    uint32_t* gq_item;   // kWaves x kGroupQ queued groups: (s << 12) | gi
    uint32_t* gq_cand;   // kWaves x kGroupQ candidate flags (bit 7 of byte j = pixel j)
    uint32_t* pq;        // kWaves x kPixelQ queued pixels: (s << 12) | col
    uint32_t* kp_list;   // kKpCap keypoints of the chunk's own pixels: (s << 16) | col
    uint32_t* misc;      // [0] keypoint-list length, [4..] per-wave sums
};

template <typename ScoreT>
__device__ __forceinline__ Smem<ScoreT> carve(uint8_t* base, const LdsLayout& L) {
    Smem<ScoreT> s;
    s.tile = base + L.tile;
    s.scores = reinterpret_cast<ScoreT*>(base + L.scores);
    s.bitmap = reinterpret_cast<uint32_t*>(base + L.bitmap);
    s.gq_item = reinterpret_cast<uint32_t*>(base + L.gq_item);
    s.gq_cand = reinterpret_cast<uint32_t*>(base + L.gq_cand);
    s.pq = reinterpret_cast<uint32_t*>(base + L.pq);
    s.kp_list = reinterpret_cast<uint32_t*>(base + L.kp_list);
    s.misc = reinterpret_cast<uint32_t*>(base + L.misc);
    return s;
}

struct ChunkCtx {
    uint32_t t;        // threshold
    uint32_t X0;       // first image column of the chunk
    uint32_t rows;     // centre rows of the band
    uint32_t nw;       // bitmap words per row
};

// Full test of `count` (<= 64) queued pixels, one per lane, starting at pq[0].
template <int NMS, int N, typename ScoreT>
__device__ __forceinline__ void test_pixels(const Smem<ScoreT>& sm, const uint32_t* pq,
                                            uint32_t count, const ChunkCtx& cc, uint32_t lane) {
    const bool act = lane < count;
    const uint32_t code = act ? pq[lane] : 0u;
    const uint32_t s = code >> 12, col = code & 0xfffu;
    // top-left of the 7x7 neighbourhood: tile row (s+3)-3, tile column (12+col)-3
    const uint8_t* nb = sm.tile + s * kPitch + 9 + col;
    const uint32_t c = nb[3 * kPitch + 3];
    uint32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = nb[(circle_dy(i) + 3) * kPitch + circle_dx(i) + 3];
    const int upper = (int)(c + cc.t), lower = (int)c - (int)cc.t;
    const uint64_t active = wave_ballot(act);
    uint64_t bright[16], dark[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bright[i] = wave_ballot((int)p[i] > upper) & active;
    const uint64_t kb = arc_test<N>(bright);
    __builtin_amdgcn_sched_barrier(0);   // keep the two polarities' 32 masks from co-residing
#pragma unroll
    for (int i = 0; i < 16; ++i) dark[i] = wave_ballot((int)p[i] < lower) & active;
    const uint64_t kd = arc_test<N>(dark);
    if (!(((kb | kd) >> lane) & 1u)) return;
    if constexpr (NMS == kNmsOff) {
        const uint32_t x = cc.X0 - 4 + col;
        atomicOr(&sm.bitmap[(s - 1) * cc.nw + (x >> 5)], 1u << (x & 31));
    } else {
        const uint32_t score = NMS == kNmsMaxThreshold
                                   ? score_max_threshold<N>(c, p, ((kd >> lane) & 1u) != 0)
                                   : score_sum_abs(c, p, cc.t);
        sm.scores[s * kScorePitch + col] = (ScoreT)score;
        // the band's own rows and the chunk's own columns go to the NMS list
        if (s >= 1 && s <= cc.rows && col >= 4 && col < 4 + kChunk) {
            const uint32_t k = atomicAdd(&sm.misc[0], 1u);
            if (k < kKpCap) sm.kp_list[k] = (s << 16) | col;
        }
    }
}

// Expand `ng` (<= 16) queued groups into the pixel queue; returns the new pixel count.
__device__ __forceinline__ uint32_t expand_groups(const uint32_t* gi_q, const uint32_t* gc_q,
                                                  uint32_t ng, uint32_t* pq, uint32_t pcount,
                                                  uint32_t lane) {
    const bool act = lane < ng;
    const uint32_t item = act ? gi_q[lane] : 0u;
    const uint32_t cand = act ? gc_q[lane] : 0u;
    const uint32_t cnt = __popc(cand);
    const uint64_t b0 = wave_ballot(cnt > 0), b1 = wave_ballot(cnt > 1);
    const uint64_t b2 = wave_ballot(cnt > 2), b3 = wave_ballot(cnt > 3);
    uint32_t pos = pcount + lanes_below(b0) + lanes_below(b1) + lanes_below(b2) +
                   lanes_below(b3);
    const uint32_t code = ((item >> 12) << 12) | (4 * (item & 0xfffu));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (cand & (0x80u << (8 * j))) pq[pos++] = code + j;
    }
    return pcount + (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
}

template <typename ScoreT>
__device__ __forceinline__ bool nms_keep(const ScoreT* sc) {
    const uint32_t v = sc[0];
    constexpr int P = kScorePitch;
    return v > sc[-P - 1] && v > sc[-P] && v > sc[-P + 1] && v > sc[-1] && v > sc[1] &&
           v > sc[P - 1] && v > sc[P] && v > sc[P + 1];
}

template <int NMS, int N>
__global__ __launch_bounds__(kThreads) void fast_band_kernel(BandParams P) {
    using ScoreT = typename std::conditional<NMS == kNmsSumAbsolute, uint16_t, uint8_t>::type;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const LdsLayout L = make_layout(P.rows, P.words_per_row, score_bytes_for(NMS));
    const Smem<ScoreT> sm = carve<ScoreT>(smem_raw, L);
    const uint32_t tid = threadIdx.x;
    // wave index as a provably wave-uniform (SGPR) value: loops bounded by it stay uniform
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
    const uint32_t W = P.width, H = P.height, nw = P.words_per_row, t = P.threshold;

    // ---- task: XCD-aware static mapping.  Blocks b and b+8 share an XCD (round-robin
    //      dispatch), so XCD k gets a contiguous run of bands and their shared halo rows
    //      stay in its L2.  Bijective for any ntasks.
    const uint32_t b = blockIdx.x;
    const uint32_t q8 = P.ntasks >> 3, r8 = P.ntasks & 7, k8 = b & 7;
    const uint32_t task = k8 * q8 + min(k8, r8) + (b >> 3);
    const uint32_t frame = task / P.bands_per_frame;
    const uint32_t band = task - frame * P.bands_per_frame;
    const uint32_t y0 = 3 + band * P.rows;                          // first centre row
    const uint32_t rows = min(P.rows, H - 3 - y0);                  // centre rows in band
    const uint8_t* img = P.frames + (uint64_t)frame * P.frame_stride;

    if (t >= 255) {                                                  // no pixel can pass
        if (tid == 0) P.counts[task] = 0;
        return;
    }
    const LerpConsts lk = lerp_consts(t);
    for (uint32_t i = tid; i < rows * nw; i += kThreads) sm.bitmap[i] = 0;

    // score rows s <-> image row y0 - 1 + s; the 1-row ring exists only for NMS
    const uint32_t s_lo = NMS == kNmsOff ? 1 : 0;
    const uint32_t s_hi = NMS == kNmsOff ? rows + 1 : rows + 2;
    const uint32_t tr_lo = NMS == kNmsOff ? 1 : 0;                  // tile rows to load
    const uint32_t tr_hi = NMS == kNmsOff ? rows + 7 : rows + 8;
    const bool aligned_rows = (W & 15) == 0 && ((uintptr_t)img & 15) == 0;

    for (uint32_t X0 = 0; X0 < W - 3; X0 += kChunk) {
        __syncthreads();   // previous chunk's readers are done with the tile
        // ---- stage tile rows [tr_lo, tr_hi) x columns [X0-16, X0+kChunk+16) into LDS
        constexpr uint32_t kVecPerRow = kPitch / 16;
        const uint32_t nvec = (P.flags & kFlagNoLoad) ? 0u : (tr_hi - tr_lo) * kVecPerRow;
        for (uint32_t v = tid; v < nvec; v += kThreads) {
            const uint32_t tr = tr_lo + v / kVecPerRow;
            const uint32_t tv = v % kVecPerRow;
            const int y = (int)y0 - 4 + (int)tr;
            const int xc = (int)X0 - 16 + 16 * (int)tv;
            uint4 val = make_uint4(0, 0, 0, 0);
            if (y >= 0 && y < (int)H && xc < (int)W && xc + 16 > 0) {
                const uint8_t* src = img + (uint64_t)y * W + xc;
                if (aligned_rows && xc >= 0 && xc + 16 <= (int)W) {
                    val = *reinterpret_cast<const uint4*>(src);
                } else {
                    uint8_t bb[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const int x = xc + k;
                        bb[k] = (x >= 0 && x < (int)W) ? src[k] : 0;
                    }
                    val = *reinterpret_cast<uint4*>(bb);
                }
            }
            *reinterpret_cast<uint4*>(sm.tile + tr * kPitch + tv * 16) = val;
        }
        if (NMS != kNmsOff && tid == 0) sm.misc[0] = 0;
        __syncthreads();

        // ---- groups gi <-> image columns X0-4+4gi .. +3, limited to those touching the
        //      needed columns: centres [X0, X0+kChunk) within [3, W-3), plus for NMS the
        //      ring columns X0-1 and X0+kChunk clamped to [2, W-3] (ring cells outside the
        //      centre domain are processed so their score is written as 0)
        const int need_lo = NMS == kNmsOff ? max((int)X0, 3) : max((int)X0 - 1, 2);
        const int need_hi = NMS == kNmsOff ? min((int)X0 + kChunk - 1, (int)W - 4)
                                           : min((int)X0 + kChunk, (int)W - 3);
        const uint32_t g_lo = (uint32_t)(need_lo - ((int)X0 - 4)) >> 2;
        const uint32_t g_hi = ((uint32_t)(need_hi - ((int)X0 - 4)) >> 2) + 1;
        const uint32_t ng = g_hi - g_lo;
        // item rows: score rows whose image row is a centre row (3 <= y < H-3); ring rows
        // outside the centre domain only need zero scores
        const uint32_t si_lo = max(s_lo, y0 < 4 ? 4 - y0 : 0u);
        const uint32_t si_hi = min(s_hi, H - 2 - y0);
        const uint32_t nitems =
            (P.flags & kFlagNoPrefilter) || si_hi <= si_lo ? 0u : (si_hi - si_lo) * ng;
        if constexpr (NMS != kNmsOff) {
            for (uint32_t ss = s_lo; ss < s_hi; ++ss) {
                if (ss >= si_lo && ss < si_hi) continue;
                for (uint32_t k = tid; k < kScorePitch; k += kThreads)
                    sm.scores[ss * kScorePitch + k] = 0;
            }
        }
        const ChunkCtx cc{t, X0, rows, nw};

        uint32_t* gqi = sm.gq_item + wave * kGroupQ;
        uint32_t* gqc = sm.gq_cand + wave * kGroupQ;
        uint32_t* pq = sm.pq + wave * kPixelQ;
        uint32_t gcount = 0, pcount = 0;
        const bool no_test = (P.flags & kFlagNoFullTest) != 0;
        const bool col_edges = X0 < 4 || X0 + kChunk + 4 > W - 3;   // some group is clipped
        // this lane's first item, then advance by kThreads items per round; `toff` tracks
        // the tile offset of the group's first byte: (s + 3) * kPitch + 12 + 4 * gi
        uint32_t item = wave * 64 + lane;
        uint32_t s = si_lo + item / ng;
        uint32_t gi = g_lo + item % ng;
        uint32_t toff = (s + 3) * kPitch + 12 + 4 * gi;
        for (uint32_t base = wave * 64; base < nitems; base += kThreads) {
            uint32_t cand = 0;
            if (item < nitems) {
                cand = prefilter_group<N>(sm.tile + toff, lk);
                if (col_edges) {
                    const int x0 = (int)X0 - 4 + 4 * (int)gi;
                    if (x0 < 3 || x0 + 4 > (int)W - 3) {
                        uint32_t vm = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (x0 + j >= 3 && x0 + j < (int)W - 3) vm |= 0x80u << (8 * j);
                        cand &= vm;
                    }
                }
                if constexpr (NMS != kNmsOff) {
                    // score (s, 4gi) = s * kScorePitch + 4 gi = toff - 3 kPitch - 12 - 16 s
                    ScoreT* sp = sm.scores + (toff - 3 * kPitch - 12 - (s << 4));
                    if constexpr (sizeof(ScoreT) == 1) *reinterpret_cast<uint32_t*>(sp) = 0;
                    else *reinterpret_cast<uint2*>(sp) = make_uint2(0, 0);
                }
            }
            const uint64_t bal = wave_ballot(cand != 0);
            if (cand != 0) {
                const uint32_t pos = gcount + lanes_below(bal);
                gqi[pos] = (s << 12) | gi;
                gqc[pos] = cand;
            }
            gcount += (uint32_t)__popcll(bal);
            if (no_test) gcount = 0;
            while (gcount >= 16) {
                gcount -= 16;
                pcount = expand_groups(gqi + gcount, gqc + gcount, 16, pq, pcount, lane);
                while (pcount >= 64) {
                    pcount -= 64;
                    test_pixels<NMS, N>(sm, pq + pcount, 64, cc, lane);
                }
            }
            item += kThreads;
            gi += kThreads;
            toff += 4 * kThreads;
            while (gi >= g_hi) {
                gi -= ng;
                ++s;
                toff += kPitch - 4 * ng;
            }
        }
        if (gcount > 0) pcount = expand_groups(gqi, gqc, gcount, pq, pcount, lane);
        while (pcount > 0) {
            const uint32_t take = min(pcount, 64u);
            pcount -= take;
            test_pixels<NMS, N>(sm, pq + pcount, take, cc, lane);
        }

        if constexpr (NMS != kNmsOff) {
            __syncthreads();
            const uint32_t nkp = sm.misc[0];
            if (nkp <= kKpCap) {
                for (uint32_t k = tid; k < nkp; k += kThreads) {
                    const uint32_t ent = sm.kp_list[k];
                    const uint32_t ss = ent >> 16, col = ent & 0xffffu;
                    const uint32_t y = y0 - 1 + ss;
                    if (y == 3 || y == H - 4) continue;              // src/fast_simd.rs:590
                    if (nms_keep(sm.scores + ss * kScorePitch + col)) {
                        const uint32_t x = X0 - 4 + col;
                        atomicOr(&sm.bitmap[(ss - 1) * nw + (x >> 5)], 1u << (x & 31));
                    }
                }
            } else {
                // keypoint list overflowed: dense pass over the chunk's own pixels
                const uint32_t npx = rows * kChunk;
                for (uint32_t k = tid; k < npx; k += kThreads) {
                    const uint32_t ss = 1 + k / kChunk, col = 4 + k % kChunk;
                    const uint32_t x = X0 - 4 + col, y = y0 - 1 + ss;
                    if (x < 3 || x >= W - 3 || y == 3 || y == H - 4) continue;
                    const ScoreT* sc = sm.scores + ss * kScorePitch + col;
                    if (sc[0] != 0 && nms_keep(sc))
                        atomicOr(&sm.bitmap[(ss - 1) * nw + (x >> 5)], 1u << (x & 31));
                }
            }
        }
    }
    __syncthreads();

    // ---- count keep-bits: thread `tid` owns a contiguous run of bitmap words
    const uint32_t nwords = rows * nw;
    const uint32_t per = (nwords + kThreads - 1) / kThreads;
    const uint32_t w_lo = min(tid * per, nwords), w_hi = min(w_lo + per, nwords);
    uint32_t mine = 0;
    for (uint32_t w = w_lo; w < w_hi; ++w) mine += __popc(sm.bitmap[w]);
    uint32_t incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
    uint32_t* wave_sum = sm.misc + 4;
    if (lane == 63) wave_sum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t v = wave_sum[w];
        before += (uint32_t)w < wave ? v : 0u;
        total += v;
    }
    if (tid == 0) P.counts[task] = total;
    if (P.flags & kFlagNoEmit) return;

    // ---- band slot: points in raster order when they fit, else the keep-bitmap
    uint8_t* slot = P.slots + (uint64_t)task * P.slot_bytes;
    if (total <= P.slot_bytes / 8) {
        uint2* pts = reinterpret_cast<uint2*>(slot);
        uint32_t idx = before + incl - mine;
        for (uint32_t w = w_lo; w < w_hi; ++w) {
            uint32_t bits = sm.bitmap[w];
            const uint32_t r = w / nw;
            const uint32_t xb = (w - r * nw) * 32;
            while (bits) {
                const uint32_t bit = __builtin_ctz(bits);
                bits &= bits - 1;
                pts[idx++] = make_uint2(xb + bit, y0 + r);
            }
        }
    } else {
        uint32_t* words = reinterpret_cast<uint32_t*>(slot);
        for (uint32_t w = tid; w < nwords; w += kThreads) words[w] = sm.bitmap[w];
    }
}

// ---------------------------------------------------------------------------------------
// Compaction: raster-order prefix over band counts, then slot -> final position copy.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kCompactTasks) void compact_kernel(CompactParams P) {
    __shared__ uint32_t s_task_off[kCompactTasks];
    __shared__ uint32_t s_wave_sum[kCompactTasks / 64];
    __shared__ unsigned long long s_base;
    __shared__ uint32_t s_group;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t ngroups = (P.ntasks + kCompactTasks - 1) / kCompactTasks;
    if (tid == 0) {   // groups in dispatch order: a group's predecessors are resident or done
        const uint32_t g = atomicAdd(P.ticket, 1u);
        if (g == ngroups - 1) atomicExch(P.ticket, 0u);
        s_group = g;
    }
    __syncthreads();
    const uint32_t g = s_group;
    const uint32_t task = g * kCompactTasks + tid;
    const uint32_t cnt = task < P.ntasks ? P.counts[task] : 0u;
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
    if (lane == 63) s_wave_sum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kCompactTasks / 64; ++w) {
        const uint32_t v = s_wave_sum[w];
        before += (uint32_t)w < wave ? v : 0u;
        total += v;
    }
    s_task_off[tid] = before + incl - cnt;

    // decoupled look-back: wave 0 probes 64 predecessor groups per round
    if (wave == 0) {
        unsigned long long excl = 0;
        if (g == 0) {
            if (lane == 0)
                __hip_atomic_store(&P.state[0], lb_pack(P.epoch, 2, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&P.state[g], lb_pack(P.epoch, 1, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            int64_t top = (int64_t)g - 1;
            while (true) {
                const int64_t idx = top - (int64_t)lane;
                uint32_t flag = 2;                                   // before group 0: 0 incl.
                unsigned long long val = 0;
                if (idx >= 0) {
                    const unsigned long long wv = __hip_atomic_load(
                        &P.state[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    flag = (uint32_t)(wv >> 48) == P.epoch ? (uint32_t)(wv >> 46) & 3u : 0u;
                    val = wv & ((1ull << 46) - 1);
                }
                const uint64_t inc = wave_ballot(flag == 2);
                const uint64_t missing = wave_ballot(flag == 0);
                const uint64_t upto = inc ? (inc & (~inc + 1)) * 2 - 1 : ~0ull;
                if (missing & upto) {
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                unsigned long long part = ((upto >> lane) & 1) ? val : 0ull;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d, 64);
                excl += part;
                if (inc) break;
                top -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&P.state[g], lb_pack(P.epoch, 2, excl + total),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_base = excl;
    }
    __syncthreads();
    const unsigned long long base = s_base;
    if (task < P.ntasks) {
        const uint32_t frame = task / P.bands_per_frame;
        const uint32_t band = task - frame * P.bands_per_frame;
        if (band == 0) P.frame_offsets[frame] = base + s_task_off[tid];
        if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = base + s_task_off[tid] + cnt;
    }

    // copy: wave w handles tasks w, w+4, ... of the group
    const uint32_t ntask_here = min((uint32_t)kCompactTasks, P.ntasks - g * kCompactTasks);
    const uint32_t slot_pts = P.slot_bytes / 8;
    for (uint32_t i = wave; i < ntask_here; i += kCompactTasks / 64) {
        const uint32_t tk = g * kCompactTasks + i;
        const uint32_t n = P.counts[tk];
        if (n == 0) continue;
        const unsigned long long off = base + s_task_off[i];
        const uint8_t* slot = P.slots + (uint64_t)tk * P.slot_bytes;
        if (n <= slot_pts) {
            const uint2* src = reinterpret_cast<const uint2*>(slot);
            for (uint32_t k = lane; k < n; k += 64)
                if (off + k < P.cap) P.out[off + k] = src[k];
        } else {
            // dense band: expand its bitmap, 64 words per round, in raster order
            const uint32_t frame = tk / P.bands_per_frame;
            const uint32_t band = tk - frame * P.bands_per_frame;
            const uint32_t y0 = 3 + band * P.rows;
            const uint32_t rows = min(P.rows, P.height - 3 - y0);
            const uint32_t nwords = rows * P.words_per_row;
            const uint32_t* words = reinterpret_cast<const uint32_t*>(slot);
            unsigned long long o = off;
            for (uint32_t w0 = 0; w0 < nwords; w0 += 64) {
                const uint32_t w = w0 + lane;
                uint32_t bits = w < nwords ? words[w] : 0u;
                const uint32_t c = __popc(bits);
                uint32_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t v = __shfl_up(inc, d, 64);
                    if (lane >= (uint32_t)d) inc += v;
                }
                unsigned long long k = o + inc - c;
                const uint32_t r = w / P.words_per_row;
                const uint32_t xb = (w - r * P.words_per_row) * 32;
                while (bits) {
                    const uint32_t bit = __builtin_ctz(bits);
                    bits &= bits - 1;
                    if (k < P.cap) P.out[k] = make_uint2(xb + bit, y0 + r);
                    ++k;
                }
                o += __shfl(inc, 63, 64);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Point scoring (extension, fdf_score_points): literal formulas of the reference's score
// functions, valid for any point, one thread per point.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void score_points_kernel(const uint8_t* img, uint32_t W,
                                                           const uint2* pts, uint32_t npts,
                                                           uint32_t nms, uint32_t t,
                                                           uint32_t n, uint16_t* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npts) return;
    const uint2 pt = pts[k];
    const int c = img[(uint64_t)pt.y * W + pt.x];
    int d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        d[i] = c - (int)img[(uint64_t)((int)pt.y + circle_dy(i)) * W + (int)pt.x + circle_dx(i)];
    uint32_t score;
    if (nms == kNmsMaxThreshold) {   // src/fast_simd.rs:623-718
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
    } else {                          // src/fast_simd.rs:722-749
        uint32_t sb = 0, sd = 0;
        for (int i = 0; i < 16; ++i) {
            sb += (uint32_t)max(d[i] - (int)t, 0);
            sd += (uint32_t)max(-d[i] - (int)t, 0);
        }
        score = max(sb, sd);
    }
    out[k] = (uint16_t)score;
}

// ---------------------------------------------------------------------------------------
// Host-side dispatch: (nms, n) -> template instance.
// ---------------------------------------------------------------------------------------
typedef void (*BandKernelFn)(BandParams);

template <int NMS>
static BandKernelFn pick_n(uint32_t n) {
    switch (n) {
        case 9: return fast_band_kernel<NMS, 9>;
        case 10: return fast_band_kernel<NMS, 10>;
        case 11: return fast_band_kernel<NMS, 11>;
        case 12: return fast_band_kernel<NMS, 12>;
        case 13: return fast_band_kernel<NMS, 13>;
        case 14: return fast_band_kernel<NMS, 14>;
        case 15: return fast_band_kernel<NMS, 15>;
        case 16: return fast_band_kernel<NMS, 16>;
        default: return nullptr;
    }
}

static BandKernelFn pick(uint32_t nms, uint32_t n) {
    switch (nms) {
        case kNmsOff: return pick_n<kNmsOff>(n);
        case kNmsMaxThreshold: return pick_n<kNmsMaxThreshold>(n);
        case kNmsSumAbsolute: return pick_n<kNmsSumAbsolute>(n);
        default: return nullptr;
    }
}

hipError_t launch_detect(const BandParams& p, const CompactParams& c, uint32_t nms, uint32_t n,
                         hipStream_t stream) {
    BandKernelFn fn = pick(nms, n);
    if (!fn) return hipErrorInvalidValue;
    const LdsLayout L = make_layout(p.rows, p.words_per_row, score_bytes_for(nms));
    if (L.total > kMaxLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fn, dim3(p.ntasks), dim3(kThreads), L.total, stream, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_compact(c, stream);
}

hipError_t launch_compact(const CompactParams& c, hipStream_t stream) {
    const uint32_t ngroups = (c.ntasks + kCompactTasks - 1) / kCompactTasks;
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

}  // namespace fdfk
