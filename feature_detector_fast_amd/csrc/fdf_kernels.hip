// fdf_kernels.hip -- FAST-9..16 corner detection for MI355X (gfx950, CDNA4).
//
// One fused kernel replaces the reference's hot path below the host/device boundary:
// detect<NONMAX>() (iwanders/feature_detector_fast src/fast_simd.rs:301-620) together with
// determine_keypoint (:115-297) and the two NMS score functions (:623-718, :722-749).
//
// Work decomposition:
//   * task  = one band of R full-width centre rows of one frame; tasks are numbered in
//             output (raster, frame-major) order and handed out by a device-wide atomic
//             counter, so a task's predecessors are always resident or finished.
//   * chunk = the band is swept left to right in 1024-column chunks.  Each chunk's input
//             (R+8 rows x 1056 bytes, 16-B aligned) is staged into LDS with 16-B loads.
//   * pre-filter: each lane takes a 4-pixel group (one LDS dword), unpacks it into two
//             packed-u16 pairs and runs the cardinal test with v_pk_{max,min,sub}_u16.
//             Exact reformulation of src/fast_simd.rs:441-509: 2-of-4 adjacent cardinals
//             <=> min(max(N,S), max(E,W)) > c+t (dark: max(min(N,S), min(E,W)) < c-t);
//             3-of-4 <=> 2nd smallest > c+t (dark: 2nd largest < c-t).
//   * candidate queue: lanes whose group has a candidate append it to a per-wave LDS
//             queue; every 16 queued groups are tested densely (4 lanes per group).
//   * full test: the 16 circle bytes come from LDS with immediate offsets; the
//             bright/dark classifications become 32 wave ballots (bit-sliced masks over
//             64 candidates) and the cyclic run test runs on them as scalar 64-bit ANDs.
//   * NMS: scores go to an LDS score map (R+2 rows incl. the 1-pixel ring); keypoints of
//             the band's own rows go to an LDS list; the 3x3 strict-max test runs over that
//             list.  Keep-bits are set in an LDS band bitmap.
//   * ordered output: decoupled look-back across tasks yields each band's global offset;
//             the bitmap is expanded into (x, y) points already in raster order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdf_kernels.h"

namespace fdfk {

// ---------------------------------------------------------------------------------------
// Circle geometry: src/fast_simd.rs:79-98 (index 0 = north, clockwise).
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr int circle_dx(int i) {
    constexpr int dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    return dx[i];
}
__host__ __device__ constexpr int circle_dy(int i) {
    constexpr int dy[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};
    return dy[i];
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 pk_max(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 pk_min(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 pk_subs(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }

// v_perm_b32: bytes 0-3 of the 8-byte source {hi, lo} come from `lo`, 4-7 from `hi`;
// selector byte 0x0c produces 0x00.
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// Cardinal pre-filter for one pair of centres held as packed u16 (c, north, south, east,
// west); returns a u32 whose u16 halves are non-zero iff that centre is a candidate.
template <int N>
__device__ __forceinline__ uint32_t prefilter_pair(u16x2 c, u16x2 nn, u16x2 ss, u16x2 ee,
                                                   u16x2 ww, u16x2 t2) {
    const u16x2 upper = c + t2;             // no overflow in u16: c, t <= 255
    const u16x2 lower = pk_subs(c, t2);     // saturating: c - t clamped at 0
    const u16x2 a = pk_max(nn, ss), cmn = pk_min(nn, ss);
    const u16x2 b = pk_max(ee, ww), dmn = pk_min(ee, ww);
    u16x2 bv, dv;
    if constexpr (N < 12) {
        bv = pk_min(a, b);       // bright on 2 adjacent cardinals
        dv = pk_max(cmn, dmn);   // dark on 2 adjacent cardinals
    } else {
        const u16x2 p = pk_max(cmn, dmn), q = pk_min(a, b);
        bv = pk_min(p, q);       // 2nd smallest of the four cardinals
        dv = pk_max(p, q);       // 2nd largest
    }
    return as_u32(pk_subs(bv, upper)) | as_u32(pk_subs(lower, dv));
}

// Bytes 0..3 of the result are non-zero iff centre j of the group is a candidate.
template <int N>
__device__ __forceinline__ uint32_t prefilter_group(const uint8_t* tile_px, uint32_t t) {
    const uint32_t c = *reinterpret_cast<const uint32_t*>(tile_px);
    const uint32_t l = *reinterpret_cast<const uint32_t*>(tile_px - 4);
    const uint32_t r = *reinterpret_cast<const uint32_t*>(tile_px + 4);
    const uint32_t n = *reinterpret_cast<const uint32_t*>(tile_px - 3 * kPitch);
    const uint32_t s = *reinterpret_cast<const uint32_t*>(tile_px + 3 * kPitch);
    const u16x2 t2 = {(unsigned short)t, (unsigned short)t};
    // even centres (bytes 0, 2) and odd centres (bytes 1, 3) of the group
    const uint32_t even = prefilter_pair<N>(
        as_pk(perm(0, c, 0x0c020c00)), as_pk(perm(0, n, 0x0c020c00)),
        as_pk(perm(0, s, 0x0c020c00)),
        as_pk(perm(r, c, 0x0c050c03)),   // east:  x+3, x+5
        as_pk(perm(c, l, 0x0c030c01)),   // west:  x-3, x-1
        t2);
    const uint32_t odd = prefilter_pair<N>(
        as_pk(perm(0, c, 0x0c030c01)), as_pk(perm(0, n, 0x0c030c01)),
        as_pk(perm(0, s, 0x0c030c01)),
        as_pk(perm(r, c, 0x0c060c04)),   // east:  x+4, x+6
        as_pk(perm(c, l, 0x0c040c02)),   // west:  x-2, x
        t2);
    return even | (odd << 8);            // halves <= 255, so bytes = centres 0..3
}

// Cyclic run test on bit-sliced masks: bit k of b[i] = "lane k's circle pixel i qualifies".
// Returns the lanes whose ring holds a run of >= N qualifying pixels (src/fast_simd.rs:247-295).
template <int N>
__device__ __forceinline__ uint64_t arc_test(const uint64_t (&b)[16]) {
    uint64_t p2[16], p4[16], p8[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p2[i] = b[i] & b[(i + 1) & 15];
#pragma unroll
    for (int i = 0; i < 16; ++i) p4[i] = p2[i] & p2[(i + 2) & 15];
#pragma unroll
    for (int i = 0; i < 16; ++i) p8[i] = p4[i] & p4[(i + 4) & 15];
    uint64_t any = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) any |= p8[i] & p8[(i + N - 8) & 15];
    return any;
}

// Max-threshold score of a keypoint (src/fast_simd.rs:623-718, scalar :172-209).  For
// 9 <= N any two N-windows of the 16-ring intersect, so min(|eh|, |el|) equals the arc
// strength of the keypoint's own polarity: bright -> max_k min_{w_k} p - c,
// dark -> c - min_k max_{w_k} p.  Dark is mapped onto bright with p -> 255 - p.
template <int N>
__device__ __forceinline__ uint32_t score_max_threshold(uint32_t c, const uint32_t (&p)[16],
                                                        bool dark) {
    const uint32_t m = dark ? 0xffu : 0u;
    uint32_t q[16], m3[16], m6[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) q[i] = p[i] ^ m;
#pragma unroll
    for (int i = 0; i < 16; ++i) m3[i] = min(min(q[i], q[(i + 1) & 15]), q[(i + 2) & 15]);
#pragma unroll
    for (int i = 0; i < 16; ++i) m6[i] = min(m3[i], m3[(i + 3) & 15]);
    // window [i, i+N) = [i, i+6) u [i+K, i+K+6) u [i+N-6, i+N), contiguous for K below
    constexpr int K = N > 12 ? N - 12 : 0;
    uint32_t best = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        best = max(best, min(min(m6[i], m6[(i + K) & 15]), m6[(i + N - 6) & 15]));
    }
    return best - (c ^ m);
}

// Sum-of-absolute-differences score (src/fast_simd.rs:722-749, scalar :278-299).
__device__ __forceinline__ uint32_t score_sum_abs(uint32_t c, const uint32_t (&p)[16],
                                                  uint32_t t) {
    const int upper = (int)(c + t), lower = (int)c - (int)t;
    uint32_t sb = 0, sd = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        sb += (uint32_t)max((int)p[i] - upper, 0);
        sd += (uint32_t)max(lower - (int)p[i], 0);
    }
    return max(sb, sd);
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

struct Smem {
    uint8_t* tile;       // (R+8) x kPitch input bytes
    uint16_t* scores;    // (R+2) x kScorePitch u16 scores (NMS only)
    uint32_t* bitmap;    // R x words_per_row keep-bits of the band
    uint32_t* q_item;    // kWaves x kQueueCap queued groups: (s << 12) | gi
    uint32_t* q_cand;    // kWaves x kQueueCap candidate bytes of the queued group
    uint32_t* kp_list;   // kKpCap keypoints of the band's own rows: (s << 16) | score col
    uint32_t* misc;      // [0] keypoint-list length, [1] look-back result lo/hi, wave sums
};

__device__ __forceinline__ Smem carve(uint8_t* base, const LdsLayout& L) {
    Smem s;
    s.tile = base + L.tile;
    s.scores = reinterpret_cast<uint16_t*>(base + L.scores);
    s.bitmap = reinterpret_cast<uint32_t*>(base + L.bitmap);
    s.q_item = reinterpret_cast<uint32_t*>(base + L.q_item);
    s.q_cand = reinterpret_cast<uint32_t*>(base + L.q_cand);
    s.kp_list = reinterpret_cast<uint32_t*>(base + L.kp_list);
    s.misc = reinterpret_cast<uint32_t*>(base + L.misc);
    return s;
}

// Dense test of up to 16 queued groups, 4 lanes per group (lane = 4*entry + pixel).
template <int NMS, int N>
__device__ __forceinline__ void test_queued(const Smem& sm, const uint32_t* qi,
                                            const uint32_t* qc, uint32_t count, uint32_t t,
                                            uint32_t X0, uint32_t rows, uint32_t nw) {
    const uint32_t lane = lane_id();
    const uint32_t e = lane >> 2, j = lane & 3;
    bool act = e < count;
    const uint32_t item = act ? qi[e] : 0u;
    const uint32_t cand = act ? qc[e] : 0u;
    act = act && ((cand >> (8 * j)) & 0xffu) != 0;
    const uint32_t s = item >> 12, gi = item & 0xfffu;
    // top-left of the 7x7 neighbourhood: tile row (s+3)-3, tile column (12+4gi+j)-3
    const uint8_t* nb = sm.tile + s * kPitch + 9 + 4 * gi + j;
    const uint32_t c = nb[3 * kPitch + 3];
    uint32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = nb[(circle_dy(i) + 3) * kPitch + circle_dx(i) + 3];
    const int upper = (int)(c + t), lower = (int)c - (int)t;
    uint64_t bright[16], dark[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bright[i] = __ballot(act && (int)p[i] > upper);
    const uint64_t kb = arc_test<N>(bright);
#pragma unroll
    for (int i = 0; i < 16; ++i) dark[i] = __ballot(act && (int)p[i] < lower);
    const uint64_t kd = arc_test<N>(dark);
    const bool is_kp = ((kb | kd) >> lane) & 1u;
    if (!is_kp) return;
    const uint32_t col = 4 * gi + j;                   // score-map column
    if constexpr (NMS == kNmsOff) {
        const uint32_t x = X0 - 4 + col;
        atomicOr(&sm.bitmap[(s - 1) * nw + (x >> 5)], 1u << (x & 31));
    } else {
        const uint32_t score = NMS == kNmsMaxThreshold
                                   ? score_max_threshold<N>(c, p, ((kd >> lane) & 1u) != 0)
                                   : score_sum_abs(c, p, t);
        sm.scores[s * kScorePitch + col] = (uint16_t)score;
        // the band's own rows and the chunk's own columns go to the NMS list
        if (s >= 1 && s <= rows && col >= 4 && col < 4 + kChunk) {
            const uint32_t k = atomicAdd(&sm.misc[0], 1u);
            if (k < kKpCap) sm.kp_list[k] = (s << 16) | col;
        }
    }
}

__device__ __forceinline__ bool nms_keep(const uint16_t* sc) {
    const uint32_t v = sc[0];
    constexpr int P = kScorePitch;
    return v > sc[-P - 1] && v > sc[-P] && v > sc[-P + 1] && v > sc[-1] && v > sc[1] &&
           v > sc[P - 1] && v > sc[P] && v > sc[P + 1];
}

__device__ __forceinline__ unsigned long long lb_pack(uint32_t epoch, uint32_t flag,
                                                      unsigned long long value) {
    return ((unsigned long long)epoch << 48) | ((unsigned long long)flag << 46) | value;
}

template <int NMS, int N>
__global__ __launch_bounds__(kThreads) void fast_band_kernel(BandParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const LdsLayout L = make_layout(P.rows, P.words_per_row, NMS != kNmsOff);
    const Smem sm = carve(smem_raw, L);
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6;
    const uint32_t lane = tid & 63;
    const uint32_t W = P.width, H = P.height, nw = P.words_per_row, t = P.threshold;

    // ---- task id in dispatch order (decoupled look-back needs resident predecessors)
    if (tid == 0) {
        const uint32_t task = atomicAdd(P.task_counter, 1u);
        if (task == P.ntasks - 1) atomicExch(P.task_counter, 0u);   // last ticket: reset
        sm.misc[2] = task;
    }
    __syncthreads();
    const uint32_t task = sm.misc[2];
    const uint32_t frame = task / P.bands_per_frame;
    const uint32_t band = task - frame * P.bands_per_frame;
    const uint32_t y0 = 3 + band * P.rows;                         // first centre row
    const uint32_t rows = min(P.rows, H - 3 - y0);                  // centre rows in band
    const uint8_t* img = P.frames + (uint64_t)frame * P.frame_stride;

    for (uint32_t i = tid; i < rows * nw; i += kThreads) sm.bitmap[i] = 0;

    // score rows s <-> image row y0 - 1 + s; the 1-row ring exists only for NMS
    const uint32_t s_lo = NMS == kNmsOff ? 1 : 0;
    const uint32_t s_hi = NMS == kNmsOff ? rows + 1 : rows + 2;
    const uint32_t tr_lo = NMS == kNmsOff ? 1 : 0;                  // tile rows to load
    const uint32_t tr_hi = NMS == kNmsOff ? rows + 7 : rows + 8;

    for (uint32_t X0 = 0; X0 < W - 3; X0 += kChunk) {
        __syncthreads();   // previous chunk's readers are done with the tile
        // ---- stage tile rows [tr_lo, tr_hi) x columns [X0-16, X0+kChunk+16) into LDS
        constexpr uint32_t kVecPerRow = kPitch / 16;
        const uint32_t nvec = (tr_hi - tr_lo) * kVecPerRow;
        for (uint32_t v = tid; v < nvec; v += kThreads) {
            const uint32_t tr = tr_lo + v / kVecPerRow;
            const uint32_t tv = v % kVecPerRow;
            const int y = (int)y0 - 4 + (int)tr;
            const int xc = (int)X0 - 16 + 16 * (int)tv;
            uint4 val = make_uint4(0, 0, 0, 0);
            if (y >= 0 && y < (int)H && xc < (int)W && xc + 16 > 0) {
                const uint8_t* src = img + (uint64_t)y * W + xc;
                if (xc >= 0 && xc + 16 <= (int)W && ((uintptr_t)src & 15) == 0) {
                    val = *reinterpret_cast<const uint4*>(src);
                } else {
                    uint8_t b[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const int x = xc + k;
                        b[k] = (x >= 0 && x < (int)W) ? src[k] : 0;
                    }
                    val = *reinterpret_cast<uint4*>(b);
                }
            }
            *reinterpret_cast<uint4*>(sm.tile + tr * kPitch + tv * 16) = val;
        }
        if (NMS != kNmsOff && tid == 0) sm.misc[0] = 0;
        __syncthreads();

        // ---- groups gi <-> image columns X0-4+4gi .. +3; only those touching the needed
        //      columns: centres [X0, X0+kChunk) within [3, W-3), plus for NMS the ring
        //      columns X0-1 and X0+kChunk, clamped to [2, W-3] (ring cells outside the
        //      centre domain are processed so that their score is written as 0)
        const int need_lo = NMS == kNmsOff ? max((int)X0, 3) : max((int)X0 - 1, 2);
        const int need_hi = NMS == kNmsOff ? min((int)X0 + kChunk - 1, (int)W - 4)
                                           : min((int)X0 + kChunk, (int)W - 3);
        const uint32_t g_lo = (uint32_t)(need_lo - ((int)X0 - 4)) >> 2;
        const uint32_t g_hi = ((uint32_t)(need_hi - ((int)X0 - 4)) >> 2) + 1;
        const uint32_t ng = g_hi - g_lo;
        const uint32_t nitems = (s_hi - s_lo) * ng;

        uint32_t* qi = sm.q_item + wave * kQueueCap;
        uint32_t* qc = sm.q_cand + wave * kQueueCap;
        uint32_t qcount = 0;
        // this lane's first item, then advance by kThreads items per round
        uint32_t item = wave * 64 + lane;
        uint32_t s = s_lo + item / ng;
        uint32_t gi = g_lo + item % ng;
        for (uint32_t base = wave * 64; base < nitems; base += kThreads) {
            uint32_t cand = 0;
            if (item < nitems) {
                const uint8_t* px = sm.tile + (s + 3) * kPitch + 12 + 4 * gi;
                cand = prefilter_group<N>(px, t);
                const int y = (int)y0 - 1 + (int)s;
                const int x0 = (int)X0 - 4 + 4 * (int)gi;
                if (y < 3 || y >= (int)H - 3) cand = 0;
                if (x0 < 3 || x0 + 4 > (int)W - 3) {
                    uint32_t vm = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (x0 + j >= 3 && x0 + j < (int)W - 3) vm |= 0xffu << (8 * j);
                    cand &= vm;
                }
                if constexpr (NMS != kNmsOff) {
                    *reinterpret_cast<uint2*>(sm.scores + s * kScorePitch + 4 * gi) =
                        make_uint2(0, 0);
                }
            }
            const bool has = cand != 0;
            const uint64_t bal = __ballot(has);
            if (has) {
                const uint32_t pos = qcount + lanes_below(bal);
                qi[pos] = (s << 12) | gi;
                qc[pos] = cand;
            }
            qcount += (uint32_t)__popcll(bal);
            while (qcount >= 16) {
                qcount -= 16;
                test_queued<NMS, N>(sm, qi + qcount, qc + qcount, 16, t, X0, rows, nw);
            }
            item += kThreads;
            gi += kThreads;
            while (gi >= g_hi) { gi -= ng; ++s; }
        }
        if (qcount > 0) test_queued<NMS, N>(sm, qi, qc, qcount, t, X0, rows, nw);

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
                    const uint16_t* sc = sm.scores + ss * kScorePitch + col;
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
    // block exclusive scan of `mine`
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
    const uint32_t excl_in_band = before + incl - mine;

    // ---- decoupled look-back over tasks (raster order): band's global offset.  Wave 0
    //      probes 64 predecessors per round (lane k reads task - 1 - k): the nearest
    //      inclusive prefix ends the walk; a window of aggregates is summed and skipped.
    if (wave == 0 && !(P.flags & kFlagNoLookback)) {
        unsigned long long* st = P.band_state;
        unsigned long long excl = 0;
        if (task == 0) {
            if (lane == 0)
                __hip_atomic_store(&st[0], lb_pack(P.epoch, 2, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&st[task], lb_pack(P.epoch, 1, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            int64_t top = (int64_t)task - 1;
            while (true) {
                const int64_t idx = top - (int64_t)lane;
                uint32_t flag = 2;                                   // before task 0: 0 incl.
                unsigned long long val = 0;
                if (idx >= 0) {
                    const unsigned long long wv = __hip_atomic_load(
                        &st[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    flag = (uint32_t)(wv >> 48) == P.epoch ? (uint32_t)(wv >> 46) & 3u : 0u;
                    val = wv & ((1ull << 46) - 1);
                }
                const uint64_t incl = __ballot(flag == 2);
                const uint64_t missing = __ballot(flag == 0);
                // lanes that matter: up to and including the nearest inclusive, else all 64
                const uint64_t upto = incl ? (incl & (~incl + 1)) * 2 - 1 : ~0ull;
                if (missing & upto) {                                // a predecessor not yet
                    __builtin_amdgcn_s_sleep(2);                     // published: re-probe
                    continue;
                }
                unsigned long long part = ((upto >> lane) & 1) ? val : 0ull;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d, 64);
                excl += part;
                if (incl) break;
                top -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&st[task], lb_pack(P.epoch, 2, excl + total),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            if (band == 0) P.frame_offsets[frame] = excl;
            if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = excl + total;
            sm.misc[1] = (uint32_t)excl;
            sm.misc[3] = (uint32_t)(excl >> 32);
        }
    } else if (tid == 0) {
        sm.misc[1] = 0;
        sm.misc[3] = 0;
    }
    __syncthreads();
    unsigned long long out_idx =
        (((unsigned long long)sm.misc[3] << 32) | sm.misc[1]) + excl_in_band;

    // ---- expand keep-bits into raster-ordered points
    if (P.flags & kFlagNoEmit) return;
    for (uint32_t w = w_lo; w < w_hi; ++w) {
        uint32_t bits = sm.bitmap[w];
        const uint32_t r = w / nw;
        const uint32_t xb = (w - r * nw) * 32;
        const uint32_t y = y0 + r;
        while (bits) {
            const uint32_t b = __builtin_ctz(bits);
            bits &= bits - 1;
            if (out_idx < P.cap) P.out[out_idx] = make_uint2(xb + b, y);
            ++out_idx;
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

hipError_t launch_band_kernel(const BandParams& p, uint32_t nms, uint32_t n,
                              hipStream_t stream) {
    BandKernelFn fn = pick(nms, n);
    if (!fn) return hipErrorInvalidValue;
    const LdsLayout L = make_layout(p.rows, p.words_per_row, nms != kNmsOff);
    if (L.total > kMaxLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fn, dim3(p.ntasks), dim3(kThreads), L.total, stream, p);
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
