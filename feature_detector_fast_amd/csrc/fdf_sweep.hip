// fdf_sweep.hip -- column-sweep FAST-9..16 kernel for MI355X (gfx950), the production path.
//
// Replaces detect<NONMAX>() (iwanders/feature_detector_fast src/fast_simd.rs:301-620) with
// determine_keypoint (:115-297) and the NMS score functions (:623-718, :722-749).
//
// One workgroup (4 waves) owns a band of R full-width centre rows of one frame.  The band is
// cut into units = (column strip) x (sub-band of rows); waves take units from an LDS counter
// and sweep them top to bottom:
//   * lane l owns LC columns (one LC-byte buffer load per row; LC = 16 without NMS, 8 with
//     NMS, whose score ring would otherwise cut the waves per CU); lanes 0 and 63 are halo
//     lanes that only feed their neighbours, so a strip covers 62 x LC centres;
//   * pixel rows stream through an 8-slot register ring: loads run 4 rows ahead, are never
//     guarded by a branch and are never copied, so the compiler's vmcnt bookkeeping keeps
//     them in flight;
//   * every pairwise comparison is made once and used by both of its pixels: the vertical
//     pair (I(y), I(y+3)) gives S-flags for row y and N-flags for row y+3, the horizontal
//     pair (I(x), I(x+3)) gives E-flags for x and W-flags for x+3 (a 3-byte shift, with the
//     neighbouring lane's bytes via DPP).  Comparisons are byte-SWAR v_lerp_u8 (exact per
//     byte, see fdf_common.h), so the cardinal pre-filter (src/fast_simd.rs:441-509) costs
//     2 lerps per pixel;
//   * candidate pixels go into a per-wave FIFO in LDS (one per lane per round).  Every
//     kSweepIssue rows, once 64 are queued, a batch is issued: each lane gathers its pixel's
//     7x7 neighbourhood with 7 row-window loads straight from the frame (the rows were just
//     streamed, so these hit L2).  The batch is evaluated kSweepIssue rows later -- by then
//     the row loads issued before it are due anyway, so waiting for it never drains the row
//     prefetch -- with the per-lane VALU segment test (fdf_common.h);
//   * NMS: scores go to a 16-row LDS score ring per wave, keypoints of owned pixels to a
//     list; whenever testing has caught up with more rows, the keypoints of the rows whose
//     neighbours are all scored pass the 3x3 strict-max test (:589-616) into the workgroup's
//     band bitmap.
// The band's keep-bits are then written to its output slot (its points in raster order, or
// the bitmap if they do not fit) and compact_kernel orders all slots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fdf_common.h"
#include "fdf_kernels.h"

namespace fdfk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// A lane's LC bytes of one pixel row (LC / 4 dwords).
template <int LC> struct LaneRow;
template <> struct LaneRow<16> { using type = u32x4; };
template <> struct LaneRow<8> { using type = u32x2; };

// DPP whole-wave shifts (GFX9 encodings): lane i reads lane i+1 / lane i-1; the lane that
// falls off the wave reads 0 (it is a halo lane whose results are never used).
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xf, 0xf, false);   // wave_shl:1
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xf, 0xf, false);   // wave_shr:1
}

struct RowSource {
    __amdgpu_buffer_rsrc_t rs;   // the frame; num_records = W * H + 15, or W * H when EXACT
    uint32_t W, H;
    int ylast;                   // last row the unit needs: later prefetches read nothing
    int tail_row;                // EXACT: rows >= tail_row may have windows crossing W * H
};

// Bytes [xb, xb+LC) of image row y: one LC-byte buffer load at any byte offset (gfx950
// buffer loads need no alignment).  No branch, so the row prefetch stays a plain stream the
// compiler's vmcnt bookkeeping can count.  Rows outside the frame and negative offsets read
// 0; columns outside [0, W) hold neighbouring bytes (the next row, or up to 15 bytes past
// the frame, which belong to the next frame of the batch or its stride gap) -- only halo
// lanes and non-centre pixels see them.  EXACT (the last frame of a batch, whose end may be
// the end of the caller's allocation): the rows whose windows can cross W * H are read byte
// by byte against num_records = W * H, so nothing past the frame is touched.
template <int LC, bool EXACT>
__device__ __forceinline__ typename LaneRow<LC>::type load_row(const RowSource& src, int y,
                                                              int xb) {
    using RowV = typename LaneRow<LC>::type;
    // y is wave-uniform, so the row test is scalar: a row outside [0, H) or past the unit's
    // last row gets an offset of 2^31 + xb, past any frame.  One VALU add per load; a
    // negative xb in row 0 wraps to >= 2^32 - LC, also out of range (reads 0).
    const bool in = y >= 0 && y < (int)src.H && y <= src.ylast;
    const uint32_t rowoff = in ? (uint32_t)(y * (int)src.W) : 0x80000000u;
    const int o = (int)(rowoff + (uint32_t)xb);
    if constexpr (EXACT) {
        if (y >= src.tail_row) {   // wave-uniform
            RowV r = (RowV)(0u);
#pragma unroll
            for (int k = 0; k < LC; ++k)
                r[k >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(src.rs, o + k, 0, 0)
                             << (8 * (k & 3));
            return r;
        }
    }
    if constexpr (LC == 16)
        return __builtin_bit_cast(RowV, __builtin_amdgcn_raw_buffer_load_b128(src.rs, o, 0, 0));
    else
        return __builtin_bit_cast(RowV, __builtin_amdgcn_raw_buffer_load_b64(src.rs, o, 0, 0));
}

struct SweepShared {
    uint32_t* pq;          // kSweepPixelQ FIFO of (row << 11) | (lane << 5) | flag bit
    void* ring;            // sweep_ring_rows x 64*LC scores (NMS), row y in slot y % rows
    uint32_t* kp;          // kSweepKpCap: (row << 10) | strip column
    uint32_t* bitmap;      // band keep-bits, R x words_per_row
};

struct UnitCtx {
    RowSource src;
    uint32_t t, nw;
    int S;                 // first owned centre column of the strip
    int r0, r1;            // owned centre rows of the unit
    int y0;                // first centre row of the band
    uint32_t lane;
    bool dense;            // NMS keypoint list overflowed: finalize densely
    uint32_t head, tail;   // candidate FIFO: entries [head, tail) at pq[i % kSweepPixelQ]
    uint32_t kpn;
    uint32_t flags;        // BandParams::flags (ablation runs only)
};

template <int LC, typename ScoreT>
__device__ __forceinline__ ScoreT* ring_at(const SweepShared& sh, int y, int cl) {
    constexpr int kRing = sweep_ring_rows(sizeof(ScoreT));   // score bytes 1 / 2 = nms 1 / 2
    return reinterpret_cast<ScoreT*>(sh.ring) + (y & (kRing - 1)) * (64 * LC) + cl;
}

// ---------------------------------------------------------------------------------------
// Full test of a batch of up to 64 queued pixels, one per lane, in two halves: issue pops
// the batch from the FIFO and starts its loads; evaluate tests the pixels (per-lane VALU
// segment test) and records keypoints / scores.
// ---------------------------------------------------------------------------------------
struct Batch {
    uint32_t code;         // (row << 10) | strip column
    bool act;
    uint32_t a0, a6;       // rows y-3, y+3: 4 bytes from x-1
    u32x2 a1, a5;          // rows y-2, y+2: 8 bytes from x-2
    u32x2 a2, a3, a4;      // rows y-1, y, y+1: 8 bytes from x-3
};

// Pops n (<= 64) entries.  n = 0 still issues the loads (all lanes at a harmless address):
// the pipelined issue points load unconditionally, so that every path through the sweep
// has the same sequence of loads and the compiler's vmcnt counts stay exact.
template <int LC>
__device__ __forceinline__ Batch issue_batch(const SweepShared& sh, UnitCtx& u, uint32_t n) {
    Batch b;
    b.act = u.lane < n;
    // FIFO entry (row << 11) | (lane << 5) | bit, bit 8j + m = lane column 4m + j  ->
    // the test's code (row << 10) | strip column
    const uint32_t e = b.act ? sh.pq[(u.head + u.lane) & (kSweepPixelQ - 1)] : 0u;
    const uint32_t bit = e & 31u;
    b.code = ((e >> 11) << 10) | (((e >> 5) & 63u) * LC + 4 * (bit & 7u) + (bit >> 3));
    u.head += n;
    const int W = (int)u.src.W;
    // inactive lanes read around centre (3, 3), which every tested frame has
    const int y = b.act ? (int)(b.code >> 10) : 3;
    const int x = b.act ? u.S - LC + (int)(b.code & 1023u) : 3;
    const int o = (y - 3) * W + x;                              // pixel (x, y - 3)
    // the windows stay inside the frame: rows y-3 .. y+3 are rows, and the 1-2 bytes past
    // a row end (rows y-1 .. y+2 only) belong to the next row
    b.a0 = __builtin_amdgcn_raw_buffer_load_b32(u.src.rs, o - 1, 0, 0);
    b.a1 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(u.src.rs, o - 2, W, 0));
    b.a2 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(u.src.rs, o - 3, 2 * W, 0));
    b.a3 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(u.src.rs, o - 3, 3 * W, 0));
    b.a4 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(u.src.rs, o - 3, 4 * W, 0));
    b.a5 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(u.src.rs, o - 2, 5 * W, 0));
    b.a6 = __builtin_amdgcn_raw_buffer_load_b32(u.src.rs, o - 1, 6 * W, 0);
    return b;
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// The ring packed 4 bytes per word (byte j of w[m] = circle pixel 4j + m) and the centre.
// Circle pixels by window byte: a0 = {15, 0, 1} at bytes 0-2; a1 = {14 @0, 2 @4};
// a2 = {13 @0, 3 @6}; a3 = {12 @0, c @3, 4 @6}; a4 = {11 @0, 5 @6}; a5 = {10 @0, 6 @4};
// a6 = {9, 8, 7} at bytes 0-2.  perm selector bytes: 0-3 = low source, 4-7 = high source,
// 0x0c = zero.
__device__ __forceinline__ void pack_ring(const Batch& b, uint32_t (&w)[4], uint32_t& c) {
    w[0] = perm(b.a3.y, b.a0, 0x0c0c0601u) | perm(b.a3.x, b.a6, 0x04010c0cu);   // 0 4 8 12
    w[1] = perm(b.a4.y, b.a0, 0x0c0c0602u) | perm(b.a2.x, b.a6, 0x04000c0cu);   // 1 5 9 13
    w[2] = perm(b.a1.y, b.a1.x, 0x000c0c04u) | perm(b.a5.y, b.a5.x, 0x0c00040cu); // 2 6 10 14
    w[3] = perm(b.a6, b.a2.y, 0x0c0c0602u) | perm(b.a0, b.a4.x, 0x04000c0cu);   // 3 7 11 15
    c = b.a3.x >> 24;
}

template <int NMS, int N, int LC, typename ScoreT>
__device__ __forceinline__ void evaluate_batch(const SweepShared& sh, UnitCtx& u,
                                               const LerpConsts& lk, const Batch& b) {
    const int y = (int)(b.code >> 10), cl = (int)(b.code & 1023u);
    const int x = u.S - LC + cl;
    uint32_t w[4], c;
    pack_ring(b, w, c);
    bool kb, kd;
    lane_segment_test_packed<N>(c, w, lk, kb, kd);
    const bool is_kp = b.act && (kb || kd);
    const bool owned = cl >= LC && cl < LC + strip_cols(LC) && y >= u.r0 && y < u.r1;
    if constexpr (NMS == kNmsOff) {
        if (is_kp && owned)
            atomicOr(&sh.bitmap[(y - u.y0) * u.nw + ((uint32_t)x >> 5)], 1u << (x & 31));
    } else {
        if (is_kp) {
            uint32_t p[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = (w[i & 3] >> (8 * (i >> 2))) & 0xffu;
            const uint32_t score = NMS == kNmsMaxThreshold ? score_max_threshold<N>(c, p, kd)
                                                           : score_sum_abs(c, p, u.t);
            *ring_at<LC, ScoreT>(sh, y, cl) = (ScoreT)score;
        }
        const bool add = is_kp && owned;
        const uint64_t bal = wave_ballot(add);
        if (add) {
            const uint32_t k = u.kpn + lanes_below(bal);
            if (k < kSweepKpCap) sh.kp[k] = b.code;
        }
        u.kpn += (uint32_t)__popcll(bal);
    }
}

// 3x3 strict maximum (src/fast_simd.rs:596-615).  All nine reads are issued before any
// compare (no short-circuit), so they cost one LDS round trip, not nine.
template <int LC, typename ScoreT>
__device__ __forceinline__ bool nms_keep_ring(const SweepShared& sh, int y, int cl) {
    const ScoreT* a = ring_at<LC, ScoreT>(sh, y - 1, cl);
    const ScoreT* m = ring_at<LC, ScoreT>(sh, y, cl);
    const ScoreT* b = ring_at<LC, ScoreT>(sh, y + 1, cl);
    const uint32_t v = m[0];
    const uint32_t n0 = a[-1], n1 = a[0], n2 = a[1], n3 = m[-1], n4 = m[1], n5 = b[-1],
                   n6 = b[0], n7 = b[1];
    const uint32_t mx = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
    return v > mx;
}

// NMS: keep-bits for the unit's keypoints in rows first .. ylim (all neighbours scored).
template <int LC, typename ScoreT>
__device__ __forceinline__ void sweep_finalize(const SweepShared& sh, UnitCtx& u, int first,
                                               int ylim) {
    const int H = (int)u.src.H;
    if (u.kpn > kSweepKpCap) u.dense = true;
    if (u.dense) {
        // rare: the list overflowed -- scan the owned columns of the rows densely
        const int lo = first > u.r0 ? first : u.r0;
        for (int y = lo; y <= ylim && y < u.r1; ++y) {
            if (y == 3 || y == H - 4) continue;
            if (u.lane < 1 || u.lane > 62) continue;
            for (int j = 0; j < LC; ++j) {
                const int cl = (int)u.lane * LC + j;
                const int x = u.S - LC + cl;
                if (x < 3 || x >= (int)u.src.W - 3) continue;
                if (*ring_at<LC, ScoreT>(sh, y, cl) != 0 && nms_keep_ring<LC, ScoreT>(sh, y, cl))
                    atomicOr(&sh.bitmap[(y - u.y0) * u.nw + ((uint32_t)x >> 5)], 1u << (x & 31));
            }
        }
        u.kpn = 0;
        return;
    }
    uint32_t kept = 0;
    for (uint32_t b0 = 0; b0 < u.kpn; b0 += 64) {
        const uint32_t i = b0 + u.lane;
        const bool act = i < u.kpn;
        const uint32_t e = act ? sh.kp[i] : 0u;
        const int y = (int)(e >> 10), cl = (int)(e & 1023u);
        const bool fin = act && y <= ylim;
        const bool carry = act && !fin;
        const uint64_t bal = wave_ballot(carry);
        if (carry) sh.kp[kept + lanes_below(bal)] = e;   // kept + idx <= i: read before write
        kept += (uint32_t)__popcll(bal);
        if (fin && y != 3 && y != H - 4 && nms_keep_ring<LC, ScoreT>(sh, y, cl)) {
            const int x = u.S - LC + cl;
            atomicOr(&sh.bitmap[(y - u.y0) * u.nw + ((uint32_t)x >> 5)], 1u << (x & 31));
        }
    }
    u.kpn = kept;
}

// Horizontal/vertical comparison flags of one lane row (bit 7 of each byte, LC pixels).
template <int LC>
struct RowFlags {
    typename LaneRow<LC>::type b, nd;
};

template <int LC>
__device__ __forceinline__ RowFlags<LC> compare_rows(const typename LaneRow<LC>::type& x,
                                                     const typename LaneRow<LC>::type& nc,
                                                     const LerpConsts& k) {
    RowFlags<LC> f;
#pragma unroll
    for (int m = 0; m < LC / 4; ++m) {
        f.b[m] = lerp_u8(lerp_u8(x[m], nc[m], k.rb), k.kb, 0);   // x - c > t
        f.nd[m] = lerp_u8(lerp_u8(x[m], nc[m], k.rd), k.kd, 0);  // NOT(x - c < -t)
    }
    return f;
}

// Test everything queued, now (FIFO overflow, a score-ring wrap, the end of a unit).
template <int NMS, int N, int LC, typename ScoreT>
__device__ __forceinline__ void flush_tests(const SweepShared& sh, UnitCtx& u,
                                            const LerpConsts& lk, bool& inflight,
                                            const Batch& batch) {
    if (inflight) {
        evaluate_batch<NMS, N, LC, ScoreT>(sh, u, lk, batch);
        inflight = false;
    }
    while (u.tail != u.head) {
        if (u.flags & kFlagNoFullTest) {
            u.head = u.tail;
            break;
        }
        const Batch b = issue_batch<LC>(sh, u, min(u.tail - u.head, 64u));
        evaluate_batch<NMS, N, LC, ScoreT>(sh, u, lk, b);
    }
}

// NMS: finalize the rows first_unfinal .. ylim (when there are any).
template <int LC, typename ScoreT>
__device__ __forceinline__ void finalize_upto(const SweepShared& sh, UnitCtx& u,
                                              int& first_unfinal, int ylim) {
    if (ylim >= first_unfinal) {
        sweep_finalize<LC, ScoreT>(sh, u, first_unfinal, ylim);
        first_unfinal = ylim + 1;
    }
}

template <int NMS, int N, bool EXACT>
__device__ __forceinline__ void sweep_unit(const SweepShared& sh, UnitCtx& u, const LerpConsts& lk) {
    using ScoreT = typename std::conditional<NMS == kNmsSumAbsolute, uint16_t, uint8_t>::type;
    constexpr int LC = lane_cols_for(NMS);
    constexpr int M = LC / 4;
    constexpr int kIssue = sweep_issue_every(NMS);
    // the oldest queued row may lag the sweep by this much before a partial batch is issued
    // (the ring keeps rows >= (oldest untested) - 2 up to the current row)
    constexpr int kLagLimit = NMS == kNmsOff ? 1 << 30
                                             : (sweep_ring_rows(NMS) - kIssue - 3 > 1
                                                    ? sweep_ring_rows(NMS) - kIssue - 3 : 1);
    using RowV = typename LaneRow<LC>::type;
    const uint32_t lane = u.lane;
    const int H = (int)u.src.H, W = (int)u.src.W;
    const int xb = u.S - LC + LC * (int)lane;
    // candidate columns of this lane: owned centres, plus for NMS the two border columns the
    // strip's edge keypoints compare against (scores only)
    // (bit 8j + m = lane column 4m + j, the order the candidate mask is built in)
    uint32_t vmask = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int x = xb + 4 * m + j;
            bool ok = x >= 3 && x < W - 3;
            if (lane == 0) ok = ok && NMS != kNmsOff && x == u.S - 1;
            if (lane == 63) ok = ok && NMS != kNmsOff && x == u.S + strip_cols(LC);
            if (ok) vmask |= 1u << (8 * j + m);
        }
    }
    const int ringr = NMS == kNmsOff ? 0 : 1;
    const int p0 = u.r0 - ringr, p1 = u.r1 + ringr;   // rows run through the pre-filter
    const int ys = p0 - 3;                             // first row of vertical comparisons
    const int T = p1 - ys;                             // sweep steps (row ys + i at step i)
    u.src.ylast = p1 + 2;                              // S-row of the last pre-filtered row
    u.head = u.tail = 0;
    u.kpn = 0;
    u.dense = false;
    int first_unfinal = u.r0;                          // NMS: rows before it are finalized
    bool inflight = false;
    Batch batch;

    // One 8-slot ring of pixel rows: row r in slot (r - ys) & 7.  At step J (row yv) it holds
    // rows yv .. yv+6 with yv+4 .. yv+6 still loading, and row yv+7 is loaded into the slot
    // of row yv-1, which is dead.  Nothing is copied, so every slot keeps its registers
    // across loop iterations and no wait is needed for a register move.
    RowV Rw[8];
#pragma unroll
    for (int k = 0; k < 7; ++k) Rw[k] = load_row<LC, EXACT>(u.src, ys + k, xb);
    RowFlags<LC> V[4];                                 // vertical flags, slot (row-ys) & 3

    // Step J: next row load, comparisons, pre-filter of row yv, enqueue of its candidates.
#define FDF_SWEEP_STEP(J)                                                                    \
    {                                                                                        \
        const int yv = ys + i0 + (J);                                                        \
        RowV cand = (RowV)(0u);                                                              \
        Rw[((J) + 7) & 7] = load_row<LC, EXACT>(u.src, yv + 7, xb);                          \
        const RowV s = Rw[((J) + 3) & 7];                  /* row yv + 3 */                  \
        const RowV c = Rw[(J) & 7];                        /* row yv */                      \
        const RowV nc = ~c;                                                                  \
        V[(J) & 3] = compare_rows<LC>(s, nc, lk);                                            \
        const bool live = yv >= p0 && yv < p1;                                               \
        if (live && yv >= 3 && yv < H - 3 && !(u.flags & kFlagNoLoad)) {                     \
            RowV e;                                                                          \
            _Pragma("unroll") for (int m = 0; m + 1 < M; ++m) e[m] = alignbyte(c[m + 1], c[m], 3); \
            e[M - 1] = alignbyte(from_next_lane(c[0]), c[M - 1], 3);                         \
            const RowFlags<LC> h = compare_rows<LC>(e, nc, lk);                              \
            const uint32_t pb = from_prev_lane(h.b[M - 1]), pnd = from_prev_lane(h.nd[M - 1]); \
            const RowFlags<LC>& vs = V[(J) & 3];                                             \
            const RowFlags<LC>& vn = V[((J) + 1) & 3];                                       \
            _Pragma("unroll") for (int m = 0; m < M; ++m) {                                  \
                const uint32_t hbw = alignbyte(h.b[m], m ? h.b[m - 1] : pb, 1);              \
                const uint32_t hndw = alignbyte(h.nd[m], m ? h.nd[m - 1] : pnd, 1);          \
                const uint32_t bn = ~vn.nd[m], bs = vs.b[m], be = h.b[m], bw = ~hndw;        \
                const uint32_t dn = ~vn.b[m], ds = vs.nd[m], de = h.nd[m], dw = ~hbw;        \
                uint32_t br, nd;                                                             \
                if constexpr (N < 12) {                                                      \
                    br = (bn | bs) & (be | bw);                                              \
                    nd = (dn & ds) | (de & dw);                                              \
                } else {                                                                     \
                    br = (bn & bs & (be | bw)) | (be & bw & (bn | bs));                      \
                    nd = (dn & ds) | (de & dw) | ((dn | ds) & (de | dw));                    \
                }                                                                            \
                cand[m] = br | ~nd;                                                          \
            }                                                                                \
        }                                                                                    \
        if constexpr (NMS != kNmsOff) {                                                      \
            if (live) {                                                                      \
                /* the ring slot of row yv still holds row yv - 16: if that row is still */  \
                /* needed as an NMS neighbour, catch testing and NMS up first */             \
                if (yv - sweep_ring_rows(NMS) >= first_unfinal - 1) {                        \
                    flush_tests<NMS, N, LC, ScoreT>(sh, u, lk, inflight, batch);             \
                    finalize_upto<LC, ScoreT>(sh, u, first_unfinal, yv - 2);                 \
                }                                                                            \
                RowV* rp = reinterpret_cast<RowV*>(ring_at<LC, ScoreT>(sh, yv, LC * (int)lane)); \
                _Pragma("unroll") for (int q = 0; q < (int)sizeof(ScoreT); ++q) rp[q] = (RowV)(0u); \
            }                                                                                \
        }                                                                                    \
        /* candidate pixels into the FIFO, one per lane per round: column 4m + j of the */   \
        /* lane is bit 8j + m of cm; the entry keeps the bit, issue_batch decodes it */      \
        const uint32_t code_base = ((uint32_t)yv << 11) | (lane << 5);                       \
        uint32_t cm = 0;                                                                     \
        _Pragma("unroll") for (int m = 0; m < M; ++m) cm |= (cand[m] >> (7 - m)) & (0x01010101u << m); \
        cm &= vmask;                                                                         \
        for (;;) {                                                                           \
            const bool has = cm != 0;                                                        \
            const uint64_t bal = wave_ballot(has);                                           \
            if (bal == 0) break;                                                             \
            if (has) {                                                                       \
                sh.pq[(u.tail + lanes_below(bal)) & (kSweepPixelQ - 1)] =                    \
                    code_base | (uint32_t)__builtin_ctz(cm);                                 \
                cm &= cm - 1;                                                                \
            }                                                                                \
            u.tail += (uint32_t)__popcll(bal);                                               \
            if (u.tail - u.head > kSweepPixelQ - 64) {                                       \
                /* dense image: test the oldest batch now, synchronously */                  \
                if (u.flags & kFlagNoFullTest) u.head += 64;                                 \
                else evaluate_batch<NMS, N, LC, ScoreT>(sh, u, lk, issue_batch<LC>(sh, u, 64u)); \
            }                                                                                \
        }                                                                                    \
        if (((J) % kIssue) == kIssue - 1) {                                                  \
            /* the batch issued kIssue rows ago is due; issue the next full one */           \
            if (inflight) {                                                                  \
                evaluate_batch<NMS, N, LC, ScoreT>(sh, u, lk, batch);                        \
                inflight = false;                                                            \
            }                                                                                \
            const uint32_t pend = u.tail - u.head;                                           \
            bool go = pend >= 64;                                                            \
            if constexpr (NMS != kNmsOff) {                                                  \
                /* a partial batch goes too once its oldest pixel would outrun the ring */   \
                if (!go && pend > 0)                                                         \
                    go = yv - (int)(sh.pq[u.head & (kSweepPixelQ - 1)] >> 11) >= kLagLimit;  \
            }                                                                                \
            if (go && (u.flags & kFlagNoFullTest)) u.head += min(pend, 64u);                 \
            const uint32_t n = (go && !(u.flags & kFlagNoFullTest)) ? min(pend, 64u) : 0u;   \
            batch = issue_batch<LC>(sh, u, n);                                               \
            inflight = n != 0;                                                               \
            if constexpr (NMS != kNmsOff) {                                                  \
                /* rows before the oldest untested candidate are fully tested */             \
                int r = yv + 1;                                                              \
                if (u.tail != u.head) r = (int)(sh.pq[u.head & (kSweepPixelQ - 1)] >> 11);   \
                if (inflight) r = min(r, (int)(__builtin_amdgcn_readfirstlane(batch.code) >> 10)); \
                finalize_upto<LC, ScoreT>(sh, u, first_unfinal, r - 2);                      \
            }                                                                                \
        }                                                                                    \
    }

    for (int i0 = 0; i0 < T; i0 += 8) {
        FDF_SWEEP_STEP(0)
        FDF_SWEEP_STEP(1)
        FDF_SWEEP_STEP(2)
        FDF_SWEEP_STEP(3)
        FDF_SWEEP_STEP(4)
        FDF_SWEEP_STEP(5)
        FDF_SWEEP_STEP(6)
        FDF_SWEEP_STEP(7)
    }
#undef FDF_SWEEP_STEP
    flush_tests<NMS, N, LC, ScoreT>(sh, u, lk, inflight, batch);
    if constexpr (NMS != kNmsOff) finalize_upto<LC, ScoreT>(sh, u, first_unfinal, p1 - 2);
}

// Occupancy target: 4 workgroups (16 waves) per CU, registers <= 128 VGPRs.
template <int NMS>
constexpr int sweep_waves_per_eu() { return 4; }

template <int NMS, int N>
__global__ __launch_bounds__(kThreads)
__attribute__((amdgpu_waves_per_eu(sweep_waves_per_eu<NMS>(), sweep_waves_per_eu<NMS>())))
void fast_sweep_kernel(BandParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    constexpr int LC = lane_cols_for(NMS);
    const SweepLayout L = make_sweep_layout(P.rows, P.words_per_row, score_bytes_for(NMS), LC);
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
    const uint32_t W = P.width, H = P.height, nw = P.words_per_row;

    // XCD-aware static task mapping: consecutive bands of a frame land on one XCD (its L2
    // then serves the halo rows two neighbouring bands share)
    const uint32_t b = blockIdx.x;
    const uint32_t q8 = P.ntasks >> 3, r8 = P.ntasks & 7, k8 = b & 7;
    const uint32_t task = k8 * q8 + min(k8, r8) + (b >> 3);
    const uint32_t frame = task / P.bands_per_frame;
    const uint32_t band = task - frame * P.bands_per_frame;
    const uint32_t y0 = 3 + band * P.rows;
    const uint32_t rows = min(P.rows, H - 3 - y0);

    uint32_t* bitmap = reinterpret_cast<uint32_t*>(smem_raw + L.bitmap);
    uint32_t* wave_sum = reinterpret_cast<uint32_t*>(smem_raw + L.bitmap + align16(P.rows * nw * 4));
    if (P.threshold >= 255) {                                        // no pixel can pass
        if (tid == 0) P.counts[task] = 0;
        return;
    }
    uint32_t* unit_ctr = wave_sum + kWaves;
    for (uint32_t i = tid; i < rows * nw; i += kThreads) bitmap[i] = 0;
    if (tid == 0) *unit_ctr = 0;
    __syncthreads();

    uint8_t* wbase = smem_raw + wave * L.wave_bytes;
    SweepShared sh;
    sh.pq = reinterpret_cast<uint32_t*>(wbase + L.pq);
    sh.ring = wbase + L.ring;
    sh.kp = reinterpret_cast<uint32_t*>(wbase + L.kp);
    sh.bitmap = bitmap;

    UnitCtx u;
    const uint8_t* img = P.frames + (uint64_t)frame * P.frame_stride;
    u.src.W = W;
    u.src.H = H;
    const bool last_frame = frame + 1 == P.ntasks / P.bands_per_frame;
    const __amdgpu_buffer_rsrc_t rs_pad = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(img), 0, (int)(W * H + 15), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_exact = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(img), 0, (int)(W * H), 0x00020000);
    u.t = P.threshold;
    u.nw = nw;
    u.y0 = (int)y0;
    u.lane = lane;
    u.flags = P.flags;
    const LerpConsts lk = lerp_consts(P.threshold);

    const uint32_t nunits = P.nstrips * P.nsub;
    const uint32_t sub_rows = (rows + P.nsub - 1) / P.nsub;
    // units are handed out dynamically: a wave that finishes early takes the next one
    // instead of idling at the workgroup barrier
    if (!(P.flags & kFlagNoPrefilter)) {
        for (;;) {
            uint32_t unit = 0;
            if (lane == 0) unit = atomicAdd(unit_ctr, 1u);
            unit = __builtin_amdgcn_readfirstlane(unit);
            if (unit >= nunits) break;
            const uint32_t strip = unit % P.nstrips, sub = unit / P.nstrips;
            u.S = (int)strip * strip_cols(LC);
            {   // first row whose last lane's window can end past W * H
                const int last_end = u.S - LC + LC * 64;
                const int num = (int)(W * H) - last_end;
                u.src.tail_row = num < 0 ? 0 : num / (int)W + 1;
            }
            u.r0 = (int)(y0 + sub * sub_rows);
            u.r1 = (int)min(y0 + (sub + 1) * sub_rows, y0 + rows);
            if (u.r0 >= u.r1) continue;
            // rows the sweep loads: up to r1 + ringr + 2
            const int ringr = NMS == kNmsOff ? 0 : 1;
            if (last_frame && u.r1 + ringr + 2 >= u.src.tail_row) {
                u.src.rs = rs_exact;
                sweep_unit<NMS, N, true>(sh, u, lk);
            } else {
                u.src.rs = rs_pad;
                sweep_unit<NMS, N, false>(sh, u, lk);
            }
        }
    }
    __syncthreads();

    // ---- count keep-bits and write the band slot
    const uint32_t nwords = rows * nw;
    const uint32_t per = (nwords + kThreads - 1) / kThreads;
    const uint32_t w_lo = min(tid * per, nwords), w_hi = min(w_lo + per, nwords);
    uint32_t mine = 0;
    for (uint32_t w = w_lo; w < w_hi; ++w) mine += __popc(bitmap[w]);
    uint32_t incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
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
    uint8_t* slot = P.slots + (uint64_t)task * P.slot_bytes;
    if (total <= P.slot_bytes / 8) {
        uint2* pts = reinterpret_cast<uint2*>(slot);
        uint32_t idx = before + incl - mine;
        for (uint32_t w = w_lo; w < w_hi; ++w) {
            uint32_t bits = bitmap[w];
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
        for (uint32_t w = tid; w < nwords; w += kThreads) words[w] = bitmap[w];
    }
}

typedef void (*SweepKernelFn)(BandParams);

template <int NMS>
static SweepKernelFn pick_sweep_n(uint32_t n) {
    switch (n) {
        case 9: return fast_sweep_kernel<NMS, 9>;
        case 10: return fast_sweep_kernel<NMS, 10>;
        case 11: return fast_sweep_kernel<NMS, 11>;
        case 12: return fast_sweep_kernel<NMS, 12>;
        case 13: return fast_sweep_kernel<NMS, 13>;
        case 14: return fast_sweep_kernel<NMS, 14>;
        case 15: return fast_sweep_kernel<NMS, 15>;
        case 16: return fast_sweep_kernel<NMS, 16>;
        default: return nullptr;
    }
}

hipError_t launch_sweep(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream) {
    SweepKernelFn fn = nullptr;
    switch (nms) {
        case kNmsOff: fn = pick_sweep_n<kNmsOff>(n); break;
        case kNmsMaxThreshold: fn = pick_sweep_n<kNmsMaxThreshold>(n); break;
        case kNmsSumAbsolute: fn = pick_sweep_n<kNmsSumAbsolute>(n); break;
        default: break;
    }
    if (!fn) return hipErrorInvalidValue;
    const SweepLayout L = make_sweep_layout(p.rows, p.words_per_row, score_bytes_for(nms),
                                            lane_cols_for(nms));
    if (L.total > kSweepMaxLds) return hipErrorInvalidValue;
    if (L.total > kMaxLds) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)L.total);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(p.ntasks), dim3(kThreads), L.total, stream, p);
    return hipGetLastError();
}

}  // namespace fdfk
