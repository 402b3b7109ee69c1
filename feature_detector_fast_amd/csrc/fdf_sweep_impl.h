// fdf_sweep_impl.h -- column-sweep FAST-9..16 kernel for MI355X (gfx950), the production path.
// Included by fdf_sweep.hip (grey frames: FDF_SWEEP_RGB 0, namespace fdfk::grey),
// fdf_sweep_latency.hip (grey frames, units leave their last 8-step block early: namespace
// fdfk::grey_lat) and fdf_sweep_rgb.hip (RGB8 frames converted to luma in the row and window
// loads: FDF_SWEEP_RGB 1, namespace fdfk::rgb); each translation unit instantiates its 24
// kernels.
//
// Replaces detect<NONMAX>() (iwanders/feature_detector_fast src/fast_simd.rs:301-620) with
// determine_keypoint (:115-297) and the NMS score functions (:623-718, :722-749).
//
// One workgroup (4 waves) owns a band of R full-width centre rows of one frame.  The band is
// cut into units = (column strip) x (sub-band of rows); waves take units from an LDS counter
// and sweep them top to bottom:
//   * lane l owns 16 columns (one 16-byte buffer load per row); lanes 0 and 63 are halo
//     lanes that only feed their neighbours, so a strip covers 62 x 16 centres;
//   * pixel rows stream through a register ring of kRing slots: kRing - 4 row loads
//     are in flight, none is guarded by a branch and none is copied, so the compiler's vmcnt
//     bookkeeping keeps them in flight;
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
//     prefetch -- with the per-lane VALU segment test (fdf_common.h).  Keypoints set their
//     bit in the band's LDS bitmap; with NMS their score goes to the frame's score map.
// NMS (src/fast_simd.rs:589-616) runs once the whole band is tested: the band also tests one
// row above and below it, so every neighbour of its keypoints is in the bitmap, and each
// keypoint is compared with the scores of the neighbours the bitmap marks.  The band's
// keep-bits are then written to its output slot (its points in raster order, or the bitmap
// if they do not fit) and compact_kernel orders all slots.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fdf_common.h"
#include "fdf_kernels.h"

#ifndef FDF_SWEEP_NS
#error "define FDF_SWEEP_RGB and FDF_SWEEP_NS before including fdf_sweep_impl.h"
#endif

namespace fdfk {
namespace FDF_SWEEP_NS {

// RGB8 input: 3 bytes per pixel, converted to luma as image 0.24.6 to_luma8 on load
constexpr bool kRgb = FDF_SWEEP_RGB != 0;
// The row ring and the occupancy target of this translation unit's kernels (kSweepRing /
// kSweepWavesPerEU: 8 slots, 4 waves per SIMD, unless the unit overrides them).  A 16-slot
// ring at 2 waves per SIMD for frames read in place over PCIe was measured slower (DESIGN.md
// §7.5: PCIe read throughput, not latency, bounds that kernel).
#ifndef FDF_SWEEP_TU_RING
#define FDF_SWEEP_TU_RING kSweepRing
#endif
#ifndef FDF_SWEEP_TU_WAVES
#define FDF_SWEEP_TU_WAVES kSweepWavesPerEU
#endif
constexpr int kRing = FDF_SWEEP_TU_RING;
constexpr int kWavesEU = FDF_SWEEP_TU_WAVES;
// Units that end inside an 8-step block leave it at their last row (FDF_SWEEP_TU_EXIT, the
// latency instances of fdf_sweep_latency.hip: a single frame's 3-row units skip 4 padding
// steps).  The exit tests perturb the long-unit loop's code (512 x 1080p max-t +0.5..+2 %,
// DESIGN.md §7.6), so the throughput instances keep whole blocks.
#ifndef FDF_SWEEP_TU_EXIT
#define FDF_SWEEP_TU_EXIT 0
#endif
constexpr bool kExitInBlock = FDF_SWEEP_TU_EXIT != 0;
constexpr int kPx = kRgb ? 3 : 1;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

// A lane's LC bytes of one pixel row (LC / 4 dwords).
template <int LC> struct LaneRow;
template <> struct LaneRow<16> { using type = u32x4; };
template <> struct LaneRow<8> { using type = u32x2; };

// DPP whole-wave shifts (GFX9 encodings): lane i reads lane i+1 / lane i-1.  The lane that
// falls off the wave (63 / 0) is a halo lane whose results are never used, so its value is
// left undefined: no `old` operand to initialise (one v_mov per shift, 3 a sweep step).
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, false);   // wave_shl:1
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, false);   // wave_shr:1
}

struct RowSource {
    __amdgpu_buffer_rsrc_t rs;   // the frame; num_records = W * H + 15, or W * H when EXACT
    __amdgpu_buffer_rsrc_t none; // num_records = 0: every load reads 0 (rows off the frame)
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
// Luma of the RGB pixel in bytes 0-2 of v (byte 3 ignored), exactly image 0.24.6's to_luma8:
// (2126 r + 7152 g + 722 b) / 10000.  The weights split as 256 hi + lo with byte-sized hi
// = (8, 27, 2) and lo = (78, 240, 210) for two v_dot4_u32_u8; x < 2^22, so x / 10000 =
// (x * 13743896) >> 37 exactly ((13743896 * 10000 - 2^37) * 2^22 < 2^37), the high half from
// one v_mul_hi_u32_u24.
__device__ __forceinline__ uint32_t luma_of(uint32_t v) {
    const uint32_t x = (__builtin_amdgcn_udot4(v, 0x00021B08u, 0u, false) << 8) +
                       __builtin_amdgcn_udot4(v, 0x00D2F04Eu, 0u, false);
    return (uint32_t)(((uint64_t)(x & 0xffffffu) * 13743896ull) >> 32) >> 5;
}

// 16 RGB pixels (48 bytes, d[0..11]) -> their 16 luma bytes.  Pixels 4m .. 4m+3 are exactly
// dwords 3m .. 3m+2.
__device__ __forceinline__ u32x4 luma16(const uint32_t (&d)[12]) {
    u32x4 r;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint32_t p0 = d[3 * m], p1 = alignbyte(d[3 * m + 1], d[3 * m], 3);
        const uint32_t p2 = alignbyte(d[3 * m + 2], d[3 * m + 1], 2), p3 = d[3 * m + 2] >> 8;
        r[m] = luma_of(p0) | (luma_of(p1) << 8) | (luma_of(p2) << 16) | (luma_of(p3) << 24);
    }
    return r;
}

template <int LC, bool EXACT>
__device__ __forceinline__ typename LaneRow<LC>::type load_row(const RowSource& src, int y,
                                                              int xb) {
    using RowV = typename LaneRow<LC>::type;
    // y is wave-uniform, so the row test is scalar: a row outside [0, H) or past the unit's
    // last row gets an offset of 2^31 + xb, past any frame.  One VALU add per load; a
    // negative xb in row 0 wraps to >= 2^32 - LC, also out of range (reads 0).  RGB frames:
    // the same in bytes (3 per pixel).
    const bool in = y >= 0 && y < (int)src.H && y <= src.ylast;
    const uint32_t rowoff = in ? (uint32_t)(y * (int)src.W * kPx) : 0x80000000u;
    const int o = (int)(rowoff + (uint32_t)(xb * kPx));
    if constexpr (kRgb) {
        static_assert(LC == 16, "RGB rows are loaded 16 pixels at a time");
        uint32_t d[12];
        if (EXACT && y >= src.tail_row) {   // wave-uniform
#pragma unroll
            for (int k = 0; k < 12; ++k) d[k] = 0u;
#pragma unroll
            for (int k = 0; k < 48; ++k)
                d[k >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(src.rs, o + k, 0, 0)
                             << (8 * (k & 3));
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(src.rs, o + 16 * k, 0, 0));
                d[4 * k] = v[0]; d[4 * k + 1] = v[1]; d[4 * k + 2] = v[2]; d[4 * k + 3] = v[3];
            }
        }
        return luma16(d);
    }
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
    if constexpr (LC == 16) {
        // the row offset as the load's scalar offset and the lane's column as its vector
        // offset (no per-lane add); a row off the frame takes the empty resource instead
        (void)o;
        return __builtin_bit_cast(RowV, __builtin_amdgcn_raw_buffer_load_b128(
            in ? src.rs : src.none, xb, in ? y * (int)src.W : 0, 0));
    }
    else
        return __builtin_bit_cast(RowV, __builtin_amdgcn_raw_buffer_load_b64(src.rs, o, 0, 0));
}

// FIFO entries keep a lane row's 16 candidate flags and its code (row - ys) << 6 | lane in
// alternate nibbles: flag of lane column 4m + j at bit 8j + 4 + m, code nibble k at bits
// 8k .. 8k+3 -- the sweep step builds the flags in that order from the compare bytes with
// three bit-field inserts, and ORs in the code, instead of packing both into 16-bit halves.
constexpr uint32_t kFlagNibbles = 0xF0F0F0F0u;
__host__ __device__ constexpr uint32_t spread_code(uint32_t v) {   // 16 bits -> low nibbles
    return (v & 0xFu) | ((v & 0xF0u) << 4) | ((v & 0xF00u) << 8) | ((v & 0xF000u) << 12);
}
// The low nibbles (or high nibbles, shifted down first) of x packed into 16 bits.
__device__ __forceinline__ uint32_t pack_nibbles(uint32_t x) {
    const uint32_t c = x | (x >> 4);                   // byte 0: nibbles 0, 1; byte 2: 2, 3
    return __builtin_amdgcn_perm(c, c, 0x0c0c0200u);
}

struct SweepShared {
    uint32_t* pq;          // kSweepPixelQ FIFO of lane rows with candidates (kFlagNibbles:
                           // flags; low nibbles: spread_code((row - ys) << 6 | lane))
    uint32_t* stage;       // 64 pixels of the batch being issued: (row - ys) << 10 | strip column
    uint32_t* bitmap;      // band keypoints: bitmap row i = image row yb + i, words_per_row each
    uint32_t* slist;       // NMS: the band's keypoints as (bitmap row * W + x) << 12 | score
    uint32_t* slist_n;     // entries appended (the list, then the spill, then only counted)
    uint32_t slist_cap;    // kScoreListCap, or 0 when a position does not fit 20 bits
    uint32_t* spill;       // NMS: entries past slist_cap, in the band's output slot (global)
    const uint32_t* seltab;  // select_bit's table (SweepLayout::seltab)
    uint32_t spill_cap;    // slot words (0 with slist_cap 0)
};

struct UnitCtx {
    RowSource src;
    uint32_t t, nw;
    int S;                 // first owned centre column of the strip
    int p0, p1;            // tested centre rows of the unit (owned rows plus NMS halo rows)
    int yb;                // image row of bitmap row 0 (band start minus the NMS halo)
    uint32_t lane;
    uint32_t head, tail;   // candidate FIFO: entries [head, tail) at pq[i % kSweepPixelQ]
    int ys;                // first row the unit sweeps (FIFO rows are relative to it)
    int rowbase;           // (ys - 3) * W: frame offset of the window row y - 3 for FIFO row 0
    uint32_t flags;        // BandParams::flags (ablation runs only)
    // max-t keypoint queue (one entry per lane, kq_n < 64 entries, wave-uniform): the packed
    // ring and pos << 12 | dark << 8 | centre of keypoints whose score is not computed yet
    uint32_t kq_w[4], kq_c, kq_n;
};

// ---------------------------------------------------------------------------------------
// Full test of a batch of up to 64 queued pixels, one per lane, in two halves: issue pops
// the batch from the FIFO and starts its loads; evaluate tests the pixels (per-lane VALU
// segment test) and records keypoints / scores.
// ---------------------------------------------------------------------------------------
struct Batch {
    uint32_t code;         // (row << 10) | strip column
    uint32_t n;            // pixels in the batch (wave-uniform)
    bool act;
    uint32_t a0, a6;       // rows y-3, y+3: 4 bytes from x-1
    u32x2 a1, a5;          // rows y-2, y+2: 8 bytes from x-2
    u32x2 a2, a3, a4;      // rows y-1, y, y+1: 8 bytes from x-3
};

// The 7 row windows around centre (x, y) with o = (y - 3) * W + x.  They stay inside the
// frame: rows y-3 .. y+3 are rows, and the 1-2 bytes past a row end (rows y-1 .. y+2 only)
// belong to the next row.
__device__ __forceinline__ void load_ring_windows(Batch& b, const __amdgpu_buffer_rsrc_t& rs,
                                                  int o, int W) {
    if constexpr (kRgb) {
        // only the 17 window bytes pack_ring reads, each converted from its RGB pixel (one
        // 12-byte load for three adjacent pixels, a 4-byte load for a single one)
        auto px = [&](int p) {      // luma of pixel p (4 bytes from 3p; byte 3 unused)
            return luma_of(__builtin_amdgcn_raw_buffer_load_b32(rs, 3 * p, 0, 0));
        };
        auto px3 = [&](int p) {     // luma of pixels p, p+1, p+2 in bytes 0-2
            const u32x3 v = __builtin_bit_cast(u32x3, __builtin_amdgcn_raw_buffer_load_b96(rs, 3 * p, 0, 0));
            return luma_of(v[0]) | (luma_of(alignbyte(v[1], v[0], 3)) << 8) |
                   (luma_of(alignbyte(v[2], v[1], 2)) << 16);
        };
        b.a0 = px3(o - 1);
        b.a1.x = px(o - 2 + W);
        b.a1.y = px(o + 2 + W);
        b.a2.x = px(o - 3 + 2 * W);
        b.a2.y = px(o + 3 + 2 * W) << 16;
        b.a3.x = px(o - 3 + 3 * W) | (px(o + 3 * W) << 24);
        b.a3.y = px(o + 3 + 3 * W) << 16;
        b.a4.x = px(o - 3 + 4 * W);
        b.a4.y = px(o + 3 + 4 * W) << 16;
        b.a5.x = px(o - 2 + 5 * W);
        b.a5.y = px(o + 2 + 5 * W);
        b.a6 = px3(o - 1 + 6 * W);
        return;
    }
    b.a0 = __builtin_amdgcn_raw_buffer_load_b32(rs, o - 1, 0, 0);
    b.a1 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o - 2, W, 0));
    b.a2 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o - 3, 2 * W, 0));
    b.a3 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o - 3, 3 * W, 0));
    b.a4 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o - 3, 4 * W, 0));
    b.a5 = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o - 2, 5 * W, 0));
    b.a6 = __builtin_amdgcn_raw_buffer_load_b32(rs, o - 1, 6 * W, 0);
}

// Inclusive prefix sum over the wave's 64 lanes (DPP row shifts, then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

// Maximum over the wave's 64 lanes, in every lane (DPP row shifts, row broadcasts, then lane
// 63's value read back).
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

// Position of the j-th (from 0) set bit of a 16-bit mask that has more than j set bits.
// seltab[b] holds the positions of byte b's set bits, the k-th in nibble k (built per
// workgroup before its sweep), so the mask needs one byte choice and one LDS read instead
// of four halving steps.
__device__ __forceinline__ uint32_t select_bit(uint32_t m, uint32_t j, const uint32_t* seltab) {
    const uint32_t c8 = (uint32_t)__popc(m & 0xffu);
    const bool hi = j >= c8;
    const uint32_t byte = hi ? m >> 8 : m & 0xffu;
    const uint32_t jj = hi ? j - c8 : j;
    return ((seltab[byte] >> (4u * jj)) & 7u) | (hi ? 8u : 0u);
}

// Pops the next 64 candidate pixels (fewer only when `force`: a flush) and starts their
// loads.  The FIFO holds lane rows; the pixels of the first 64 entries are counted with a
// wave prefix sum, every contributing entry writes its pixels to the staging array in
// order, and an entry only partly taken keeps its other pixels at the FIFO head.  Without
// a batch the loads are still issued (all lanes at a harmless address): the pipelined issue
// points load unconditionally, so that every path through the sweep has the same sequence
// of loads and the compiler's vmcnt counts stay exact.
// The FIFO entries a batch is built from (read when the batch is built: a read earlier in
// the step goes stale when the step's overflow path takes entries).
struct FifoPeek {
    uint32_t nent;         // entries read (wave-uniform)
    uint32_t e;            // this lane's entry (0 past nent)
};
__device__ __forceinline__ FifoPeek fifo_peek(const SweepShared& sh, const UnitCtx& u) {
    FifoPeek f;
    f.nent = min(u.tail - u.head, 64u);
    f.e = u.lane < f.nent ? sh.pq[(u.head + u.lane) & (kSweepPixelQ - 1)] : 0u;
    return f;
}

template <int LC>
__device__ __forceinline__ Batch issue_batch(const SweepShared& sh, UnitCtx& u, bool force,
                                             const FifoPeek& pk) {
    static_assert(LC == 16, "16-bit lane masks");
    Batch b;
    b.n = 0;
    b.act = false;
    b.code = 0;
    const int W = (int)u.src.W;
    int o = 3;                                        // pixel (x, y - 3) of centre (3, 3)
    const uint32_t nent = pk.nent;
    if (nent != 0) {
        const uint32_t lane = u.lane;
        const bool has = lane < nent;
        const uint32_t e = pk.e;
        uint32_t m = e & kFlagNibbles;
        const uint32_t k = (uint32_t)__popc(m);
        const uint32_t inc = wave_incl_scan(k);
        const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
        if (total >= 64u || (force && total != 0u)) {
            b.n = min(total, 64u);
            const uint32_t excl = inc - k;
            uint32_t scode = 0;
            // no per-pixel loop: entry lane e marks the slot its pixels start at, a ballot of
            // the marks gives every batch lane its entry (the marks at or below it, less
            // entry 0's, which always starts at slot 0), and the lane selects its bit of that
            // entry's mask
            sh.stage[lane] = 0u;
            if (has && k != 0u && excl < 64u) sh.stage[excl] = 1u;
            // other lanes' stores feed this load: without the (instruction-free) wavefront
            // fence the compiler forwards the lane's own zero store (per-thread semantics)
            // and loads only where it stored
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint64_t starts = wave_ballot(sh.stage[lane] != 0u);
            const uint32_t src = lanes_below(starts >> 1);
            const uint32_t se = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)e);
            const uint32_t sx = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)excl);
            // the entry's flags as 16 bits: bit 4j + m = lane column 4m + j
            const uint32_t bit = select_bit(pack_nibbles((se >> 4) & ~kFlagNibbles), lane - sx, sh.seltab);
            // stage code as the loop writes it: (row - ys) << 10 | lane << 4 | column,
            // kept in the lane (no LDS round trip: the lane reads only its own pixel)
            scode = (pack_nibbles(se & ~kFlagNibbles) << 4) | ((bit & 3u) << 2) | (bit >> 2);
            // the partial entry keeps the flags past the ones taken: batch lane 63 took its
            // last one (an entry is partial only when the batch is full), so one readlane
            // replaces a second select; flag 4j + m sits at entry bit 8j + 4 + m
            if (has && excl < 64u && inc > 64u) {
                const uint32_t b63 = __builtin_amdgcn_readlane(bit, 63);
                m &= ~0u << (8u * (b63 >> 2) + 5u + (b63 & 3u));
            }
            // entries [0, nfull) are taken whole; entry nfull keeps what is left of it
            const uint32_t nfull = (uint32_t)__popcll(wave_ballot(has && inc <= 64u));
            if (has && excl < 64u && inc > 64u)
                sh.pq[(u.head + lane) & (kSweepPixelQ - 1)] = (e & ~kFlagNibbles) | m;
            u.head += nfull;
            b.act = lane < b.n;
            if (b.act) {
                const uint32_t sc = scode;
                b.code = ((uint32_t)(u.ys + (int)(sc >> 10)) << 10) | (sc & 1023u);
                // rows relative to the unit (< 2^10) times W (< 2^16): a 24-bit multiply
                o = u.rowbase + (int)__umul24(sc >> 10, (uint32_t)W) + u.S - LC + (int)(sc & 1023u);
            }
        }
    }
    load_ring_windows(b, u.src.rs, o, W);
    return b;
}

template <int LC>
__device__ __forceinline__ Batch issue_batch(const SweepShared& sh, UnitCtx& u, bool force) {
    return issue_batch<LC>(sh, u, force, fifo_peek(sh, u));
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

// Appends one score-list entry per active lane: the band's LDS list, past its capacity the
// band's slot (global), past that only counted.
__device__ __forceinline__ void append_scores(const SweepShared& sh, const UnitCtx& u, bool act,
                                              uint64_t bal, uint32_t e) {
    uint32_t base = 0;
    if (u.lane == 0) base = atomicAdd(sh.slist_n, (uint32_t)__popcll(bal));
    base = __builtin_amdgcn_readfirstlane(base);
    if (act) {
        const uint32_t idx = base + lanes_below(bal);
        if (idx < sh.slist_cap) sh.slist[idx] = e;
        else if (idx - sh.slist_cap < sh.spill_cap) sh.spill[idx - sh.slist_cap] = e;
    }
}

// Scores the first n entries of the max-t keypoint queue (one per lane) and lists them.
template <int N>
__device__ __forceinline__ void score_kp_queue(const SweepShared& sh, UnitCtx& u, uint32_t n) {
    const bool act = u.lane < n;
    // dark keypoints score as bright ones on 255 - p: the packed words are inverted before
    // they are unpacked (4 XORs instead of 16)
    const uint32_t inv = (u.kq_c & 0x100u) ? ~0u : 0u;
    const uint32_t c = (u.kq_c ^ inv) & 0xffu;
    uint32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = ((u.kq_w[i & 3] ^ inv) >> (8 * (i >> 2))) & 0xffu;
    const uint32_t score = score_max_threshold<N>(c, p, false);
    append_scores(sh, u, act, n >= 64 ? ~0ull : (1ull << n) - 1ull,
                  (u.kq_c & 0xfffff000u) | score);
}

template <int NMS, int N, int LC>
__device__ __forceinline__ void evaluate_batch(const SweepShared& sh, UnitCtx& u,
                                               const LerpConsts& lk, const Batch& b) {
    if (ablation_flags(u.flags) & kFlagNoEval) {   // ablation: consume the loads, test nothing
        if (b.act && (b.a0 ^ b.a1.x ^ b.a2.x ^ b.a3.x ^ b.a4.x ^ b.a5.x ^ b.a6) == 0x5a5a5a5au)
            u.flags |= kFlagNoEval;
        return;
    }
    const int y = (int)(b.code >> 10), cl = (int)(b.code & 1023u);
    const int x = u.S - LC + cl;
    uint32_t w[4], c;
    pack_ring(b, w, c);
    bool kb, kd;
    lane_segment_test_packed<N>(c, w, lk, kb, kd);
    // every queued pixel is a centre of the unit's strip and tested rows (vmask, p0 .. p1)
    const bool is_kp = b.act && (kb || kd);
    if (is_kp) atomicOr(&sh.bitmap[__umul24((uint32_t)(y - u.yb), u.nw) + ((uint32_t)x >> 5)], 1u << (x & 31));
    if constexpr (NMS == kNmsMaxThreshold) {
        // ~28% of a batch's lanes are keypoints (S1), and the max-t score is ~100 VALU on
        // every lane: keypoints move into the wave's queue (lane q + rank, via the staging
        // array -- free between a batch's issue and the next -- and ds_bpermute), and a full
        // queue of 64 is scored at once.  Keypoints past the 64th wrap to lanes 0.. of the
        // next queue; the same permuted values serve both.
        const uint64_t bal = wave_ballot(is_kp);
        if (bal) {
            const uint32_t k = (uint32_t)__popcll(bal);
            const uint32_t q = u.kq_n;
            if (is_kp) sh.stage[(q + lanes_below(bal)) & 63u] = u.lane;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // see issue_batch
            const int src = (int)(sh.stage[u.lane] << 2);
            // list position (bitmap row * W + x) with a full-rate 24-bit multiply
            const uint32_t pk = ((mul_u24_s(u.src.W, (uint32_t)(y - u.yb) & 0x3ffu) + (uint32_t)x) << 12) |
                                (kd ? 0x100u : 0u) | c;
            uint32_t nwv[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) nwv[m] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)w[m]);
            const uint32_t npk = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pk);
            if (u.lane >= q && u.lane < q + k) {
#pragma unroll
                for (int m = 0; m < 4; ++m) u.kq_w[m] = nwv[m];
                u.kq_c = npk;
            }
            if (q + k >= 64u) {
                score_kp_queue<N>(sh, u, 64u);
                if (u.lane + 64u < q + k) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) u.kq_w[m] = nwv[m];
                    u.kq_c = npk;
                }
            }
            u.kq_n = (q + k) & 63u;
        }
        return;
    }
    if constexpr (NMS == kNmsSumAbsolute) {
        // scores go to the band's LDS list, past its capacity to the band's slot (global),
        // past that they are only counted (the band NMS pass then recomputes all scores)
        const uint64_t bal = wave_ballot(is_kp);
        if (bal) {
            uint32_t base = 0;
            if (u.lane == 0) base = atomicAdd(sh.slist_n, (uint32_t)__popcll(bal));
            base = __builtin_amdgcn_readfirstlane(base);
            if (is_kp) {
                const uint32_t score = score_sum_abs_packed(c, w, u.t);
                const uint32_t idx = base + lanes_below(bal);
                const uint32_t e = ((mul_u24_s(u.src.W, (uint32_t)(y - u.yb) & 0x3ffu) + (uint32_t)x) << 12) | score;
                if (idx < sh.slist_cap) sh.slist[idx] = e;
                else if (idx - sh.slist_cap < sh.spill_cap) sh.spill[idx - sh.slist_cap] = e;
            }
        }
    }
}

// Horizontal/vertical comparison flags of one lane row (bit 7 of each byte, LC pixels).
template <int LC>
struct RowFlags {
    typename LaneRow<LC>::type b, nd;
};

// Pre-filter comparisons of one lane row (bit 7 of each byte), exact (fdf_common.h).
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

// Test everything queued, now (FIFO overflow, the end of a unit).
template <int NMS, int N, int LC>
__device__ __forceinline__ void flush_tests(const SweepShared& sh, UnitCtx& u,
                                            const LerpConsts& lk, bool (&inflight)[kSweepBatchSlots],
                                            Batch (&batch)[kSweepBatchSlots]) {
    constexpr int QL = kSweepBatchSlots - 1;
#pragma unroll
    for (int q = 0; q < QL; ++q) {
        if (inflight[q]) {
            evaluate_batch<NMS, N, LC>(sh, u, lk, batch[q]);
            inflight[q] = false;
        }
    }
    if (ablation_flags(u.flags) & kFlagNoFullTest) u.head = u.tail;
    // max-t measured 0.6-1.0% slower with the pipelined flush (its keypoint queue and score
    // keep more registers live), NMS off and SAD 0.2-1.5% faster (profiles/r02/ab_flush_rowdiv.txt)
    constexpr bool serial = NMS == kNmsMaxThreshold;
    if constexpr (serial) {
        if (inflight[QL]) evaluate_batch<NMS, N, LC>(sh, u, lk, batch[QL]);
        inflight[QL] = false;
        while (u.tail != u.head) {
            const Batch b = issue_batch<LC>(sh, u, true);
            evaluate_batch<NMS, N, LC>(sh, u, lk, b);
        }
        return;
    }
    // Pipelined: the next batch's gathers are issued before the one in flight is evaluated,
    // so a unit end with several queued batches waits for about one gather latency instead
    // of one per batch (the order keypoints are found in does not matter: bitmap bits, and
    // list entries ranked by position later).  Two batches alternate in fixed registers
    // (A = the last slot, B), so no register with a load pending is ever copied.
    Batch& A = batch[QL];
    bool pa = inflight[QL];
    while (u.tail != u.head) {
        const Batch B = issue_batch<LC>(sh, u, true);
        if (pa) evaluate_batch<NMS, N, LC>(sh, u, lk, A);
        pa = false;
        if (u.tail == u.head) {
            evaluate_batch<NMS, N, LC>(sh, u, lk, B);
            break;
        }
        A = issue_batch<LC>(sh, u, true);
        pa = true;
        evaluate_batch<NMS, N, LC>(sh, u, lk, B);
    }
    if (pa) evaluate_batch<NMS, N, LC>(sh, u, lk, A);
    inflight[QL] = false;
}

template <int NMS, int N, bool EXACT>
__device__ __forceinline__ void sweep_unit(const SweepShared& sh, UnitCtx& u, const LerpConsts& lk) {
    constexpr int LC = kLaneCols;
    constexpr int M = LC / 4;
    constexpr int kIssue = kSweepIssue;
    using RowV = typename LaneRow<LC>::type;
    const uint32_t lane = u.lane;
    const int W = (int)u.src.W;
    const int xb = u.S - LC + LC * (int)lane;
    // candidate columns of this lane: the strip's centres (halo lanes 0 and 63 own none)
    // (bit 8j + 4 + m = lane column 4m + j, the order the FIFO entry's flags are built in)
    uint32_t vmask = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int x = xb + 4 * m + j;
            if (x >= 3 && x < W - 3 && lane >= 1 && lane <= 62) vmask |= 1u << (8 * j + 4 + m);
        }
    }
    const uint32_t lane_code = spread_code(lane);
    const int p0 = u.p0, p1 = u.p1;                    // rows run through the pre-filter
    const int ys = p0;                                 // first swept row
    u.ys = ys;
    u.rowbase = (ys - 3) * W;
    const int T = p1 - ys;                             // sweep steps (row ys + i at step i)
    u.src.ylast = p1 + 2;                              // S-row of the last pre-filtered row
    u.head = u.tail = 0;
    // kSweepBatchSlots batches in flight, in static slots (issue point q of the K-step loop
    // body uses slot q % slots), each evaluated slots issue points after it was issued
    bool inflight[kSweepBatchSlots];
    Batch batch[kSweepBatchSlots];
#pragma unroll
    for (int q = 0; q < kSweepBatchSlots; ++q) inflight[q] = false;

    // One kRing-slot ring of pixel rows: row r in slot (r - ys) % kRing.  At step J
    // (row yv) it holds rows yv .. yv+K-2 (K = kRing) with yv+4 .. yv+K-2 still loading,
    // and row yv+K-1 is loaded into the slot of row yv-1, which is dead.  Nothing is copied,
    // so every slot keeps its registers across loop iterations and no wait is needed for a
    // register move.  The loop body is K steps, so unit sweeps are whole multiples of K.
    constexpr int K = kRing;
    RowV Rw[K];
    // The N flags of rows p0 .. p0+2 come from the vertical comparisons of rows p0-3 .. p0-1
    // with them, which the steps of those rows would have made: a prologue makes only those
    // three comparisons (3 loads and 48 lerps instead of three whole pre-filter steps whose
    // candidates are masked)
    RowV up[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) up[k] = load_row<LC, EXACT>(u.src, ys - 3 + k, xb);
#pragma unroll
    for (int k = 0; k < K - 1; ++k) Rw[k] = load_row<LC, EXACT>(u.src, ys + k, xb);
    RowFlags<LC> V[4];                                 // vertical flags, slot (row-ys) & 3
#pragma unroll
    for (int k = 0; k < 3; ++k) V[k + 1] = compare_rows<LC>(Rw[k], ~up[k], lk);
    // Step J: next row load, comparisons, pre-filter of row yv, enqueue of its candidates.
    // Rows outside [p0, p1) (look-ahead and padding steps) run the pre-filter too and have
    // their candidates masked: a branch around it costs the zeroing of `cand` on every step.
#define FDF_SWEEP_STEP(J)                                                                    \
    {                                                                                        \
        const int yv = ys + i0 + (J);                                                        \
        RowV cand = (RowV)(0u);                                                              \
        Rw[((J) + K - 1) % K] = load_row<LC, EXACT>(u.src, yv + K - 1, xb);                  \
        const RowV s = Rw[((J) + 3) % K];                  /* row yv + 3 */                  \
        const RowV c = Rw[(J) % K];                        /* row yv */                      \
        const RowV nc = ~c;                                                                  \
        V[(J) & 3] = compare_rows<LC>(s, nc, lk);                                            \
        const bool live = yv >= p0 && yv < p1 && !(ablation_flags(u.flags) & kFlagNoLoad);                  \
        {                                                                                    \
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
                    /* >= 3 of 4 bright = and3(n,s,e) | (maj3(n,s,e) & w); NOT dark = >= 2 */  \
                    /* of 4 not-dark = maj3(n,s,e) | (or3(n,s,e) & w): six v_bitop3 on the */  \
                    /* raw flag words (inversions in the tables) where the compiler made 10 */ \
                    constexpr uint32_t kMaj = lut3([](int a, int b, int c) {                \
                        return (!a + b + c) >= 2; });                                        \
                    constexpr uint32_t kAnd = lut3([](int a, int b, int c) {                \
                        return !a && b && c; });                                             \
                    constexpr uint32_t kOr = lut3([](int a, int b, int c) {                 \
                        return !a || b || c; });                                             \
                    constexpr uint32_t kJoin = lut3([](int a, int b, int c) {               \
                        return a || (b && !c); });                                           \
                    const uint32_t m1 = __builtin_amdgcn_bitop3_b32(vn.nd[m], bs, be, kMaj); \
                    const uint32_t t1 = __builtin_amdgcn_bitop3_b32(vn.nd[m], bs, be, kAnd); \
                    br = __builtin_amdgcn_bitop3_b32(t1, m1, hndw, kJoin);                   \
                    const uint32_t m2 = __builtin_amdgcn_bitop3_b32(vn.b[m], ds, de, kMaj);  \
                    const uint32_t o2 = __builtin_amdgcn_bitop3_b32(vn.b[m], ds, de, kOr);   \
                    nd = __builtin_amdgcn_bitop3_b32(m2, o2, hbw, kJoin);                    \
                    (void)bn; (void)bw; (void)dn; (void)dw;                                  \
                }                                                                            \
                cand[m] = br | ~nd;                                                          \
            }                                                                                \
        }                                                                                    \
        /* the lane row's candidates into the FIFO as one entry: column 4m + j of the */     \
        /* lane is bit 8j + 4 + m (bit 7 of byte j of cand[m], moved by bit-field */         \
        /* inserts), the row and lane code in the low nibbles */                             \
        static_assert(M == 4, "four flag dwords per lane row");                              \
        /* three select-by-mask bitop3s (each after a shift), then the column mask */       \
        uint32_t cm = bitop3_sel(0x80808080u, cand[3], cand[2] >> 1);                        \
        cm = bitop3_sel(0xC0C0C0C0u, cm, cand[1] >> 2);                                      \
        cm = bitop3_sel(0xE0E0E0E0u, cm, cand[0] >> 3) & vmask;                              \
        if (live) {                                                                          \
            const bool has = cm != 0u;                                                       \
            const uint64_t bal = wave_ballot(has);                                           \
            if (has)                                                                         \
                sh.pq[(u.tail + lanes_below(bal)) & (kSweepPixelQ - 1)] =                    \
                    cm | lane_row_code | spread_code((uint32_t)(J) << 6);                    \
            u.tail += (uint32_t)__popcll(bal);                                               \
            while (u.tail - u.head > kSweepPixelQ - 64) {                                    \
                /* dense image: test the oldest pixels now, synchronously */                 \
                if (ablation_flags(u.flags) & kFlagNoFullTest) u.head = u.tail;                              \
                else evaluate_batch<NMS, N, LC>(sh, u, lk, issue_batch<LC>(sh, u, true));    \
            }                                                                                \
        }                                                                                    \
        if (((J) % kIssue) == kIssue - 1) {                                                  \
            /* the batch of this slot is due; issue the next full one into it */             \
            constexpr int q = ((J) / kIssue) % kSweepBatchSlots;                             \
            if (inflight[q]) {                                                               \
                evaluate_batch<NMS, N, LC>(sh, u, lk, batch[q]);                             \
                inflight[q] = false;                                                         \
            }                                                                                \
            if (ablation_flags(u.flags) & kFlagNoFullTest) u.head = u.tail;                                  \
            batch[q] = issue_batch<LC>(sh, u, false);                                        \
            inflight[q] = batch[q].n != 0;                                                   \
        }                                                                                    \
    }

    static_assert(K == 8 || K == 16, "ring of 8 or 16 rows (a power of two: row codes OR together)");
    static_assert((K / kIssue) % kSweepBatchSlots == 0 || kSweepBatchSlots == 1,
                  "issue points per loop body must cycle through the batch slots");
    for (int i0 = 0; i0 < T; i0 += K) {
        // FIFO code of row ys + i0 + J: i0 is a multiple of K, so its spread ORs with J's
        const uint32_t lane_row_code = lane_code | spread_code((uint32_t)i0 << 6);
        // (latency instances: leave the block after the unit's last row, wave-uniform)
#define FDF_STEP_EXIT(J) if constexpr (kExitInBlock) { if (i0 + (J) + 1 >= T) break; }
        FDF_SWEEP_STEP(0) FDF_STEP_EXIT(0)
        FDF_SWEEP_STEP(1) FDF_STEP_EXIT(1)
        FDF_SWEEP_STEP(2) FDF_STEP_EXIT(2)
        FDF_SWEEP_STEP(3) FDF_STEP_EXIT(3)
        FDF_SWEEP_STEP(4) FDF_STEP_EXIT(4)
        FDF_SWEEP_STEP(5) FDF_STEP_EXIT(5)
        FDF_SWEEP_STEP(6) FDF_STEP_EXIT(6)
        FDF_SWEEP_STEP(7)
        if constexpr (K >= 12) {
            FDF_STEP_EXIT(7)
            FDF_SWEEP_STEP(8) FDF_STEP_EXIT(8)
            FDF_SWEEP_STEP(9) FDF_STEP_EXIT(9)
            FDF_SWEEP_STEP(10) FDF_STEP_EXIT(10)
            FDF_SWEEP_STEP(11)
        }
        if constexpr (K >= 16) {
            FDF_STEP_EXIT(11)
            FDF_SWEEP_STEP(12) FDF_STEP_EXIT(12)
            FDF_SWEEP_STEP(13) FDF_STEP_EXIT(13)
            FDF_SWEEP_STEP(14) FDF_STEP_EXIT(14)
            FDF_SWEEP_STEP(15)
        }
#undef FDF_STEP_EXIT
    }
#undef FDF_SWEEP_STEP
    flush_tests<NMS, N, LC>(sh, u, lk, inflight, batch);
}

// Three bitmap bits of one bitmap row: columns x-1, x, x+1 (x-1 >= 2, x+1 < W - 3).  Both
// words are read unconditionally (the bitmap has a pad word after its last row).
__device__ __forceinline__ uint32_t bits3(const uint32_t* row, int x) {
    const int xm = x - 1, wi = xm >> 5, sh = xm & 31;
    return __builtin_amdgcn_alignbit(row[wi + 1], row[wi], (uint32_t)sh) & 7u;   // funnel shift
}

// Raster rank of bitmap position (row, x): keypoints before it in the band's bitmap.
// bprefix[row * nb + k] counts the keypoints before word 4k of the row (all rows above
// included); the position's 4-word block is one 16-byte LDS read (bitmap rows are whole
// blocks, bitmap_words_per_row).
__device__ __forceinline__ uint32_t bitmap_rank(const uint32_t* bitmap, const uint16_t* bprefix,
                                                const uint32_t* /*rprefix*/, uint32_t nw,
                                                uint32_t nb, uint32_t row, uint32_t x) {
    static_assert(kRankBlock == 4, "one 16-byte block per rank prefix");
    const uint32_t wi = x >> 5, blk = wi / kRankBlock, j = wi % kRankBlock;
    const uint4 q = reinterpret_cast<const uint4*>(bitmap + row * nw)[blk];
    uint32_t r = bprefix[row * nb + blk];
    r += j > 0 ? (uint32_t)__popc(q.x) : 0u;
    r += j > 1 ? (uint32_t)__popc(q.y) : 0u;
    r += j > 2 ? (uint32_t)__popc(q.z) : 0u;
    const uint32_t w = j == 0 ? q.x : (j == 1 ? q.y : (j == 2 ? q.z : q.w));
    return r + (uint32_t)__popc(w & ((1u << (x & 31)) - 1u));
}

// Neighbour bits of bitmap position (row, x) among the R2 bitmap rows: bit k of the up /
// down rows = column x-1+k, mid row bits 0 and 2 (columns x-1, x+1).  Non-zero iff the
// keypoint has a neighbouring keypoint.
__device__ __forceinline__ uint32_t neighbour_bits(const uint32_t* bitmap, uint32_t nw, uint32_t R2,
                                                   uint32_t row, uint32_t x) {
    return (row > 0 ? bits3(bitmap + (row - 1) * nw, (int)x) : 0u) |
           (bits3(bitmap + row * nw, (int)x) & 5u) |
           (row + 1 < R2 ? bits3(bitmap + (row + 1) * nw, (int)x) : 0u);
}

// Rank prefixes of the band's keypoint bitmap (R2 rows): bprefix[row * nb + k] = keypoints
// before word 4k of the row, the rows above included (rprefix: the row prefixes on the
// way).  Returns the bitmap's keypoint total (every thread).
__device__ uint32_t band_rank_prefixes(const uint32_t* bitmap, uint32_t R2, uint32_t nw,
                                       uint16_t* bprefix, uint32_t* rprefix, uint32_t* total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t nb_blocks = (nw + kRankBlock - 1) / kRankBlock;
    if (nb_blocks <= 32) {
        // one bitmap row per 16-lane DPP row (or per 32-lane half-wave when it has more than
        // 16 blocks, e.g. 4K): lane k counts block k, a row_shr scan (+ row_bcast:15 across
        // the two rows of a half) turns the counts into the row's block prefixes, and the
        // row's last lane ends with the row total
        const uint32_t span = nb_blocks <= 16 ? 16u : 32u;
        for (uint32_t base = 0; base < R2; base += kThreads / span) {
            const uint32_t row = base + tid / span, k = tid & (span - 1u);
            const bool act = row < R2 && k < nb_blocks;
            uint32_t cnt = 0;
            if (act) {
                const uint32_t* rw = bitmap + row * nw;
#pragma unroll
                for (uint32_t j = 0; j < kRankBlock; ++j)
                    cnt += kRankBlock * k + j < nw ? __popc(rw[kRankBlock * k + j]) : 0u;
            }
            uint32_t inc = cnt;
            inc += __builtin_amdgcn_update_dpp(0u, inc, 0x111, 0xf, 0xf, false);   // row_shr:1
            inc += __builtin_amdgcn_update_dpp(0u, inc, 0x112, 0xf, 0xf, false);   // row_shr:2
            inc += __builtin_amdgcn_update_dpp(0u, inc, 0x114, 0xf, 0xf, false);   // row_shr:4
            inc += __builtin_amdgcn_update_dpp(0u, inc, 0x118, 0xf, 0xf, false);   // row_shr:8
            if (span == 32u)
                inc += __builtin_amdgcn_update_dpp(0u, inc, 0x142, 0xa, 0xf, false);   // row_bcast:15
            if (act) bprefix[row * nb_blocks + k] = (uint16_t)(inc - cnt);
            if (row < R2 && k == span - 1u) rprefix[row] = inc;
        }
    } else {
        for (uint32_t i = tid; i < R2 * nb_blocks; i += kThreads) {
            const uint32_t row = i / nb_blocks, k = i - row * nb_blocks;
            const uint32_t* rw = bitmap + row * nw;
            uint32_t cnt = 0;
            for (uint32_t j = kRankBlock * k; j < min(kRankBlock * k + kRankBlock, nw); ++j)
                cnt += __popc(rw[j]);
            bprefix[i] = (uint16_t)cnt;
        }
        __syncthreads();
        for (uint32_t row = tid; row < R2; row += kThreads) {
            uint32_t acc = 0;
            for (uint32_t k = 0; k < nb_blocks; ++k) {
                const uint32_t c = bprefix[row * nb_blocks + k];
                bprefix[row * nb_blocks + k] = (uint16_t)acc;
                acc += c;
            }
            rprefix[row] = acc;
        }
    }
    __syncthreads();
    if (tid < 64) {   // exclusive scan of the row totals
        uint32_t carry = 0;
        for (uint32_t base = 0; base < R2; base += 64) {
            const uint32_t v = base + lane < R2 ? rprefix[base + lane] : 0u;
            uint32_t incl = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(incl, d, 64);
                if (lane >= (uint32_t)d) incl += o;
            }
            if (base + lane < R2) rprefix[base + lane] = carry + incl - v;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) *total = carry;
    }
    __syncthreads();
    // block prefixes absolute (the rows above included): one read per rank (u16 holds them:
    // the ranked tiers hold at most nms_area_entries keypoints)
    {
        const RowDiv nbd = make_rowdiv(nb_blocks);
        for (uint32_t i = tid; i < R2 * nb_blocks; i += kThreads)
            bprefix[i] = (uint16_t)(bprefix[i] + rprefix[udiv(i, nbd)]);
    }
    __syncthreads();
    return *total;
}

// Strict 3x3 maximum of list entry e (src/fast_simd.rs:596-615) against the scores of its
// neighbouring keypoints, read by raster rank from `sranked`; rows 3 / h-4 and the rows
// outside the band are reported as suppressed / not compared by the caller's rules below.
// Returns e with its score field replaced by 1 (suppressed) or 0 (kept).
// RANKED (the LDS list, at most kScoreListCap entries): the scatter left the entry's raster
// rank + 1 in its low 12 bits (its score is at that rank), so its own rank is not looked up
// again.
template <bool RANKED>
__device__ __forceinline__ uint32_t nms_entry(uint32_t e, const uint32_t* bitmap, uint32_t nw,
                                              uint32_t nb_blocks, uint32_t y0, RowDiv W,
                                              uint32_t H, uint32_t R2, const uint16_t* sranked,
                                              const uint16_t* bprefix, const uint32_t* rprefix) {
    const uint32_t pos = e >> 12, row = udiv(pos, W), x = pos - row * W;
    if (row == 0 || row == R2 - 1) return e;          // bitmap rows 0, R2-1: neighbours only
    const uint32_t y = y0 - 1 + row;
    const uint32_t low = e & 0xfffu;
    bool suppressed = y == 3 || y == H - 4;
    if (low != 0 && !suppressed) {
        const uint32_t own = RANKED ? (uint32_t)sranked[low - 1u] : low;
        uint32_t mx = 0;
        const uint32_t mid = bits3(bitmap + row * nw, (int)x);
        if (mid & 5u) {
            const uint32_t ro = RANKED ? low - 1u
                                       : bitmap_rank(bitmap, bprefix, rprefix, nw, nb_blocks, row, x);
            if (mid & 1u) mx = max(mx, (uint32_t)sranked[ro - 1]);
            if (mid & 4u) mx = max(mx, (uint32_t)sranked[ro + 1]);
        }
#pragma unroll
        for (int d = -1; d <= 1; d += 2) {
            const uint32_t nbits = bits3(bitmap + (row + d) * nw, (int)x);
            if (nbits) {
                uint32_t r = bitmap_rank(bitmap, bprefix, rprefix, nw, nb_blocks, row + d, x - 1);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    if ((nbits >> k) & 1u) {
                        mx = max(mx, (uint32_t)sranked[r]);
                        ++r;
                    }
                }
            }
        }
        suppressed = own <= mx;
    }
    return (e & ~0xfffu) | (suppressed ? 1u : 0u);
}

// Rank-order scatter of list entry e: a keypoint with a neighbouring keypoint puts its score
// at its raster rank; an isolated one is kept without comparison, marked by a zero score.
template <bool RANKED = false>
__device__ __forceinline__ uint32_t nms_scatter(uint32_t e, const uint32_t* bitmap, uint32_t nw,
                                                uint32_t R2, uint32_t nb_blocks, RowDiv W,
                                                uint16_t* sranked, const uint16_t* bprefix,
                                                const uint32_t* rprefix) {
    const uint32_t pos = e >> 12, row = udiv(pos, W), x = pos - row * W;
    if (neighbour_bits(bitmap, nw, R2, row, x) == 0) return e & ~0xfffu;
    const uint32_t rank = bitmap_rank(bitmap, bprefix, rprefix, nw, nb_blocks, row, x);
    sranked[rank] = (uint16_t)(e & 0xfffu);
    if constexpr (RANKED) return (e & ~0xfffu) | (rank + 1u);
    return e;
}

__device__ __forceinline__ void nms_clear(uint32_t e, uint32_t* bitmap, uint32_t nw, RowDiv W) {
    if ((e & 0xfffu) == 1u) {
        const uint32_t pos = e >> 12, row = udiv(pos, W), x = pos - row * W;
        atomicAnd(&bitmap[row * nw + (x >> 5)], ~(1u << (x & 31)));
    }
}

// Band NMS (src/fast_simd.rs:589-616) from the band's score list, in place on the keypoint
// bitmap (bitmap rows 0 and rows + 1 are the rows just outside the band, neighbours only).
// The list holds every keypoint of the bitmap once; its scores are scattered into raster
// rank order, then each keypoint of the band's own rows reads its neighbours' scores by
// rank, and the suppressed ones are cleared once every comparison has read the bitmap.
// Rows 3 and h-4 are never output (:590-592, :342).
//   n <= cap: the list is in LDS and the ranked scores go to the FIFO area.
//   n > cap (the band_nms_spill variant): entries past the LDS list were appended to the
//   band's slot (`spill`); the LDS entries move to registers (kSpillPer per thread), so the
//   ranked scores can use the whole FIFO + staging + list area.
template <int NMS, int N>
__device__ void band_nms_lds(uint32_t* bitmap, uint32_t rows, uint32_t nw, uint32_t y0, RowDiv W,
                             uint32_t H, uint32_t* slist, uint32_t n, uint16_t* sranked,
                             uint16_t* bprefix, uint32_t* rprefix, uint32_t* total, uint32_t flags) {
    const uint32_t tid = threadIdx.x;
    const uint32_t R2 = rows + 2, nb_blocks = (nw + kRankBlock - 1) / kRankBlock;
    band_rank_prefixes(bitmap, R2, nw, bprefix, rprefix, total);
    if (flags & kFlagNmsPrefixOnly) return;
    for (uint32_t i = tid; i < n; i += kThreads)
        slist[i] = nms_scatter<true>(slist[i], bitmap, nw, R2, nb_blocks, W, sranked, bprefix,
                                     rprefix);
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kThreads)
        slist[i] = nms_entry<true>(slist[i], bitmap, nw, nb_blocks, y0, W, H, R2, sranked, bprefix,
                                   rprefix);
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kThreads) nms_clear(slist[i], bitmap, nw, W);
    __syncthreads();
}

constexpr uint32_t kSpillPer = kScoreListCap / kThreads;

template <int NMS, int N>
__device__ void band_nms_spill(uint32_t* bitmap, uint32_t rows, uint32_t nw, uint32_t y0, RowDiv W,
                               uint32_t H, const uint32_t* slist, uint32_t cap, uint32_t* spill,
                               uint32_t n, uint16_t* sranked, uint16_t* bprefix, uint32_t* rprefix,
                               uint32_t* total) {
    const uint32_t tid = threadIdx.x;
    const uint32_t R2 = rows + 2, nb_blocks = (nw + kRankBlock - 1) / kRankBlock;
    uint32_t ent[kSpillPer];
#pragma unroll
    for (uint32_t j = 0; j < kSpillPer; ++j) ent[j] = slist[tid + j * kThreads];
    band_rank_prefixes(bitmap, R2, nw, bprefix, rprefix, total);   // barriers: list area free
#pragma unroll
    for (uint32_t j = 0; j < kSpillPer; ++j)
        ent[j] = nms_scatter(ent[j], bitmap, nw, R2, nb_blocks, W, sranked, bprefix, rprefix);
    for (uint32_t i = tid; i < n - cap; i += kThreads)
        spill[i] = nms_scatter(spill[i], bitmap, nw, R2, nb_blocks, W, sranked, bprefix, rprefix);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kSpillPer; ++j)
        ent[j] = nms_entry<false>(ent[j], bitmap, nw, nb_blocks, y0, W, H, R2, sranked, bprefix,
                                  rprefix);
    for (uint32_t i = tid; i < n - cap; i += kThreads)
        spill[i] = nms_entry<false>(spill[i], bitmap, nw, nb_blocks, y0, W, H, R2, sranked, bprefix,
                                    rprefix);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kSpillPer; ++j) nms_clear(ent[j], bitmap, nw, W);
    for (uint32_t i = tid; i < n - cap; i += kThreads) nms_clear(spill[i], bitmap, nw, W);
    __syncthreads();
}

// Score of the keypoint at (x, y) recomputed from the frame (the same windows, packing and
// score functions as the sweep's full test).
template <int NMS, int N>
__device__ __forceinline__ uint32_t keypoint_score(const __amdgpu_buffer_rsrc_t& rs, int W, int x,
                                                   int y, const LerpConsts& lk, uint32_t t) {
    Batch b;
    load_ring_windows(b, rs, (y - 3) * W + x, W);
    uint32_t w[4], c;
    pack_ring(b, w, c);
    if constexpr (NMS == kNmsSumAbsolute) {
        return score_sum_abs_packed(c, w, t);
    } else {
        bool kb, kd;
        lane_segment_test_packed<N>(c, w, lk, kb, kd);
        uint32_t p[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = (w[i & 3] >> (8 * (i >> 2))) & 0xffu;
        return score_max_threshold<N>(c, p, kd);
    }
}

// Band NMS for bands too dense for the list and its spill (more keypoints than the LDS
// list plus the slot hold, or a frame too wide for 20-bit list positions): no scores are
// stored.  Each keypoint with a neighbouring keypoint recomputes its own and its neighbours'
// scores; the kill masks go to the slot (one word per bitmap word, exactly the slot's size)
// and are applied after.  Rows 3 and h-4 are never output (:590-592, :342); the caller
// clears them.
template <int NMS, int N>
__device__ void band_nms_dense(uint32_t* bitmap, uint32_t rows, uint32_t nw, uint32_t y0,
                               uint32_t W, uint32_t* slot, __amdgpu_buffer_rsrc_t frame,
                               LerpConsts lk, uint32_t t) {
    const uint32_t tid = threadIdx.x;
    const uint32_t R2 = rows + 2;
    for (uint32_t wi = nw + tid; wi < (R2 - 1) * nw; wi += kThreads) {
        const uint32_t row = wi / nw;
        uint32_t bits = bitmap[wi], kill = 0;
        while (bits) {
            const uint32_t bit = __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t x = (wi - row * nw) * 32 + bit;
            const int y = (int)(y0 - 1 + row);
            const uint32_t mid = bits3(bitmap + row * nw, (int)x) & 5u;
            const uint32_t up = bits3(bitmap + (row - 1) * nw, (int)x);
            const uint32_t dn = bits3(bitmap + (row + 1) * nw, (int)x);
            if ((mid | up | dn) == 0) continue;
            const uint32_t own = keypoint_score<NMS, N>(frame, (int)W, (int)x, y, lk, t);
            bool suppressed = false;
#pragma unroll
            for (int d = -1; d <= 1; ++d) {
                const uint32_t nbits = d < 0 ? up : (d == 0 ? mid : dn);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    if (!suppressed && ((nbits >> k) & 1u) &&
                        keypoint_score<NMS, N>(frame, (int)W, (int)x - 1 + k, y + d, lk, t) >= own)
                        suppressed = true;
                }
            }
            if (suppressed) kill |= 1u << bit;
        }
        slot[wi - nw] = kill;
    }
    __syncthreads();
    for (uint32_t wi = nw + tid; wi < (R2 - 1) * nw; wi += kThreads) bitmap[wi] &= ~slot[wi - nw];
    __syncthreads();
}

// Direct output (BandParams::direct): the band's first output index -- the keypoints of all
// bands before it -- by a decoupled look-back.  The band publishes its own count (aggregate)
// at once, then wave 0 reads the descriptors of the 64 bands before it in one load per lane
// (agent-scope relaxed atomics: sc1 loads and stores, each descriptor one 8-byte word, so a
// flag and its value can never be seen apart), sums the aggregates down to the nearest band
// that has published its inclusive prefix, and publishes its own prefix.  A band's number is
// its workgroup's start ticket (fast_sweep_kernel), so it only waits for bands whose
// workgroups started before it -- running or done -- and every wait ends without assuming
// the grid is resident.  A wait is still bounded (~30 ms; a band waits microseconds): past
// the bound the band publishes no prefix, sets P.lookback_error and returns kLbNoBase, and
// the host recovers the output from the slots (fdf_api.cpp).  Returns the base in every
// thread.
__device__ uint64_t band_lookback(const BandParams& P, uint32_t task, uint32_t total,
                                  uint64_t* s_base) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint64_t ep = (uint64_t)P.epoch << 32;
    if (tid == 0)
        __hip_atomic_store(&P.lookback[task], ep | kLbAggregate | total, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 64) {
        uint64_t excl = 0;
        int64_t j = (int64_t)task - 1;
        uint32_t polls = 0;
        bool timed_out = false;                      // wave-uniform (polls is)
        while (j >= 0) {
            const int64_t k = j - (int64_t)lane;
            // bands before band 0 read as an inclusive prefix of 0
            const uint64_t d = k >= 0 ? __hip_atomic_load(&P.lookback[k], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : (ep | kLbPrefix);
            const bool ok = (d >> 32) == P.epoch && (d & (kLbAggregate | kLbPrefix)) != 0;
            const uint64_t pref = wave_ballot(ok && (d & kLbPrefix));
            const uint32_t stop = pref ? (uint32_t)__builtin_ctzll(pref) : 63u;
            const uint64_t need = stop == 63u ? ~0ull : (2ull << stop) - 1ull;
            if ((wave_ballot(ok) & need) != need) {
                if (++polls > (1u << 20)) {
                    timed_out = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint64_t v = lane <= stop ? (d & kLbValue) : 0ull;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            excl += v;
            if (pref) break;
            j -= 64;
        }
        if (lane == 0) {
            if (timed_out) {
                // no prefix: later bands chained on it time out the same way
                if (P.lookback_error)
                    __hip_atomic_fetch_or(P.lookback_error, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
                *s_base = kLbNoBase;
            } else {
                __hip_atomic_store(&P.lookback[task], ep | kLbPrefix | ((excl + total) & kLbValue),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *s_base = excl;
            }
        }
    }
    __syncthreads();
    return *s_base;
}

// The band (task) a workgroup sweeps.  XCD-aware static task mapping: each XCD takes a contiguous range of bands (raster
    // order), so consecutive bands of a frame land on one XCD (its L2 then serves the halo
    // rows two neighbouring bands share).  Within its range an XCD dispatches the frames'
    // full bands first and their (shorter) last bands at the end, where they fill the grid's
    // tail.
__device__ __forceinline__ uint32_t band_task(const BandParams& P) {
    const uint32_t b = blockIdx.x;
#ifdef FDF_LINEAR_TASKS
    {   // A/B variant: block b -> the b-th band in raster order over the whole grid (the
        // frames' full bands first, their last bands at the end), no XCD ranges
        const uint32_t B = P.bands_per_frame, nfull = (P.ntasks / B) * (B - 1);
        if (B <= 1) return b;
        return b < nfull ? (b / (B - 1)) * B + b % (B - 1) : (b - nfull) * B + (B - 1);
    }
#endif
    const uint32_t q8 = P.ntasks >> 3, r8 = P.ntasks & 7, k8 = b & 7;
    const uint32_t c0 = k8 * q8 + min(k8, r8), j = b >> 3;
    uint32_t task = c0 + j;
    {
        const uint32_t c1 = c0 + q8 + (k8 < r8 ? 1u : 0u);
        const uint32_t B = P.bands_per_frame;
        if (B > 1) {
            const uint32_t s0 = c0 / B, s1 = c1 / B;          // last bands before c0 / c1
            const uint32_t n_full = (c1 - c0) - (s1 - s0);
            if (j < n_full) {
                const uint32_t u = (c0 - s0) + j;              // index among full bands
                task = (u / (B - 1)) * B + u % (B - 1);
            } else {
                task = (s0 + (j - n_full)) * B + (B - 1);
            }
        }
    }
    return task;
}

// Sweeps band `task`, runs its NMS and writes its slot; returns the band's keypoint count.
template <int NMS, int N>
__device__ __forceinline__ uint32_t sweep_band(const BandParams& P, uint8_t* smem_raw, uint32_t task,
                                              uint64_t (&ph)[4]) {
    constexpr int LC = kLaneCols;
    const SweepLayout L = make_sweep_layout(P.rows, P.words_per_row, NMS);
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
    const uint32_t W = P.width, H = P.height, nw = P.words_per_row;
    constexpr uint32_t halo = NMS == kNmsOff ? 0u : 1u;
    const uint32_t frame = task / P.bands_per_frame;
    const uint32_t band = task - frame * P.bands_per_frame;
    const uint32_t y0 = 3 + band * P.rows;
    const uint32_t rows = min(P.rows, H - 3 - y0);

    uint32_t* bitmap = reinterpret_cast<uint32_t*>(smem_raw + L.bitmap);
    uint32_t* wave_sum = reinterpret_cast<uint32_t*>(smem_raw + L.misc);
    if (P.threshold >= 255) {                                        // no pixel can pass
        if (P.direct && tid == 0) {
            if (band == 0) P.frame_offsets[frame] = 0;
            if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = 0;
        }
        return 0;
    }
    uint32_t* unit_ctr = wave_sum + kWaves;
    // the bitmap and its pad word, cleared 16 bytes per store up to the (16-byte aligned)
    // end of its LDS area
    for (uint32_t i = tid; i < L.pq / 16; i += kThreads)
        reinterpret_cast<uint4*>(bitmap)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (tid == 0) {
        unit_ctr[0] = 0;
        unit_ctr[1] = 0;
    }
    {   // select_bit's table: the positions of byte tid's set bits, the k-th in nibble k
        static_assert(kThreads == 256, "one table entry per thread");
        uint32_t word = 0, k = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t bit = (tid >> i) & 1u;
            word |= bit ? i << (4u * k) : 0u;
            k += bit;
        }
        reinterpret_cast<uint32_t*>(smem_raw + L.seltab)[tid] = word;
    }
    if (P.chunk_flags && wave == 0) {
        // an overlapped upload (fdf_detect): wave 0 waits for the chunk holding the last row
        // the band reads -- its tested rows (with the NMS halo row) + 3 -- then acquires at
        // system scope, so that no line of the frame cached before the copy landed is read.
        // (Wave-uniform control flow: a per-thread wait loop costs the sweep registers.)
        const uint32_t last_row = min(H - 1, y0 + rows + halo + 2);
        uint32_t* flag = const_cast<uint32_t*>(P.chunk_flags) + last_row / P.chunk_rows;
        for (uint32_t polls = 0;; ++polls) {
            const uint32_t v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (v == P.chunk_epoch) break;
            if (polls > (1u << 20)) {                 // ~30 ms: the copy never landed
                if (P.lookback_error && lane == 0)
                    __hip_atomic_fetch_or(P.lookback_error, 2u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        // the invalidate completes asynchronously: the barrier below waits for it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if constexpr (kDebugBuild) ph[0] = __builtin_amdgcn_s_memtime();   // setup done

    SweepShared sh;
    sh.pq = reinterpret_cast<uint32_t*>(smem_raw + L.pq + wave * L.wave_bytes);
    sh.stage = reinterpret_cast<uint32_t*>(smem_raw + L.stage + wave * 64 * 4);
    sh.bitmap = bitmap;
    sh.slist = reinterpret_cast<uint32_t*>(smem_raw + L.slist);
    sh.slist_n = unit_ctr + 1;
    // list positions are (bitmap row * W + x) in 20 bits
    sh.slist_cap = (uint64_t)(rows + 2 * halo) * W <= (1u << 20) ? kScoreListCap : 0u;
    sh.spill = reinterpret_cast<uint32_t*>(P.slots + (uint64_t)task * P.slot_bytes);
    sh.spill_cap = sh.slist_cap ? P.slot_bytes / 4 : 0u;
    sh.seltab = reinterpret_cast<const uint32_t*>(smem_raw + L.seltab);

    UnitCtx u;
    const uint8_t* img = P.frames + (uint64_t)frame * P.frame_stride;
    u.src.W = W;
    u.src.H = H;
    const bool last_frame = frame + 1 == P.ntasks / P.bands_per_frame;
    // frames before the last may be read up to 15 pixels past their end (inside the batch)
    const __amdgpu_buffer_rsrc_t rs_pad = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(img), 0, (int)((W * H + 15) * kPx), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_exact = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(img), 0, (int)(W * H * kPx), 0x00020000);
    u.src.none = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(img), 0, 0, 0x00020000);
    u.t = P.threshold;
    u.nw = nw;
    u.yb = (int)(y0 - halo);
    u.lane = lane;
    u.flags = ablation_flags(P.flags);
    const LerpConsts lk = lerp_consts(P.threshold);

    const uint32_t nunits = P.nstrips * P.nsub;
    const uint32_t sub_rows = (rows + P.nsub - 1) / P.nsub;
    u.kq_n = 0;
    // units are handed out dynamically: a wave that finishes early takes the next one
    // instead of idling at the workgroup barrier
    if (!(ablation_flags(P.flags) & kFlagNoPrefilter)) {
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
            const int r0 = (int)(y0 + sub * sub_rows);
            const int r1 = (int)min(y0 + (sub + 1) * sub_rows, y0 + rows);
            if (r0 >= r1) continue;
            // NMS: the band's first and last units also test the rows just outside the band
            u.p0 = (halo && sub == 0 && r0 > 3) ? r0 - 1 : r0;
            u.p1 = (halo && r1 == (int)(y0 + rows) && r1 < (int)H - 3) ? r1 + 1 : r1;
            // rows the sweep loads: up to p1 + 2
            if (last_frame && u.p1 + 2 >= u.src.tail_row) {
                u.src.rs = rs_exact;
                sweep_unit<NMS, N, true>(sh, u, lk);
            } else {
                u.src.rs = rs_pad;
                sweep_unit<NMS, N, false>(sh, u, lk);
            }
        }
        // the band's last keypoints: a partial queue (once per wave and band)
        if constexpr (NMS == kNmsMaxThreshold)
            if (u.kq_n != 0) score_kp_queue<N>(sh, u, u.kq_n);
    }
    if constexpr (kDebugBuild) {
        ph[1] = __builtin_amdgcn_s_memtime();   // this wave's sweep done
        // every wave's sweep end (low 32 bits of the shader clock), for the stamps
        if (P.stamps && lane == 0)
            reinterpret_cast<uint32_t*>(smem_raw + L.misc + 48)[wave] = (uint32_t)ph[1];
    }
    __syncthreads();

    const uint32_t nwords = rows * nw;
    const RowDiv Wd = make_rowdiv(W), nwd = make_rowdiv(nw);
    if constexpr (NMS != kNmsOff) {
        const uint32_t n = *sh.slist_n;
        if (tid == 0 && P.kp_stats) atomicAdd(P.kp_stats, n);
        if (ablation_flags(P.flags) & kFlagNoNms) {
        } else if (n <= sh.slist_cap) {
            band_nms_lds<NMS, N>(bitmap, rows, nw, y0, Wd, H, sh.slist, n,
                                 reinterpret_cast<uint16_t*>(smem_raw + L.pq),
                                 reinterpret_cast<uint16_t*>(smem_raw + L.bprefix),
                                 reinterpret_cast<uint32_t*>(smem_raw + L.rprefix), unit_ctr + 2,
                                 ablation_flags(P.flags));
        } else if (n - sh.slist_cap <= sh.spill_cap && n <= L.nms_area_entries) {
            // more keypoints than the LDS list holds: the rest were appended to the slot
            band_nms_spill<NMS, N>(bitmap, rows, nw, y0, Wd, H, sh.slist, sh.slist_cap, sh.spill, n,
                                   reinterpret_cast<uint16_t*>(smem_raw + L.pq),
                                   reinterpret_cast<uint16_t*>(smem_raw + L.bprefix),
                                   reinterpret_cast<uint32_t*>(smem_raw + L.rprefix), unit_ctr + 2);
        } else {
            band_nms_dense<NMS, N>(bitmap, rows, nw, y0, W,
                                   reinterpret_cast<uint32_t*>(P.slots + (uint64_t)task * P.slot_bytes),
                                   rs_exact, lk, P.threshold);
            // rows 3 and h - 4 keep no keypoints (they were neighbours only)
            for (uint32_t y : {3u, H - 4u}) {
                if (y < y0 || y >= y0 + rows) continue;
                for (uint32_t w = tid; w < nw; w += kThreads) bitmap[(y - y0 + 1) * nw + w] = 0;
            }
            __syncthreads();
        }
        // the band's own rows are now its keep-bits
    }
    const uint32_t* keep = bitmap + halo * nw;
    if constexpr (kDebugBuild) ph[2] = __builtin_amdgcn_s_memtime();   // NMS done

    // ---- count keep-bits and write the band slot
    // Each wave owns a contiguous quarter of the bitmap and sweeps it 256 words per round:
    // lane = 4 words of one row (rows are whole 4-word groups, bitmap_words_per_row), one
    // 16-byte LDS read each, and a wave prefix sum of the lanes' keypoint counts places the
    // round's points consecutively in the slot.
    const uint4* keep4 = reinterpret_cast<const uint4*>(keep);
    const uint32_t ngroups = nwords / 4;
    const uint32_t gq = (ngroups + kWaves - 1) / kWaves;
    const uint32_t gb = min(wave * gq, ngroups), ge = min(gb + gq, ngroups);
    uint32_t mine = 0;
    for (uint32_t g = gb + lane; g < ge; g += 64) {
        const uint4 q = keep4[g];
        mine += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
    }
    const uint32_t wave_total = __builtin_amdgcn_readlane(wave_incl_scan(mine), 63);
    if (lane == 0) wave_sum[wave] = wave_total;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t v = wave_sum[w];
        before += (uint32_t)w < wave ? v : 0u;
        total += v;
    }
    if (ablation_flags(P.flags) & kFlagNoEmit) return total;
    uint8_t* slot = P.slots + (uint64_t)task * P.slot_bytes;
    const bool listed = total <= P.slot_bytes / 8;
    uint64_t dbase = 0;
    bool direct = P.direct != 0;
    if (direct) {
        dbase = band_lookback(P, task, total, reinterpret_cast<uint64_t*>(smem_raw + L.misc + 32));
        if constexpr (kDebugBuild) ph[3] = __builtin_amdgcn_s_memtime();   // look-back done
        direct = dbase != kLbNoBase;                  // timed out: the slot only
    }
    if (direct && tid == 0) {
        if (band == 0) P.frame_offsets[frame] = dbase;
        if (task == P.ntasks - 1) P.frame_offsets[frame + 1] = dbase + total;
    }
    if (listed || direct) {
        uint2* pts = reinterpret_cast<uint2*>(slot);
        uint32_t o = before;
        for (uint32_t g0 = gb; g0 < ge; g0 += 64) {
            const uint32_t g = g0 + lane;
            const uint4 q = g < ge ? keep4[g] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t c = __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
            const uint32_t inc = wave_incl_scan(c);
            uint32_t idx = o + inc - c;
            o += __builtin_amdgcn_readlane(inc, 63);
            const uint32_t r = udiv(4 * g, nwd);
            const uint32_t xb = (4 * g - r * nw) * 32;
            uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
            while (lo | hi) {
                uint32_t bit;
                if (lo) {
                    bit = (uint32_t)__builtin_ctzll(lo);
                    lo &= lo - 1;
                } else {
                    bit = 64u + (uint32_t)__builtin_ctzll(hi);
                    hi &= hi - 1;
                }
                const uint2 pt = make_uint2(xb + bit, y0 + r);
                if (listed) pts[idx] = pt;
                if (direct && dbase + idx < P.cap) P.out[dbase + idx] = pt;
                ++idx;
            }
        }
    }
    if (!listed) {
        uint32_t* words = reinterpret_cast<uint32_t*>(slot);
        for (uint32_t w = tid; w < nwords; w += kThreads) words[w] = keep[w];
    }
    return total;
}

// Occupancy target: kWavesEU waves per SIMD (4: 128 VGPRs each, 2: 256).
template <int NMS, int N>
__global__ __launch_bounds__(kThreads)
__attribute__((amdgpu_waves_per_eu(kWavesEU, kWavesEU)))
void fast_sweep_kernel(BandParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    uint64_t t0 = 0, r0 = 0;
    if constexpr (kDebugBuild) {   // workgroup timeline stamps (tools/stamps.py)
        if (P.stamps) {
            t0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    uint32_t task;
    if (P.direct) {
        // the band is the workgroup's start ticket (see band_lookback), raster order
        uint32_t* s_ticket = reinterpret_cast<uint32_t*>(
            smem_raw + make_sweep_layout(P.rows, P.words_per_row, NMS).misc + 40);
        if (threadIdx.x == 0) *s_ticket = atomicAdd(P.ticket, 1u) - P.ticket_base;
        __syncthreads();
        task = *s_ticket;
        // a ticket past the grid means the counter and the host's base disagree: touch no
        // band's memory, report it (bit 2 of the error word; fdf_api.cpp take_lookback_error)
        if (task >= P.ntasks) {
            if (threadIdx.x == 0 && P.lookback_error)
                __hip_atomic_fetch_or(P.lookback_error, 4u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
    } else {
        task = band_task(P);
    }
    uint64_t ph[4] = {0, 0, 0, 0};
    const uint32_t total = sweep_band<NMS, N>(P, smem_raw, task, ph);
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        P.counts[task] = total;
        if (P.group_sums) atomicAdd(&P.group_sums[task / P.tasks_per_group], total);
    }
    if constexpr (kDebugBuild) {
        if (P.stamps) {
            __syncthreads();
            if (tid == 0) {
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
                uint64_t* s = P.stamps + (uint64_t)blockIdx.x * kStampWords;
                s[0] = t0;
                s[1] = t1;
                s[2] = r0;
                s[3] = r1;
                // HW_REG_XCC_ID (20) and HW_REG_HW_ID (4), whole registers
                s[4] = ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(0xF814) << 32) |
                       (uint32_t)__builtin_amdgcn_s_getreg(0xF804);
                s[5] = task;
                for (int k = 0; k < 4; ++k) s[6 + k] = ph[k];   // phases (wave 0's view)
                const uint32_t* we = reinterpret_cast<const uint32_t*>(smem_raw +
                    make_sweep_layout(P.rows, P.words_per_row, NMS).misc + 48);
                s[10] = ((uint64_t)we[1] << 32) | we[0];          // waves' sweep ends
                s[11] = ((uint64_t)we[3] << 32) | we[2];
            }
        }
    }
}

typedef void (*SweepKernelFn)(BandParams);

template <int NMS>
static SweepKernelFn pick_sweep_n(uint32_t n) {
#if defined(FDF_ISA_ONE_N)   // ISA studies only (tools/isa_loops.py): one count per NMS mode
    return n == FDF_ISA_ONE_N ? fast_sweep_kernel<NMS, FDF_ISA_ONE_N> : nullptr;
#elif defined(FDF_AB_COUNTS)   // A/B variant builds (tools/build_variant.sh): the bench's n = 9, 12
    return n == 9 ? fast_sweep_kernel<NMS, 9> : (n == 12 ? fast_sweep_kernel<NMS, 12> : nullptr);
#else
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
#endif
}

static SweepKernelFn pick_sweep(uint32_t nms, uint32_t n) {
    switch (nms) {
        case kNmsOff: return pick_sweep_n<kNmsOff>(n);
        case kNmsMaxThreshold: return pick_sweep_n<kNmsMaxThreshold>(n);
        case kNmsSumAbsolute: return pick_sweep_n<kNmsSumAbsolute>(n);
        default: return nullptr;
    }
}

hipError_t occupancy(uint32_t nms, uint32_t n, uint32_t lds_bytes, int* wg_per_cu) {
    SweepKernelFn fn = pick_sweep(nms, n);
    if (!fn || !wg_per_cu) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(wg_per_cu, reinterpret_cast<const void*>(fn),
                                                        kThreads, lds_bytes);
}

hipError_t launch(const BandParams& p, uint32_t nms, uint32_t n, hipStream_t stream,
                  hipEvent_t start, hipEvent_t stop) {
    SweepKernelFn fn = pick_sweep(nms, n);
    if (!fn) return hipErrorInvalidValue;
    const SweepLayout L = make_sweep_layout(p.rows, p.words_per_row, nms);
    if (L.total > kSweepMaxLds) return hipErrorInvalidValue;
    if (L.total > kMaxLds) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)L.total);
        if (e != hipSuccess) return e;
    }
    if (start || stop)
        hipExtLaunchKernelGGL(fn, dim3(p.ntasks), dim3(kThreads), L.total, stream, start, stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(p.ntasks), dim3(kThreads), L.total, stream, p);
    return hipGetLastError();
}

}  // namespace FDF_SWEEP_NS
}  // namespace fdfk
