// fdf_common.h -- device helpers of the FAST kernels (fdf_sweep.hip, fdf_kernels.hip):
// circle geometry, byte-SWAR comparisons, wave ballots, the per-lane segment test and the
// two NMS score functions of the reference (iwanders/feature_detector_fast).
#pragma once
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

constexpr uint32_t kHigh = 0x80808080u;

__device__ __forceinline__ uint32_t lerp_u8(uint32_t a, uint32_t b, uint32_t r) {
    return __builtin_amdgcn_lerp(a, b, r);
}
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
// v_cmp straight into an SGPR pair (HIP's __ballot(int) round-trips the bool through a VGPR).
__device__ __forceinline__ uint64_t wave_ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// base + the set bits of `mask` below this lane (mbcnt's accumulator: no separate add)
__device__ __forceinline__ uint32_t lanes_below_plus(uint64_t mask, uint32_t base) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, base));
}
// The v_bitop3 truth table of f(a, b, c): bit (a << 2 | b << 1 | c) = f(a, b, c).
template <typename F>
__host__ __device__ constexpr uint32_t lut3(F f) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i)
        if (f((i >> 2) & 1, (i >> 1) & 1, i & 1)) r |= 1u << i;
    return r;
}
// sel ? a : b, bit by bit, in one v_bitop3 (LUT 0xCA: src0 selects src1 over src2)
__device__ __forceinline__ uint32_t bitop3_sel(uint32_t sel, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(sel, a, b, 0xCA);
}
// a * b for a, b < 2^24 as one full-rate v_mul_u32_u24 (the compiler turns both the
// masked product and __umul24 into a quarter-rate v_mul_lo_u32 here); `a` wave-uniform
__device__ __forceinline__ uint32_t mul_u24_s(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(a), "v"(b));
    return r;
}

// Division by a per-launch divisor d (a frame width, bitmap words per row) for x < 2^24:
// q = hi32(x * m) with m = ceil(2^32 / d) is q_true or q_true + 1 (x * (m d - 2^32) / d
// < x < 2^32 / 2^8), then one 24-bit multiply-compare corrects it -- 4 VALU instead of the
// ~20 of a u32 division by a runtime value.  d = 1 has no 32-bit m (m = 0 marks it).
// Converts to d, so `row * W` reads as before.
struct RowDiv {
    uint32_t d, m;
    __device__ __forceinline__ operator uint32_t() const { return d; }
};
__device__ __forceinline__ RowDiv make_rowdiv(uint32_t d) {
    RowDiv r;
    r.d = d;
    r.m = d >= 2u ? 0xffffffffu / d + 1u : 0u;
    return r;
}
__device__ __forceinline__ uint32_t udiv(uint32_t x, const RowDiv& r) {
    if (r.m == 0u) return x;
    const uint32_t q = __umulhi(x, r.m);
    return q - (__umul24(q, r.d) > x ? 1u : 0u);
}

// Byte 0 of x in all four bytes: one v_perm (x * 0x01010101 is a quarter-rate v_mul_lo_u32).
__device__ __forceinline__ uint32_t bcast_byte(uint32_t x) {
    return __builtin_amdgcn_perm(0u, x, 0u);
}

// Per-launch byte constants of the lerp comparisons (threshold t < 255).
struct LerpConsts {
    uint32_t rb, kb, rd, kd;
};
__device__ __forceinline__ LerpConsts lerp_consts(uint32_t t) {
    LerpConsts k;
    const uint32_t ob = t & 1u, od = (t + 1u) & 1u;
    k.rb = ob * 0x01010101u;
    k.kb = (128u - ((t + ob) >> 1)) * 0x01010101u;
    k.rd = od * 0x01010101u;
    k.kd = (255u - ((254u - t + od) >> 1)) * 0x01010101u;
    return k;
}

// Segment test, one pixel per lane, all in VALU.
// run_of: `m` holds the 16 circle flags twice (pixel i at bits i and i+16); true when some
// cyclic run of >= N flags is set (src/fast_simd.rs:247-295), by doubling ANDs: after the
// k-th AND, bit i means "flags i .. i + 2^k - 1 are all set".
template <int N>
__device__ __forceinline__ bool run_of(uint32_t m) {
    m &= m >> 1;
    m &= m >> 2;
    m &= m >> 4;
    if constexpr (N > 8) m &= m >> (N - 8);
    return (m & 0xffffu) != 0;
}

// Bit 7 of byte j of f[m] is the flag of circle pixel 4j + m -> pixels 0..7 in byte 1 and
// 8..15 in byte 3 (pixel i at bit 8 + i, resp. 24 + i - 8), of the flags or (INV) of their
// inverses: the flags go to bits 7..4 of each byte by masked selects (zero below), then
// each byte's nibble joins the next byte's: 8 VALU, the inversion in the select tables.
template <bool INV>
__device__ __forceinline__ uint32_t gather_ring(const uint32_t (&f)[4]) {
    constexpr uint32_t kSel = lut3([](int s, int a, int b) { return s ? (INV ? !a : a) : b; });
    constexpr uint32_t kTop = lut3([](int s, int a, int) { return s && (INV ? !a : a); });
    uint32_t t = __builtin_amdgcn_bitop3_b32(0x80808080u, f[3], 0u, kTop);
    t = __builtin_amdgcn_bitop3_b32(0x40404040u, f[2] >> 1, t, kSel);
    t = __builtin_amdgcn_bitop3_b32(0x20202020u, f[1] >> 2, t, kSel);
    t = __builtin_amdgcn_bitop3_b32(0x10101010u, f[0] >> 3, t, kSel);
    return t | (t << 4);
}

// Runs of >= N in two 16-bit cyclic rings at once (bright in bits 0-15, dark in 16-31):
// bit i of a half ANDed with the half rotated right by 1, 2, 4 and N - 8 (packed 16-bit
// shifts), so bit i ends as "flags i .. i + N - 1 of that ring all set".
template <int N>
__device__ __forceinline__ uint32_t runs16x2(uint32_t m) {
    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t kAndOr = lut3([](int a, int b, int c) { return a && (b || c); });
    auto step = [&](uint32_t x, uint16_t s) {
        const u16x2 v = __builtin_bit_cast(u16x2, x);
        const u16x2 hi = v >> (u16x2)(s), lo = v << (u16x2)((uint16_t)(16 - s));
        return __builtin_amdgcn_bitop3_b32(x, __builtin_bit_cast(uint32_t, hi),
                                           __builtin_bit_cast(uint32_t, lo), kAndOr);
    };
    m = step(m, 1);
    m = step(m, 2);
    m = step(m, 4);
    if constexpr (N > 8) m = step(m, N - 8);
    return m;
}

// Bright / dark runs of >= N (src/fast_simd.rs:115-297) on the ring packed 4 bytes per word
// (byte j of w[m] = circle pixel 4j + m), compared with the exact lerp SWAR.
template <int N>
__device__ __forceinline__ void lane_segment_test_packed(uint32_t c, const uint32_t (&w)[4],
                                                         const LerpConsts& k, bool& bright,
                                                         bool& dark) {
    const uint32_t nc = ~bcast_byte(c);
    uint32_t fb[4], fn[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        fb[m] = lerp_u8(lerp_u8(w[m], nc, k.rb), k.kb, 0);   // p - c > t
        fn[m] = lerp_u8(lerp_u8(w[m], nc, k.rd), k.kd, 0);   // NOT(p - c < -t)
    }
    // bright ring in bits 0-15, dark (inverted fn) in bits 16-31: bytes 1 and 3 of each
    const uint32_t rings = __builtin_amdgcn_perm(gather_ring<true>(fn), gather_ring<false>(fb),
                                                 0x07050301u);
    const uint32_t m = runs16x2<N>(rings);
    bright = (m & 0xffffu) != 0;
    dark = m > 0xffffu;
}

// The same on 16 separate ring bytes.
template <int N>
__device__ __forceinline__ void lane_segment_test(uint32_t c, const uint32_t (&p)[16],
                                                  const LerpConsts& k, bool& bright, bool& dark) {
    uint32_t w[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        w[m] = p[m] | (p[m + 4] << 8) | (p[m + 8] << 16) | (p[m + 12] << 24);
    lane_segment_test_packed<N>(c, w, k, bright, dark);
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

// The same SAD score from the packed ring (byte j of w[m] = circle pixel 4j + m) with
// v_sad_u8 (per-byte |a - b| summed into an accumulator).  With U = min(c + t, 255) and
// L = max(c - t, 0) (clamping changes no term: p <= 255, p >= 0) and max(x, 0) = (|x| + x) / 2:
//   sum max(p - U, 0) = (sum |p - U| + sum p - 16 U) / 2
//   sum max(L - p, 0) = (sum |p - L| - sum p + 16 L) / 2
// -- 12 v_sad_u8 instead of ~100 unpack / sub / max / add operations.
__device__ __forceinline__ uint32_t score_sum_abs_packed(uint32_t c, const uint32_t (&w)[4],
                                                         uint32_t t) {
    const uint32_t U = min(c + t, 255u), L = c > t ? c - t : 0u;
    const uint32_t U4 = bcast_byte(U), L4 = bcast_byte(L);
    uint32_t su = 0, sl = 0, sp = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        su = __builtin_amdgcn_sad_u8(w[m], U4, su);
        sl = __builtin_amdgcn_sad_u8(w[m], L4, sl);
        sp = __builtin_amdgcn_sad_u8(w[m], 0u, sp);
    }
    return max((su + sp - 16u * U) >> 1, (sl + 16u * L - sp) >> 1);
}

}  // namespace fdfk
