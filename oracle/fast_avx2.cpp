// fast_avx2.cpp -- TEST / BASELINE INFRASTRUCTURE ONLY: a C++ port of the reference's AVX2
// detector (iwanders/feature_detector_fast src/fast_simd.rs:51-859), intrinsic for
// intrinsic, so bench.py can time "the reference's own AVX2 CPU path" on the GPU box's
// host cores (the Rust toolchain is absent there and here).  It is never
// linked into the product (feature_detector_fast_amd/), and tests check it against the
// scalar oracle before bench.py times it (cpu_baseline.kind = "port").
//
// Built with -O3 -mavx2 (mirrors .cargo/config.toml:2).  One deliberate deviation: the
// reference's 4-byte gathers read up to 3 bytes past the last pixel;
// callers here must pass buffers with >= 4 readable padding bytes after the image.
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <vector>

namespace {

struct Pt {
    uint32_t x, y;
};

constexpr int kNorth = 0, kEast = 4, kSouth = 8, kWest = 12;   // src/fast_simd.rs:69-72
constexpr int kCircle[16][2] = {{0, -3}, {1, -3}, {2, -2}, {3, -1}, {3, 0}, {3, 1},
                                {2, 2},  {1, 3},  {0, 3},  {-1, 3}, {-2, 2}, {-3, 1},
                                {-3, 0}, {-3, -1}, {-2, -2}, {-1, -3}};
constexpr int kOff = 0, kMaxT = 1, kSad = 2;   // NONMAX_* (:74-76)

// :104-110
void calculate_offsets(uint32_t w, int32_t off[16]) {
    for (int i = 0; i < 16; ++i) off[i] = kCircle[i][1] * (int32_t)w + kCircle[i][0];
}

// :753-760 unsigned byte compare via the sign flip
inline __m128i cmpgt_epu8(__m128i a, __m128i b) {
    const __m128i k = _mm_set1_epi8((char)0x80);
    return _mm_cmpgt_epi8(_mm_xor_si128(a, k), _mm_xor_si128(b, k));
}
// :762-770
inline uint16_t minpos_epu16_256(__m256i v) {
    const int lo = _mm_extract_epi16(_mm_minpos_epu16(_mm256_extracti128_si256(v, 0)), 0);
    const int hi = _mm_extract_epi16(_mm_minpos_epu16(_mm256_extracti128_si256(v, 1)), 0);
    return (uint16_t)std::min(lo, hi);
}
// :773-794 rotate 16 u16 lanes left by one across the two 128-bit halves
inline __m256i rotate_across_2(__m256i v) {
    const __m256i r = _mm256_alignr_epi8(v, v, 2);
    const __m256i swapped = _mm256_permute2x128_si256(r, r, 1);
    const __m256i mask = _mm256_set_epi64x((long long)0xFFFF000000000000ull, 0,
                                           (long long)0xFFFF000000000000ull, 0);
    return _mm256_blendv_epi8(r, swapped, mask);
}
// :797-812
inline __m128i consecutive_mask_128(int n) {
    alignas(16) uint8_t m[16] = {};
    for (int i = 0; i < n; ++i) m[i] = 0xff;
    return _mm_load_si128(reinterpret_cast<const __m128i*>(m));
}
inline __m256i consecutive_mask_256(int n) {
    alignas(32) uint16_t m[16] = {};
    for (int i = 0; i < n; ++i) m[i] = 0xffff;
    return _mm256_load_si256(reinterpret_cast<const __m256i*>(m));
}
// :815-817
inline __m128i rotate_across_1(__m128i v) { return _mm_alignr_epi8(v, v, 1); }
// :821-824
inline uint32_t sum_epu8(__m128i v) {
    const __m128i s = _mm_sad_epu8(v, _mm_setzero_si128());
    return (uint32_t)(_mm_cvtsi128_si32(s) + _mm_extract_epi16(s, 4));
}

// :623-718
uint16_t score_max_threshold(uint8_t base, __m128i pixels, int n) {
    const __m256i px = _mm256_set_m128i(_mm_set1_epi64x(0), pixels);
    const __m256i centers = _mm256_set1_epi16(base);
    const __m256i idx = _mm256_set_epi64x(0x0700000007ll, 0x0300000002ll, 0x0700000007ll,
                                          0x0100000000ll);
    const __m256i two_lanes = _mm256_permutevar8x32_epi32(px, idx);
    const __m256i as_i16 = _mm256_unpacklo_epi8(two_lanes, _mm256_setzero_si256());
    __m256i diff = _mm256_sub_epi16(_mm256_add_epi16(centers, _mm256_set1_epi16(512)), as_i16);
    const __m256i cm = consecutive_mask_256(n);
    const __m256i not_cm = _mm256_andnot_si256(cm, _mm256_set1_epi8(-1));
    alignas(32) uint16_t mins[16], maxs[16];
    for (int k = 0; k < 16; ++k) {
        mins[k] = minpos_epu16_256(_mm256_or_si256(_mm256_and_si256(diff, cm), not_cm));
        const __m256i from_top = _mm256_sub_epi16(_mm256_set1_epi16(-1), diff);
        maxs[k] = minpos_epu16_256(_mm256_or_si256(_mm256_and_si256(from_top, cm), not_cm));
        diff = rotate_across_2(diff);
    }
    const __m256i minv = _mm256_load_si256(reinterpret_cast<const __m256i*>(mins));
    const int lowest_min = minpos_epu16_256(_mm256_sub_epi16(_mm256_set1_epi16(1024), minv));
    const int16_t extreme_highest = (int16_t)(1024 - lowest_min - 512);
    const __m256i maxv = _mm256_load_si256(reinterpret_cast<const __m256i*>(maxs));
    const int lowest_max = minpos_epu16_256(_mm256_sub_epi16(_mm256_set1_epi16(1024), maxv));
    const int16_t extreme_lowest = (int16_t)(lowest_max - (1024 + 512 + 1));
    const int a = extreme_highest < 0 ? -extreme_highest : extreme_highest;
    const int b = extreme_lowest < 0 ? -extreme_lowest : extreme_lowest;
    return (uint16_t)std::min(a, b);
}

// :722-749
uint16_t score_sum_abs(__m128i pixels, __m128i centers, __m128i above, __m128i below,
                       __m128i thr) {
    const __m128i bright = _mm_and_si128(_mm_subs_epu8(_mm_subs_epu8(centers, pixels), thr), below);
    const __m128i dark = _mm_and_si128(_mm_subs_epu8(_mm_subs_epu8(pixels, centers), thr), above);
    return (uint16_t)std::max(sum_epu8(bright), sum_epu8(dark));
}

// :115-297
template <int NMS>
inline bool determine_keypoint(const uint8_t* data, const int32_t off[16], uint32_t w,
                               uint32_t x, uint32_t y, uint8_t t, uint8_t n,
                               __m128i consec, uint16_t* score) {
    const size_t base = (size_t)y * w + x;
    const uint8_t base_v = data[base];
    const __m128i thr = _mm_set1_epi8((char)t);
    const __m128i center = _mm_set1_epi8((char)base_v);
    const int* lookup = reinterpret_cast<const int*>(data + base);
    const __m256i g0 = _mm256_i32gather_epi32(
        lookup, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&off[0])), 1);
    const __m256i m0 = _mm256_set_epi64x((long long)0x8080808080808080ull, 0x808080800c080400ll,
                                         (long long)0x8080808080808080ull, 0x808080800c080400ll);
    const __m256i first = _mm256_shuffle_epi8(g0, m0);
    const __m256i g1 = _mm256_i32gather_epi32(
        lookup, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&off[kSouth])), 1);
    const __m256i m1 = _mm256_set_epi64x(0x808080800c080400ll, (long long)0x8080808080808080ull,
                                         0x808080800c080400ll, (long long)0x8080808080808080ull);
    const __m256i second = _mm256_shuffle_epi8(g1, m1);
    const __m256i both = _mm256_or_si256(first, second);
    const __m256i idx = _mm256_set_epi64x(0x0100000001ll, 0x0100000001ll, 0x0600000002ll,
                                          0x0400000000ll);
    const __m128i p = _mm256_extracti128_si256(_mm256_permutevar8x32_epi32(both, idx), 0);

    const __m128i upper = _mm_adds_epu8(center, thr);
    const __m128i lower = _mm_subs_epu8(center, thr);
    const __m128i above = cmpgt_epu8(p, upper);
    const __m128i below = cmpgt_epu8(lower, p);
    const __m128i ones = _mm_set1_epi8(-1);
    __m128i cm = consec;
    for (int k = 0; k < 16; ++k) {
        const __m128i tail = _mm_andnot_si128(cm, ones);
        const __m128i a = _mm_or_si128(_mm_and_si128(above, cm), tail);
        const __m128i b = _mm_or_si128(_mm_and_si128(below, cm), tail);
        if (_mm_test_all_ones(a) || _mm_test_all_ones(b)) {
            if (NMS == kMaxT) *score = score_max_threshold(base_v, p, n);
            if (NMS == kSad) *score = score_sum_abs(p, center, above, below, thr);
            return true;
        }
        cm = rotate_across_1(cm);
    }
    return false;
}

// :301-620
template <int NMS>
void detect(const uint8_t* data, uint32_t w, uint32_t h, uint8_t t, uint8_t n,
            std::vector<Pt>& r) {
    std::vector<uint16_t> pending((size_t)w * 3, 0);
    uint16_t* rows[3] = {pending.data(), pending.data() + w, pending.data() + 2 * w};
    int32_t off[16];
    calculate_offsets(w, off);
    const __m128i thr = _mm_set1_epi8((char)t);
    const __m128i consec = consecutive_mask_128(n);
    const uint32_t chunks = (w - 6) / 16;
    for (uint32_t y = 3; y < h - 3; ++y) {
        uint16_t* y2 = rows[(y + 0) % 3];
        uint16_t* y1 = rows[(y + 1) % 3];
        uint16_t* y0 = rows[(y + 2) % 3];
        std::fill(y0, y0 + w, (uint16_t)0);
        for (uint32_t xs = 0; xs < chunks; ++xs) {
            const uint32_t x = 3 + xs * 16;
            const size_t b = (size_t)y * w + x;
            auto load = [&](int64_t o) {
                return _mm_loadu_si128(reinterpret_cast<const __m128i*>(data + (int64_t)b + o));
            };
            const __m128i c = load(0);
            const __m128i north = load(off[kNorth]), east = load(off[kEast]);
            const __m128i south = load(off[kSouth]), west = load(off[kWest]);
            const __m128i upper = _mm_adds_epu8(c, thr), lower = _mm_subs_epu8(c, thr);
            const __m128i na = cmpgt_epu8(north, upper), ea = cmpgt_epu8(east, upper);
            const __m128i sa = cmpgt_epu8(south, upper), wa = cmpgt_epu8(west, upper);
            const __m128i nb = cmpgt_epu8(lower, north), eb = cmpgt_epu8(lower, east);
            const __m128i sb = cmpgt_epu8(lower, south), wb = cmpgt_epu8(lower, west);
            __m128i check;
            if (n < 12) {   // :441-472
                const __m128i a2 = _mm_or_si128(_mm_or_si128(_mm_and_si128(sa, wa), _mm_and_si128(na, wa)),
                                                _mm_or_si128(_mm_and_si128(na, ea), _mm_and_si128(ea, sa)));
                const __m128i b2 = _mm_or_si128(_mm_or_si128(_mm_and_si128(sb, wb), _mm_and_si128(nb, wb)),
                                                _mm_or_si128(_mm_and_si128(nb, eb), _mm_and_si128(eb, sb)));
                check = _mm_or_si128(a2, b2);
            } else {        // :473-506
                const __m128i a3 = _mm_or_si128(
                    _mm_or_si128(_mm_and_si128(_mm_and_si128(ea, sa), wa), _mm_and_si128(_mm_and_si128(na, sa), wa)),
                    _mm_or_si128(_mm_and_si128(_mm_and_si128(na, ea), wa), _mm_and_si128(_mm_and_si128(na, ea), sa)));
                const __m128i b3 = _mm_or_si128(
                    _mm_or_si128(_mm_and_si128(_mm_and_si128(eb, sb), wb), _mm_and_si128(_mm_and_si128(nb, sb), wb)),
                    _mm_or_si128(_mm_and_si128(_mm_and_si128(nb, eb), wb), _mm_and_si128(_mm_and_si128(nb, eb), sb)));
                check = _mm_or_si128(a3, b3);
            }
            if (_mm_test_all_zeros(check, check)) continue;   // :518-520
            __m128i shift = _mm_set_epi64x(0, 0xff);
            for (uint32_t xx = x; xx < x + 16; ++xx) {          // :524-555
                const bool unset = _mm_test_all_zeros(check, shift);
                shift = _mm_bslli_si128(shift, 1);
                if (unset) continue;
                uint16_t s = 0;
                if (determine_keypoint<NMS>(data, off, w, xx, y, t, n, consec, &s)) {
                    if (NMS == kOff) r.push_back({xx, y});
                    else y0[xx] = s;
                }
            }
        }
        for (uint32_t xs = chunks * 16; xs < w - 6; ++xs) {   // tail :559-586
            const uint32_t x = xs + 3;
            uint16_t s = 0;
            if (determine_keypoint<NMS>(data, off, w, x, y, t, n, consec, &s)) {
                if (NMS == kOff) r.push_back({x, y});
                else y0[x] = s;
            }
        }
        if (NMS != kOff) {                                     // :589-616
            if (y == 4) continue;
            for (uint32_t x = 3; x < w - 3; ++x) {
                const uint16_t s = y1[x];
                if (!s) continue;
                if (s > y2[x - 1] && s > y2[x] && s > y2[x + 1] && s > y1[x - 1] &&
                    s > y1[x + 1] && s > y0[x - 1] && s > y0[x] && s > y0[x + 1])
                    r.push_back({x, y - 1});
            }
        }
    }
}

}  // namespace

extern "C" {

// Returns the keypoint count (first `cap` written to out_xy as x,y pairs) or a negative
// error: -1 count, -2 size, -4 nms (same codes as the scalar oracle).
int64_t fdf_avx2_detect(const uint8_t* data, uint32_t w, uint32_t h, uint8_t t, uint8_t n,
                        uint8_t nms, uint32_t* out_xy, size_t cap) {
    if (n < 9 || n > 16) return -1;
    if (nms > 2) return -4;
    if (h < 3) return -2;
    if (h <= 6) return 0;
    if (w < 6) return -2;
    if (w == 6) return 0;
    std::vector<Pt> r;
    if (nms == kOff) detect<kOff>(data, w, h, t, n, r);
    else if (nms == kMaxT) detect<kMaxT>(data, w, h, t, n, r);
    else detect<kSad>(data, w, h, t, n, r);
    for (size_t i = 0; i < r.size() && i < cap; ++i) {
        out_xy[2 * i] = r[i].x;
        out_xy[2 * i + 1] = r[i].y;
    }
    return (int64_t)r.size();
}

// Times `reps` passes over `n_frames` frames (frame f at frames + f * frame_stride, each
// padded as above), spreading frames over `threads` std::threads.  Returns wall seconds
// and the keypoint total of one pass in *total.
// With `cpus` (threads entries), worker i pins itself to CPU cpus[i] before it starts.
double fdf_avx2_time_pinned(const uint8_t* frames, uint32_t n_frames, size_t frame_stride,
                            uint32_t w, uint32_t h, uint8_t t, uint8_t n, uint8_t nms,
                            int threads, int reps, const int* cpus, uint64_t* total) {
    if (threads < 1) threads = 1;
    std::vector<uint64_t> counts(threads, 0);
    auto worker = [&](int tid) {
        if (cpus) {
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(cpus[tid], &set);
            (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        uint64_t c = 0;
        for (int rep = 0; rep < reps; ++rep) {
            for (uint32_t f = tid; f < n_frames; f += threads) {
                std::vector<Pt> r;   // the reference allocates its Vec per call
                const uint8_t* d = frames + (size_t)f * frame_stride;
                if (nms == kOff) detect<kOff>(d, w, h, t, n, r);
                else if (nms == kMaxT) detect<kMaxT>(d, w, h, t, n, r);
                else detect<kSad>(d, w, h, t, n, r);
                if (rep == 0) c += r.size();
            }
        }
        counts[tid] = c;
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int i = 1; i < threads; ++i) pool.emplace_back(worker, i);
    worker(0);
    for (auto& th : pool) th.join();
    const auto t1 = std::chrono::steady_clock::now();
    uint64_t sum = 0;
    for (uint64_t c : counts) sum += c;
    if (total) *total = sum;
    return std::chrono::duration<double>(t1 - t0).count();
}

// Whole-batch checker: the keypoints of every frame (frame f at frames + f * frame_stride,
// the batch padded as above), frame f on worker f % threads, concatenated in frame order.
// offsets[f] .. offsets[f+1] are frame f's points; the first `cap` points go to out_xy.
// Returns the total, or a negative error as fdf_avx2_detect.
int64_t fdf_avx2_detect_batch(const uint8_t* frames, uint32_t n_frames, size_t frame_stride,
                              uint32_t w, uint32_t h, uint8_t t, uint8_t n, uint8_t nms,
                              int threads, uint32_t* out_xy, size_t cap, uint64_t* offsets) {
    if (n < 9 || n > 16) return -1;
    if (nms > 2) return -4;
    if (h < 3 || (h > 6 && w < 6)) return -2;
    if (threads < 1) threads = 1;
    std::vector<std::vector<Pt>> per(n_frames);
    auto worker = [&](int tid) {
        for (uint32_t f = tid; f < n_frames; f += threads) {
            if (h <= 6 || w == 6) continue;
            const uint8_t* d = frames + (size_t)f * frame_stride;
            if (nms == kOff) detect<kOff>(d, w, h, t, n, per[f]);
            else if (nms == kMaxT) detect<kMaxT>(d, w, h, t, n, per[f]);
            else detect<kSad>(d, w, h, t, n, per[f]);
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < threads; ++i) pool.emplace_back(worker, i);
    worker(0);
    for (auto& th : pool) th.join();
    uint64_t k = 0;
    for (uint32_t f = 0; f < n_frames; ++f) {
        if (offsets) offsets[f] = k;
        for (const Pt& p : per[f]) {
            if (k < cap) {
                out_xy[2 * k] = p.x;
                out_xy[2 * k + 1] = p.y;
            }
            ++k;
        }
    }
    if (offsets) offsets[n_frames] = k;
    return (int64_t)k;
}

double fdf_avx2_time(const uint8_t* frames, uint32_t n_frames, size_t frame_stride,
                     uint32_t w, uint32_t h, uint8_t t, uint8_t n, uint8_t nms, int threads,
                     int reps, uint64_t* total) {
    return fdf_avx2_time_pinned(frames, n_frames, frame_stride, w, h, t, n, nms, threads, reps,
                                nullptr, total);
}

// Criterion-like single-frame protocol (benches/benchmark.rs:18-50): `warmup` untimed
// calls, then `samples` calls timed one by one (steady_clock, ms into out_ms).  The frame
// must be padded as above.  Returns the keypoint count of one call.
int64_t fdf_avx2_samples(const uint8_t* frame, uint32_t w, uint32_t h, uint8_t t, uint8_t n,
                         uint8_t nms, int warmup, int samples, double* out_ms) {
    int64_t count = 0;
    for (int i = -warmup; i < samples; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<Pt> r;   // the reference allocates its Vec per call
        if (nms == kOff) detect<kOff>(frame, w, h, t, n, r);
        else if (nms == kMaxT) detect<kMaxT>(frame, w, h, t, n, r);
        else detect<kSad>(frame, w, h, t, n, r);
        const auto t1 = std::chrono::steady_clock::now();
        count = (int64_t)r.size();
        if (i >= 0) out_ms[i] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    return count;
}

}  // extern "C"
