/*
 * fast_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C, scalar restatement of the reference's FAST semantics, used by tests/,
 * __graft_entry__.smoke() and bench.py's parity checks.  Nothing under
 * feature_detector_fast_amd/ links or calls this file.
 *
 * What it follows (all paths under the reference iwanders/feature_detector_fast):
 *   - detection:        src/opencv_compat.rs:79-169   (neg/pos classification :115-122,
 *                                                      cyclic run test :140-165)
 *   - max-t score:      src/opencv_compat.rs:172-209  (32-entry difference ring, window = count)
 *   - SAD score:        src/opencv_compat.rs:278-299  (paper eq. 3 over all 16 pixels)
 *   - NMS:              src/opencv_compat.rs:212-262  (skip y==3 and y==h-4 :238-240,
 *                                                      strict '>' over keypoint neighbours)
 *   - loop bounds:      src/fast_simd.rs:342, :369-371, :559-562
 *   - panics -> errors: src/fast_simd.rs:302-305 (n<9), :800 (n>16), :342/:369 (size)
 *
 * The one deliberate difference from opencv_compat.rs is performance only: its NMS looks
 * neighbours up with Vec::contains (O(K^2), :249); here a keypoint flag map answers the
 * same question.  A neighbour counts only when it is itself a keypoint, exactly as there.
 *
 * Parity of this oracle is pinned by the reference's own fixtures (tests/golden/, decoded
 * from the media/ PNGs: 309 keypoints NMS off, 131 max-t, identical for the Rust crate and
 * OpenCV 3.2) and the reference unit-test KATs (tests/test_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fast_oracle.h"

/* src/opencv_compat.rs:42-61 and src/fast_simd.rs:79-98 (same ring, same order). */
static const int kCircle[16][2] = {
    {0, -3}, {1, -3}, {2, -2}, {3, -1}, {3, 0}, {3, 1}, {2, 2}, {1, 3},
    {0, 3}, {-1, 3}, {-2, 2}, {-3, 1}, {-3, 0}, {-3, -1}, {-2, -2}, {-1, -3},
};

static void circle_values(const uint8_t* img, size_t stride, uint32_t x, uint32_t y,
                          uint8_t out[16]) {
    for (int i = 0; i < 16; ++i) {
        out[i] = img[(size_t)(y + kCircle[i][1]) * stride + (x + kCircle[i][0])];
    }
}

/* src/opencv_compat.rs:140-165: for each start s, count the cyclic take_while run. */
static int has_run(const int flags[16], int consecutive) {
    for (int s = 0; s < 16; ++s) {
        int run = 0;
        for (int k = 0; k < 16; ++k) {
            if (!flags[(s + k) % 16]) break;
            ++run;
        }
        if (run >= consecutive) return 1;
    }
    return 0;
}

int fdf_oracle_is_corner(uint8_t center, const uint8_t circle[16], uint8_t t, uint8_t n) {
    int neg[16], pos[16];
    for (int i = 0; i < 16; ++i) {
        int d = (int)center - (int)circle[i];          /* :110 delta = base - pixel */
        int a = d < 0 ? -d : d;
        neg[i] = d < 0 && a > (int)t;                   /* :119 */
        pos[i] = d > 0 && a > (int)t;                   /* :120 */
    }
    return has_run(neg, n) || has_run(pos, n);
}

/* src/opencv_compat.rs:172-209, literally: difference[i] = base - circle[i % 16], i < 32. */
uint16_t fdf_oracle_score_max_threshold(uint8_t center, const uint8_t circle[16], uint8_t n) {
    int16_t diff[32];
    for (int i = 0; i < 32; ++i) diff[i] = (int16_t)((int)center - (int)circle[i % 16]);
    int16_t extreme_highest = INT16_MIN;
    for (int k = 0; k < 16; ++k) {
        int16_t m = diff[k];
        for (int i = k; i < k + n; ++i) m = diff[i] < m ? diff[i] : m;
        extreme_highest = m > extreme_highest ? m : extreme_highest;
    }
    int16_t extreme_lowest = INT16_MAX;
    for (int k = 0; k < 16; ++k) {
        int16_t m = diff[k];
        for (int i = k; i < k + n; ++i) m = diff[i] > m ? diff[i] : m;
        extreme_lowest = m < extreme_lowest ? m : extreme_lowest;
    }
    int a = extreme_highest < 0 ? -extreme_highest : extreme_highest;
    int b = extreme_lowest < 0 ? -extreme_lowest : extreme_lowest;
    return (uint16_t)(a < b ? a : b);
}

/* src/opencv_compat.rs:278-299, literally (u8 arithmetic is safe: |d| > t implies no wrap). */
uint16_t fdf_oracle_score_sum_abs(uint8_t center, const uint8_t circle[16], uint8_t t) {
    uint16_t sum_dark = 0, sum_light = 0;
    for (int i = 0; i < 16; ++i) {
        int d = (int)center - (int)circle[i];
        int a = d < 0 ? -d : d;
        if (d > 0 && a > (int)t) sum_light += (uint8_t)((uint8_t)(center - circle[i]) - t);
        if (d < 0 && a > (int)t) sum_dark += (uint8_t)((uint8_t)(circle[i] - center) - t);
    }
    return sum_dark > sum_light ? sum_dark : sum_light;
}

int fdf_oracle_check(uint32_t w, uint32_t h, uint8_t n, uint8_t nms, int* empty) {
    *empty = 0;
    if (n < 9 || n > 16) return FDF_ORACLE_ERR_COUNT;      /* :302-305, :800 */
    if (nms > 2) return FDF_ORACLE_ERR_NMS;
    if (h < 3) return FDF_ORACLE_ERR_SIZE;                /* height - 3 underflows, :342 */
    if (h <= 6) { *empty = 1; return 0; }                 /* empty row range */
    if (w < 6) return FDF_ORACLE_ERR_SIZE;                /* width - 3 - 3 underflows, :369 */
    if (w == 6) { *empty = 1; return 0; }
    return 0;
}

int64_t fdf_oracle_detect(const uint8_t* img, uint32_t w, uint32_t h, size_t stride,
                          uint8_t t, uint8_t n, uint8_t nms, uint32_t* out_xy, size_t cap,
                          uint16_t* out_scores) {
    int empty = 0;
    int rc = fdf_oracle_check(w, h, n, nms, &empty);
    if (rc) return rc;
    if (empty) return 0;

    /* Detection, raster order (src/opencv_compat.rs:90-91). */
    uint8_t* flag = (uint8_t*)calloc((size_t)w * h, 1);
    uint16_t* score = nms ? (uint16_t*)calloc((size_t)w * h, sizeof(uint16_t)) : NULL;
    if (!flag || (nms && !score)) { free(flag); free(score); return FDF_ORACLE_ERR_ALLOC; }
    uint8_t c16[16];
    for (uint32_t y = 3; y < h - 3; ++y) {
        for (uint32_t x = 3; x < w - 3; ++x) {
            uint8_t c = img[(size_t)y * stride + x];
            circle_values(img, stride, x, y, c16);
            if (!fdf_oracle_is_corner(c, c16, t, n)) continue;
            flag[(size_t)y * w + x] = 1;
            if (nms == 1) score[(size_t)y * w + x] = fdf_oracle_score_max_threshold(c, c16, n);
            if (nms == 2) score[(size_t)y * w + x] = fdf_oracle_score_sum_abs(c, c16, t);
        }
    }

    int64_t count = 0;
    for (uint32_t y = 3; y < h - 3; ++y) {
        for (uint32_t x = 3; x < w - 3; ++x) {
            size_t i = (size_t)y * w + x;
            if (!flag[i]) continue;
            if (nms) {
                /* src/opencv_compat.rs:236-260 */
                if (y == 3 || y == h - 4) continue;
                uint16_t s = score[i];
                int keep = 1;
                for (int dx = -1; dx <= 1 && keep; ++dx) {
                    for (int dy = -1; dy <= 1; ++dy) {
                        if (!dx && !dy) continue;
                        size_t j = (size_t)(y + dy) * w + (x + dx);
                        if (!flag[j]) continue;            /* keypoints.contains :249 */
                        if (s <= score[j]) { keep = 0; break; }
                    }
                }
                if (!keep) continue;
            }
            if ((size_t)count < cap) {
                out_xy[2 * count] = x;
                out_xy[2 * count + 1] = y;
                if (out_scores) out_scores[count] = nms ? score[i] : 0;
            }
            ++count;
        }
    }
    free(flag);
    free(score);
    return count;
}

/* image 0.24.6 color.rs rgb_to_luma for u8 (its Larger type is u32): the crate is not
 * vendored in the reference, so this restates its published integer formula,
 *   SRGB_LUMA = [2126, 7152, 722], SRGB_LUMA_DIV = 10000, l / SRGB_LUMA_DIV (truncating).
 * Grey input (r = g = b) maps to itself; colour input is parity-unpinned. */
void fdf_oracle_rgb_to_luma(const uint8_t* rgb, uint32_t w, uint32_t h, size_t rgb_stride,
                            uint8_t* out) {
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* row = rgb + (size_t)y * rgb_stride;
        for (uint32_t x = 0; x < w; ++x) {
            const uint32_t l = 2126u * row[3 * x] + 7152u * row[3 * x + 1] + 722u * row[3 * x + 2];
            out[(size_t)y * w + x] = (uint8_t)(l / 10000u);
        }
    }
}

/* Scores of given image points with the functions above (test helper for the GPU's
 * fdf_score_points at scale): kind 1 = max-threshold (window n, src/opencv_compat.rs:172-209),
 * kind 2 = SAD (threshold t, :278-299).  Points must be centres (3 from every border). */
void fdf_oracle_score_points(const uint8_t* img, size_t stride, const uint32_t* xy,
                             size_t n_pts, uint8_t kind, uint8_t t, uint8_t n, uint16_t* out) {
    uint8_t c16[16];
    for (size_t k = 0; k < n_pts; ++k) {
        const uint32_t x = xy[2 * k], y = xy[2 * k + 1];
        const uint8_t c = img[(size_t)y * stride + x];
        circle_values(img, stride, x, y, c16);
        out[k] = kind == 2 ? fdf_oracle_score_sum_abs(c, c16, t)
                           : fdf_oracle_score_max_threshold(c, c16, n);
    }
}

/* Scores of (centre, ring) tuples (test helper for the GPU's fdf_score_rings): kind as
 * fdf_oracle_score_points; ring k is rings[16 k .. 16 k + 16) in circle order. */
void fdf_oracle_score_rings(const uint8_t* centers, const uint8_t* rings, size_t n_rings,
                            uint8_t kind, uint8_t t, uint8_t n, uint16_t* out) {
    for (size_t k = 0; k < n_rings; ++k)
        out[k] = kind == 2 ? fdf_oracle_score_sum_abs(centers[k], rings + 16 * k, t)
                           : fdf_oracle_score_max_threshold(centers[k], rings + 16 * k, n);
}
