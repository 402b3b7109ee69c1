/* fast_oracle.h -- TEST INFRASTRUCTURE ONLY: scalar CPU restatement of the reference's
 * FAST semantics (see fast_oracle.c for the file:line it follows). */
#ifndef FDF_FAST_ORACLE_H
#define FDF_FAST_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Negative return codes of fdf_oracle_detect (mirror include/fdf.h's FDF_ERR_* values). */
#define FDF_ORACLE_ERR_COUNT (-1)
#define FDF_ORACLE_ERR_SIZE (-2)
#define FDF_ORACLE_ERR_NMS (-4)
#define FDF_ORACLE_ERR_ALLOC (-7)

int fdf_oracle_is_corner(uint8_t center, const uint8_t circle[16], uint8_t t, uint8_t n);
uint16_t fdf_oracle_score_max_threshold(uint8_t center, const uint8_t circle[16], uint8_t n);
uint16_t fdf_oracle_score_sum_abs(uint8_t center, const uint8_t circle[16], uint8_t t);
int fdf_oracle_check(uint32_t w, uint32_t h, uint8_t n, uint8_t nms, int* empty);
/* image 0.24.6 DynamicImage::to_luma8 on Rgb<u8> (src/main.rs:58, tests/compare.rs:33):
 * luma = (2126 r + 7152 g + 722 b) / 10000, integer division.  Rows of 3*w bytes at
 * rgb_stride; output packed w*h. */
void fdf_oracle_rgb_to_luma(const uint8_t* rgb, uint32_t w, uint32_t h, size_t rgb_stride,
                            uint8_t* out);

/* Returns the keypoint count (>= 0; only the first `cap` are written as x,y pairs into
 * out_xy and, if non-NULL, their NMS scores into out_scores) or a negative error code. */
int64_t fdf_oracle_detect(const uint8_t* img, uint32_t w, uint32_t h, size_t stride,
                          uint8_t t, uint8_t n, uint8_t nms, uint32_t* out_xy, size_t cap,
                          uint16_t* out_scores);

/* Scores of image points (test helper): kind 1 = max-threshold (window n), 2 = SAD (t). */
void fdf_oracle_score_points(const uint8_t* img, size_t stride, const uint32_t* xy,
                             size_t n_pts, uint8_t kind, uint8_t t, uint8_t n, uint16_t* out);

/* Scores of (centre, 16 circle pixels) tuples: kind as fdf_oracle_score_points. */
void fdf_oracle_score_rings(const uint8_t* centers, const uint8_t* rings, size_t n_rings,
                            uint8_t kind, uint8_t t, uint8_t n, uint16_t* out);

#ifdef __cplusplus
}
#endif
#endif
