/*
 * rectify_oracle.h -- CPU restatement of cv::initUndistortRectifyMap (CV_16SC2) and cv::remap
 * (INTER_LINEAR, BORDER_CONSTANT 0) as the reference's StereoRectifier uses them
 * (stereo_vision/src/stereo_rectifier.cpp:7-11, 39-40).  TEST INFRASTRUCTURE ONLY; see
 * rectify_oracle.c for the restated formulas and why parity with OpenCV is unpinned.
 */
#ifndef SDR_RECTIFY_ORACLE_H
#define SDR_RECTIFY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* iR = inv(P[:, :3] * R), P row-major with p_cols (3 or 4) columns */
void orc_rectify_inv_matrix(const double K[9], const double R[9], const double P[12], int p_cols,
                            double iR[9]);

/* map1: int16 [H][W][2] (integer x, y), map2: uint16 [H][W] (5-bit fractional y*32 + x) */
void orc_init_undistort_rectify_map(const double K[9], const double* dist, int ndist,
                                    const double R[9], const double P[12], int p_cols, int W, int H,
                                    int16_t* map1, uint16_t* map2);

/* remap of an 8-bit image with cn (1 or 3) interleaved channels, dst dw x dh */
void orc_remap_bilinear_u8(const uint8_t* src, int sw, int sh, size_t sstride, int cn,
                           const int16_t* map1, const uint16_t* map2, int dw, int dh,
                           uint8_t* dst, size_t dstride);

#ifdef __cplusplus
}
#endif
#endif
