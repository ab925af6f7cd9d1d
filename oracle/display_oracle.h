/*
 * display_oracle.h -- CPU restatement of the reference's display outputs.
 * TEST INFRASTRUCTURE ONLY.  Parity against OpenCV 4.6 is UNPINNED (see display_oracle.c).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_COLORMAP_JET = 2, ORC_COLORMAP_TURBO = 20 }; /* cv::COLORMAP_* codes */

/* 256-entry BGR table of a colormap from its published definition */
int orc_colormap_lut(int colormap, uint8_t lut_bgr[768]);

/* StereoDisparity::show_disparityMap on one frame; prev (nullable) = prev_vis */
void orc_show_disparity_map(const float* disp, int width, int height, int num_disp,
                            const uint8_t* prev, uint8_t* out);

/* show_depthMap's range smoothing: zrange = {zmin_smooth, zmax_smooth} in/out; returns the
 * convertTo scale and shift as the floats the conversion uses */
void orc_depth_range_update(const float* xyz, int width, int height, int channels,
                            double zrange[2], float* scale, float* shift);

/* StereoDisparity::show_depthMap on one frame (updates zrange); prev (nullable) = prev_depth_vis */
void orc_show_depth_map(const float* xyz, int width, int height, int channels, double zrange[2],
                        const uint8_t* lut_bgr, const uint8_t* prev_bgr, uint8_t* out_bgr);

/* applyColorMap(8UC1 -> 8UC3) with a BGR table */
void orc_apply_colormap(const uint8_t* src, size_t n, const uint8_t* lut_bgr, uint8_t* out_bgr);

/* cv::addWeighted on 8U data (n values) */
void orc_add_weighted_u8(const uint8_t* a, double alpha, const uint8_t* b, double beta,
                         double gamma, size_t n, uint8_t* out);

/* resize(bgr, 0.5, 0.5, INTER_AREA) of an 8UC3 image (even sizes) */
void orc_resize_area_half_bgr(const uint8_t* src, int width, int height, size_t stride,
                              uint8_t* dst);

/* StereoDisplayer::depth_coverage: percentage of pixels with Z in [0, 12000] (not NaN) among
 * columns >= col0, over all rows*cols pixels */
double orc_depth_coverage(const float* xyz, int width, int height, int col0);

#ifdef __cplusplus
}
#endif
