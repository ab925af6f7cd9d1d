/*
 * sgbm_oracle.h -- CPU restatement of the reference's hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the stereo_depth_ruler_amd engine.  It restates, in plain
 * scalar C, the third-party algorithms the reference calls on its hot path:
 *
 *   cv::StereoSGBM::compute          OpenCV 4.6.0 modules/calib3d/src/stereosgbm.cpp
 *   cv::medianBlur(ksize=3, CV_16S)  OpenCV 4.6.0 modules/imgproc/src/median_blur.simd.hpp
 *   cv::filterSpeckles               OpenCV 4.6.0 modules/calib3d/src/stereosgbm.cpp
 *   cv::reprojectImageTo3D           OpenCV 4.6.0 modules/calib3d/src/calibration.cpp
 *   cv::cvtColor(BGR2GRAY, 8U)       OpenCV 4.6.0 modules/imgproc/src/color_rgb.simd.hpp
 *   cv::resize(0.5, INTER_AREA, 8U)  OpenCV 4.6.0 modules/imgproc/src/resize.cpp (area-fast path)
 *
 * Reference call sites (under /root/reference):
 *   stereo_vision/src/stereo_disparity.cpp:5-9    StereoSGBM::create(0,80,5,600,2400,1,63,12,200,2,3WAY)
 *   stereo_vision/src/stereo_disparity.cpp:19-24  cvtColor BGR2GRAY + resize 0.5 INTER_AREA
 *   stereo_vision/src/stereo_disparity.cpp:27-28  matcher->compute / right_matcher->compute
 *   stereo_vision/src/stereo_disparity.cpp:78     reprojectImageTo3D(disp, depth, Q)
 *   point_cloud/src/pcd_write.cpp:102-116         SGBM compute + convertTo(1/16) + reproject(handleMissing)
 *
 * PARITY UNPINNED against real OpenCV: OpenCV 4.6.0 is a third-party dependency (Ubuntu apt,
 * reference Dockerfile:1,11-16) that is absent from /root/reference and from this image, and the
 * reference holds no golden vectors, fixtures or tests for this path.  The
 * restatement follows the published OpenCV 4.6.0 algorithm as recalled in SURVEY.md Appendix A
 * (corrections noted inline where the survey's recollection was revised) and is pinned instead by
 * analytic known-answer tests and independent numpy/scipy restatements of each stage
 * (tests/test_oracle_*.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline.  The product path never links it.
 */
#ifndef SDR_SGBM_ORACLE_H
#define SDR_SGBM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_MODE_SGBM = 0, ORC_MODE_HH = 1, ORC_MODE_SGBM_3WAY = 2, ORC_MODE_HH4 = 3 };
enum { ORC_UNIQ_AUTO = 0, ORC_UNIQ_SCALAR = 1, ORC_UNIQ_SIMD = 2 };

/* Same field order and meaning as cv::StereoSGBM::create(minDisparity, numDisparities,
 * blockSize, P1, P2, disp12MaxDiff, preFilterCap, uniquenessRatio, speckleWindowSize,
 * speckleRange, mode), plus the two knobs OpenCV fixes internally. */
typedef struct orc_params {
    int minDisparity;
    int numDisparities;
    int blockSize;
    int P1;
    int P2;
    int disp12MaxDiff;
    int preFilterCap;
    int uniquenessRatio;
    int speckleWindowSize;
    int speckleRange;
    int mode;
    int nstripes;   /* MODE_SGBM_3WAY stripe count; OpenCV 4.x fixes it at 4 */
    int uniq_rule;  /* ORC_UNIQ_AUTO: 3WAY uses the SIMD threshold rule, SGBM/HH the scalar rule */
} orc_params;

/* Full StereoSGBM::compute: mode function, medianBlur(3), filterSpeckles if speckleWindowSize>0.
 * left/right: 8-bit single channel, same stride.  disp: CV_16S (1/16 px). Returns 0 on success. */
int orc_sgbm_compute(const uint8_t* left, const uint8_t* right, int width, int height,
                     size_t stride, const orc_params* p, int16_t* disp, size_t disp_stride_elems);

/* Stage flags for orc_sgbm_compute_stages (bit set = run that stage). */
enum { ORC_STAGE_MEDIAN = 1, ORC_STAGE_SPECKLE = 2 };
int orc_sgbm_compute_stages(const uint8_t* left, const uint8_t* right, int width, int height,
                            size_t stride, const orc_params* p, int16_t* disp,
                            size_t disp_stride_elems, int stages);

/* StereoSGBM::compute on 8-bit images with cn (1 or 3) interleaved channels (calcPixelCostBT's
 * cn == 3 branch: per-channel Sobel and raw costs summed), stride bytes per row. */
int orc_sgbm_compute_cn(const uint8_t* left, const uint8_t* right, int width, int height,
                        size_t stride, int cn, const orc_params* p, int16_t* disp,
                        size_t disp_stride_elems, int stages);

/* Cost volume C(y, x, d) = P2 + 5x5 (blockSize) box sum of the BT pixel cost, exactly as the
 * SGBM (stripe start s0 = 0) driver forms it, for every row.  mode selects the bottom-row rule
 * (HH keeps the initial P2 on rows the running sum never reaches).  out: [height][width1][D]. */
int orc_cost_volume(const uint8_t* left, const uint8_t* right, int width, int height,
                    size_t stride, const orc_params* p, int16_t* out);
int orc_cost_volume_cn(const uint8_t* left, const uint8_t* right, int width, int height,
                       size_t stride, int cn, const orc_params* p, int16_t* out);

/* One row of Birchfield-Tomasi pixel costs (calcPixelCostBT), out: [width1][D]. */
int orc_pixel_cost_row(const uint8_t* left, const uint8_t* right, int width, int height,
                       size_t stride, int y, int minD, int numD, int preFilterCap, int16_t* out);

/* cv::medianBlur(src, dst, 3) on CV_16S, replicate border. src != dst. */
void orc_median3x3_s16(const int16_t* src, int16_t* dst, int width, int height);

/* cv::filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on CV_16S, in place. */
void orc_filter_speckles_s16(int16_t* img, int width, int height, int newVal,
                             int maxSpeckleSize, int maxDiff);

/* cv::reprojectImageTo3D(disp CV_32F, xyz CV_32FC3, Q, handleMissingValues). */
void orc_reproject_f32(const float* disp, int width, int height, const double Q[16],
                       int handle_missing, float* xyz);

/* cv::cvtColor(bgr, gray, COLOR_BGR2GRAY) for 8U. */
void orc_bgr2gray(const uint8_t* bgr, int width, int height, size_t bgr_stride, uint8_t* gray);

/* cv::resize(src, dst, Size(), 0.5, 0.5, INTER_AREA) for 8U single channel, even sizes. */
void orc_resize_area_half(const uint8_t* src, int width, int height, size_t stride, uint8_t* dst);

/* disp.convertTo(f, CV_32F, 1/16). */
void orc_disp_to_float(const int16_t* disp, int n, float* out);

#ifdef __cplusplus
}
#endif
#endif
