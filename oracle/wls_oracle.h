/*
 * wls_oracle.h -- CPU restatement of the class path's post-filter (TEST INFRASTRUCTURE ONLY).
 *
 *   cv::ximgproc::createDisparityWLSFilter(matcher)  opencv_contrib 4.6.0 ximgproc/src/disparity_filters.cpp
 *   DisparityWLSFilter::filter(dl, left_view, out, dr)          (same file)
 *   cv::ximgproc::FastGlobalSmootherFilter::filter              ximgproc/src/fgs_filter.cpp
 *
 * Reference call sites: stereo_vision/src/stereo_disparity.cpp:11-13 (create, setLambda(8000),
 * setSigmaColor(1.1)) and :31 (filter(disp_left, left_small, filtered, disp_right)).
 *
 * PARITY UNPINNED against real opencv_contrib: it is a third-party apt dependency (reference
 * Dockerfile:11-16) absent from /root/reference and this image, with no fixtures in the
 * reference.  This restates the published algorithm (Min et al., "Fast Global Image Smoothing
 * Based on Weighted Least Squares", TIP 2014, as implemented by ximgproc) as recalled:
 *
 *   confidence  = 255 * min(discL(x), discR(x - dL>>4)) where |dL + dR(x - dL>>4)| < LRC_thresh,
 *                 0 where that test fails, discL(x) where x - dL>>4 leaves the right ROI;
 *                 disc = max(1 - roll_off * var7x7(d), 0), var = boxmean(d^2) - boxmean(d)^2
 *                 over the ROI copy with BORDER_REFLECT_101 (radius ceil(0.5*blockSize)).
 *   FGS         = num_iter x (row tridiagonal solve, column tridiagonal solve), lambda *= 0.25
 *                 per iteration; weights w = exp(-sqrt(|dI|^2)/sigma) between 4-neighbours of
 *                 the guide, system (1 + lambda*sum w) u_p - lambda*sum w u_q = f_p (Thomas).
 *                 Two solvers of that system are restated (fgs_solver): ORC_FGS_THOMAS, the
 *                 sequential elimination ximgproc runs; ORC_FGS_PCR, parallel cyclic reduction
 *                 (the engine's default: every stage is data-parallel).  Both solve the same
 *                 diagonally dominant system; they differ only in float rounding (tests pin PCR
 *                 against THOMAS at <= 1 int16 level on the WLS output).
 *   output      = saturate_cast<short>(FGS(conf * d) / FGS(conf)) (0 where FGS(conf) == 0)
 *                 inside the valid ROI, 16*(minDisparity-1) outside.
 *   ROI (SGBM)  = (max(0, minD+numD), 0, W - that - max(0, -minD), H).
 *
 * The float operation order is this file's; the GPU path follows it exactly (contraction off,
 * IEEE division, the same host-computed weight table), so GPU parity against THIS oracle is
 * bit-exact while parity against OpenCV stays unpinned.
 */
#ifndef SDR_WLS_ORACLE_H
#define SDR_WLS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double lambda;             /* setLambda (stereo_disparity.cpp:12: 8000) */
    double sigma_color;        /* setSigmaColor (stereo_disparity.cpp:13: 1.1) */
    int lrc_thresh;            /* 24 */
    int depth_disc_radius;     /* ceil(0.5 * blockSize) for StereoSGBM */
    float roll_off;            /* depth_discontinuity_roll_off_factor, 0.001 */
    double lambda_attenuation; /* FGS default 0.25 */
    int num_iter;              /* FGS default 3 */
    int roi_x, roi_y, roi_w, roi_h; /* valid ROI of the left disparity map */
    int min_disp;              /* left matcher minDisparity (outside-ROI value 16*(min_disp-1)) */
    int fgs_solver;            /* ORC_FGS_THOMAS (default: ximgproc's order) or ORC_FGS_PCR */
} orc_wls_params;

enum { ORC_FGS_PCR = 0, ORC_FGS_THOMAS = 1 };

/* createDisparityWLSFilter(StereoSGBM) defaults for a W x H left map. */
void orc_wls_params_for_sgbm(int minDisparity, int numDisparities, int blockSize, int width,
                             int height, orc_wls_params* p);

/* FGS weight table: lut[i] = -exp(-sqrt(i)/sigma), i = squared guide difference (0..65025). */
void orc_fgs_lut(double sigma_color, float* lut /* 65026 */);

/* Depth-discontinuity confidence of `d` inside roi (ones elsewhere): out W*H floats. */
void orc_wls_disc_map(const int16_t* d, int width, int height, int rx, int ry, int rw, int rh,
                      int radius, float roll_off, float* out);

/* DisparityWLSFilter confidence map (x255), W*H floats. */
void orc_wls_confidence(const int16_t* dl, const int16_t* dr, int width, int height,
                        const orc_wls_params* p, float* conf);

/* FastGlobalSmootherFilter(guide, lambda, sigma, attenuation, iters).filter(img) in place;
 * img and guide are w x h (guide row stride gstride bytes).  Sequential (Thomas) line solves. */
void orc_fgs_filter_f32(const uint8_t* guide, size_t gstride, int w, int h, double lambda,
                        double sigma_color, double lambda_attenuation, int num_iter, float* img);
/* The same filter with the line solver chosen by `solver` (ORC_FGS_*). */
void orc_fgs_filter_f32_ex(const uint8_t* guide, size_t gstride, int w, int h, double lambda,
                           double sigma_color, double lambda_attenuation, int num_iter, int solver,
                           float* img);

/* DisparityWLSFilter::filter(dl, guide, out, dr): out W*H int16; conf_out (nullable) W*H. */
void orc_wls_filter(const int16_t* dl, const int16_t* dr, const uint8_t* guide, size_t gstride,
                    int width, int height, const orc_wls_params* p, int16_t* out, float* conf_out);

#ifdef __cplusplus
}
#endif
#endif
