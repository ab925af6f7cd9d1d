/*
 * sdr.h -- C ABI of the MI355X-native stereo disparity engine (stereo_depth_ruler_amd).
 *
 * Drop-in boundary for the reference's hot path: every entry point takes plain pointers and
 * sizes (no OpenCV, no torch types) and replaces one OpenCV call the reference makes:
 *
 *   sdr_sgbm_create / sdr_sgbm_set_params
 *       <- cv::StereoSGBM::create(0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, MODE_SGBM_3WAY)
 *          stereo_vision/src/stereo_disparity.cpp:5-9, point_cloud/src/pcd_write.cpp:102-108
 *   sdr_sgbm_compute / sdr_sgbm_compute_device
 *       <- matcher->compute(L, R, disp)  stereo_vision/src/stereo_disparity.cpp:27-28,
 *          sgbm->compute(left_gray, right_gray, disp)  point_cloud/src/pcd_write.cpp:111
 *   sdr_reproject / sdr_reproject_device / sdr_disp16_reproject_device
 *       <- cv::reprojectImageTo3D(disp, xyz, Q, handleMissing)  stereo_disparity.cpp:78,
 *          pcd_write.cpp:116 (with disp.convertTo(CV_32F, 1/16) at pcd_write.cpp:112)
 *   sdr_bgr2gray_device / sdr_resize_area_half_device
 *       <- cv::cvtColor(BGR2GRAY) / cv::resize(0.5, INTER_AREA)  stereo_disparity.cpp:19-24
 *   sdr_right_matcher_params
 *       <- cv::ximgproc::createRightMatcher(matcher)  stereo_disparity.cpp:10
 *
 * Error behaviour mirrors the CV_Assert()s of StereoSGBMImpl::compute: a negative status is
 * returned instead of throwing; sdr_last_error() returns the thread's last message.
 * Threading: one handle = one HIP stream + scratch; a handle must not be used by two threads at
 * once (as with cv::StereoSGBM, whose impl owns a scratch buffer); handles are independent.
 */
#ifndef SDR_SDR_H
#define SDR_SDR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDR_ABI_VERSION 4

/* cv::StereoSGBM::MODE_* */
enum { SDR_MODE_SGBM = 0, SDR_MODE_HH = 1, SDR_MODE_SGBM_3WAY = 2, SDR_MODE_HH4 = 3 };

/* uniqueness test form: AUTO = 3WAY uses OpenCV's SIMD threshold form
 * cost <= (100*minS)/(100-u), SGBM/HH the scalar form cost*(100-u) < minS*100 */
enum { SDR_UNIQ_AUTO = 0, SDR_UNIQ_SCALAR = 1, SDR_UNIQ_SIMD = 2 };

/* status codes */
enum {
    SDR_OK = 0,
    SDR_ERR_ARG = -1,         /* null pointer, non-positive size, bad stride */
    SDR_ERR_NUMDISP = -2,     /* numDisparities <= 0 or not a multiple of 16 (OpenCV assert) */
    SDR_ERR_MODE = -3,        /* unknown mode */
    SDR_ERR_SIZE = -4,        /* image too narrow for the disparity range / block size */
    SDR_ERR_TYPE = -5,        /* channels other than 1 or 3 (CV_8UC1 / CV_8UC3) */
    SDR_ERR_DEVICE = -6,      /* HIP runtime error */
    SDR_ERR_NOMEM = -7,
    SDR_ERR_LIMIT = -8        /* numDisparities > 512, or outside the int16 cost domain */
};

/* Field order and meaning of cv::StereoSGBM::create(...) + two knobs OpenCV fixes internally. */
typedef struct sdr_sgbm_params {
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
    int nstripes;   /* MODE_SGBM_3WAY stripes; 0 -> 4 (OpenCV 4.x fixed value) */
    int uniq_rule;  /* SDR_UNIQ_* */
} sdr_sgbm_params;

typedef struct sdr_sgbm sdr_sgbm;
typedef struct sdr_wls sdr_wls; /* ximgproc::DisparityWLSFilter (below) */

/* StereoSGBM::create defaults: (0, 16, 3, 0, 0, 0, 0, 0, 0, 0, MODE_SGBM) */
void sdr_sgbm_params_default(sdr_sgbm_params* p);
/* createRightMatcher: minD' = -(minD+numD)+1, uniqueness 0, disp12MaxDiff 1e6, speckle off */
void sdr_right_matcher_params(const sdr_sgbm_params* left, sdr_sgbm_params* right);

int sdr_sgbm_create(const sdr_sgbm_params* p, int device, sdr_sgbm** out);
int sdr_sgbm_destroy(sdr_sgbm* h);
int sdr_sgbm_set_params(sdr_sgbm* h, const sdr_sgbm_params* p);
int sdr_sgbm_get_params(const sdr_sgbm* h, sdr_sgbm_params* p);
/* HIP stream (hipStream_t) the handle launches on (NULL = the HIP null stream, e.g. torch's
 * default stream); a new handle uses a stream of its own, restored by sdr_sgbm_reset_stream.
 * Changing the stream orders the handle's earlier work before the new stream's.
 * sdr_sgbm_set_stream binds a TRANSIENT stream: the caller may destroy it as soon as the calls
 * made on it have returned (and its work is done, as hipStreamDestroy requires); the handle
 * never touches it afterwards -- at the end of every call on it the handle records an event
 * there and relays it through its own stream, which later switches, sdr_sgbm_last_status and
 * sdr_sgbm_destroy use instead.  The next call must follow a set_stream / reset_stream naming a
 * live stream.
 * sdr_sgbm_set_stream_ex(.., SDR_STREAM_PERSISTENT) binds a stream that outlives the handle's use
 * of it (a pooled stream such as torch's, or one the caller keeps until it has moved the handle
 * off it): no event is recorded per call, only at the next switch (an event record is a queue
 * barrier: ~6 us of idle queue per class-path frame when recorded after every call).  The
 * Python layer passes the flag for torch's pooled and default streams, not for external ones. */
enum { SDR_STREAM_PERSISTENT = 1 };
int sdr_sgbm_set_stream(sdr_sgbm* h, void* stream);
int sdr_sgbm_set_stream_ex(sdr_sgbm* h, void* stream, int flags);
int sdr_sgbm_reset_stream(sdr_sgbm* h);
void* sdr_sgbm_get_stream(const sdr_sgbm* h);

/* Host-pointer compute (H2D, compute, D2H, synchronous): left/right 8-bit with `channels` (1 or 3)
 * interleaved channels, `stride` bytes per row; disp int16 (1/16 px), `disp_stride` ELEMENTS per row.  Replaces StereoSGBM::compute on
 * host cv::Mat (stereo_disparity.cpp:27-34, pcd_write.cpp:111).  The copies go through the
 * handle's persistent page-locked staging in ~1 MB row chunks that overlap the CPU copy with the
 * DMA; no allocation per call once the handle has seen the frame size. */
int sdr_sgbm_compute(sdr_sgbm* h, const uint8_t* left, const uint8_t* right, int width, int height,
                     int channels, size_t stride, int16_t* disp, size_t disp_stride);

/* Host-pointer form of the fused hot path of pcd_write.cpp:111-116 (synchronous): compute ->
 * convertTo(CV_32F, 1/16) -> reprojectImageTo3D(Q, handle_missing) with the disparity kept on
 * the device; xyz float32x3 rows of `xyz_stride` ELEMENTS (>= 3*width).  disp (optional, may be
 * NULL) receives the int16 disparity as sdr_sgbm_compute would, its copy-out overlapping the
 * reprojection. */
int sdr_sgbm_compute_reproject(sdr_sgbm* h, const uint8_t* left, const uint8_t* right, int width,
                               int height, size_t stride, int16_t* disp, size_t disp_stride,
                               const double Q[16], int handle_missing, float* xyz,
                               size_t xyz_stride);

/* Device-pointer batch compute, asynchronous on the handle's stream: nframes frames spaced
 * frame_stride bytes (inputs) / disp_frame_stride elements (output) apart.  Once a call of the
 * same shape has sized the scratch, the enqueue allocates nothing and may be captured into a
 * hipGraph on the handle's stream (hipStreamBeginCapture, global mode) and replayed; a captured
 * batched MODE_HH call takes the per-direction chains instead of the row sweeps. */
int sdr_sgbm_compute_device(sdr_sgbm* h, const uint8_t* d_left, const uint8_t* d_right,
                            int width, int height, size_t stride, size_t frame_stride,
                            int nframes, int16_t* d_disp, size_t disp_stride,
                            size_t disp_frame_stride);

/* sdr_sgbm_compute_device for 8-bit images with `channels` (1 or 3) interleaved channels (stride
 * and frame_stride in bytes): StereoSGBM::compute on CV_8UC3 input, whose calcPixelCostBT sums each
 * channel's Sobel and raw costs (stereosgbm.cpp, cn == 3 branch). */
int sdr_sgbm_compute_device_cn(sdr_sgbm* h, const uint8_t* d_left, const uint8_t* d_right,
                               int width, int height, int channels, size_t stride,
                               size_t frame_stride, int nframes, int16_t* d_disp,
                               size_t disp_stride, size_t disp_frame_stride);

/* Fused hot path of point_cloud/src/pcd_write.cpp:111-116 on device: compute + convertTo(1/16)
 * + reprojectImageTo3D(Q, handle_missing) -> xyz float32x3 [nframes][height][width][3]. */
int sdr_sgbm_compute_reproject_device(sdr_sgbm* h, const uint8_t* d_left, const uint8_t* d_right,
                                      int width, int height, size_t stride, size_t frame_stride,
                                      int nframes, int16_t* d_disp, const double Q[16],
                                      int handle_missing, float* d_xyz);

/* reprojectImageTo3D on a CV_32F disparity (host pointers, synchronous; per-thread persistent
 * device buffers and page-locked staging, no allocation per call). */
int sdr_reproject(const float* disp, int width, int height, size_t disp_stride, const double Q[16],
                  int handle_missing, float* xyz, size_t xyz_stride);
/* Device versions (asynchronous on `stream`, a hipStream_t; NULL = default stream). */
int sdr_reproject_device(const float* d_disp, int width, int height, size_t disp_stride,
                         const double Q[16], int handle_missing, float* d_xyz, size_t xyz_stride,
                         int nframes, void* stream);
int sdr_disp16_reproject_device(const int16_t* d_disp, int width, int height, size_t disp_stride,
                                const double Q[16], int handle_missing, float* d_xyz,
                                size_t xyz_stride, int nframes, void* stream);
/* cv::filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on dense int16 frames [nframes][H][W],
 * in place, asynchronous on `stream`.  This is the post-filter StereoSGBM::compute applies with
 * newVal = (minDisparity-1)*16, maxDiff = 16*speckleRange; scratch is
 * stream-ordered, from a device memory pool the library keeps for the process (freed blocks stay
 * mapped for the next call). */
int sdr_filter_speckles_device(int16_t* d_img, int width, int height, int nframes, int newVal,
                               int maxSpeckleSize, int maxDiff, void* stream);
/* disp.convertTo(f, CV_32F, 1/16) on device. */
int sdr_disp16_to_float_device(const int16_t* d_disp, float* d_out, size_t n, void* stream);

/* Class-path pre-steps on device (stereo_disparity.cpp:19-24). */
int sdr_bgr2gray_device(const uint8_t* d_bgr, int width, int height, size_t bgr_stride,
                        uint8_t* d_gray, size_t gray_stride, int nframes, void* stream);
int sdr_resize_area_half_device(const uint8_t* d_src, int width, int height, size_t stride,
                                uint8_t* d_dst, size_t dst_stride, int nframes, void* stream);

/* StereoDisparity::computeDisparity class path (stereo_disparity.cpp:17-39) on host BGR frames:
 * cvtColor(BGR2GRAY) -> resize(0.5, INTER_AREA) -> left->compute(L, R) -> right->compute(R, L)
 * -> wls->filter(dl, left_small, filtered, dr) -> convertTo(CV_32F, 1/16), all on the left
 * matcher's device.  out: float (height/2)x(width/2).  right and wls may be NULL (no WLS: out is
 * the left matcher's disparity).  disp_left/disp_right/filtered (int16) and conf (float, the
 * getConfidenceMap() of stereo_disparity.cpp:36) are optional host outputs of (h/2)x(w/2). */
int sdr_stereo_class_compute(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                             const uint8_t* bgr_left, const uint8_t* bgr_right, int width,
                             int height, size_t bgr_stride, float* out, size_t out_stride,
                             int16_t* disp_left, int16_t* disp_right, int16_t* filtered,
                             float* conf);

/* ---- ximgproc DisparityWLSFilter / FastGlobalSmootherFilter (class path, stereo_disparity.cpp:11-13,31,36) ----
 * Field meaning follows opencv_contrib 4.6 ximgproc (disparity_filters.cpp, fgs_filter.cpp):
 * the valid ROI of a W x H left map is (left_offset, top_offset, W-left-right, H-top-bottom). */
typedef struct sdr_wls_params {
    double lambda;                  /* setLambda (default 8000; the reference sets 8000) */
    double sigma_color;             /* setSigmaColor (default 1.5; the reference sets 1.1) */
    int lrc_thresh;                 /* setLRCthresh (24) */
    int depth_discontinuity_radius; /* setDepthDiscontinuityRadius (SGBM: ceil(0.5*blockSize)) */
    float roll_off;                 /* depth_discontinuity_roll_off_factor (0.001) */
    double lambda_attenuation;      /* FGS lambda attenuation per iteration (0.25) */
    int num_iter;                   /* FGS iterations (3) */
    int left_offset, right_offset, top_offset, bottom_offset;
    int min_disp;                   /* outside-ROI value is 16*(min_disp-1) */
    int fgs_solver;                 /* SDR_FGS_THOMAS (default) or SDR_FGS_PCR (below) */
} sdr_wls_params;

/* Solver of the FGS line systems (I + lambda*L) u = f.  ximgproc runs the sequential Thomas
 * elimination; SDR_FGS_THOMAS (the default since round 5) reproduces it operation for operation
 * (bit-exact with oracle/wls_oracle.c fgs_line), one lane per image line, the later passes'
 * elimination coefficients computed alongside the first.  SDR_FGS_PCR solves the same systems by
 * parallel cyclic reduction, a workgroup per line, with the diagonal carried as the row sum: it is
 * ~200x closer to the exact solution than the sequential sweep in float32, and on the reference's
 * own frames within 1 int16 level of it, but where the confidence map is sparse the sequential
 * sweep's own float error reaches hundreds of levels (profiles/r5_pcr_vs_thomas.json), so PCR is
 * not a drop-in there; lines of at most 4096 samples. */
enum { SDR_FGS_PCR = 0, SDR_FGS_THOMAS = 1 };

/* cv::ximgproc::createDisparityWLSFilter(matcher_left) (stereo_disparity.cpp:11): fills the
 * filter parameters for an SGBM left matcher AND mutates the matcher's parameters the way
 * ximgproc does (disp12MaxDiff = 1000000, speckleWindowSize = 0, uniquenessRatio = 0). */
void sdr_wls_params_for_sgbm(sdr_sgbm_params* left_matcher, sdr_wls_params* out);
int sdr_wls_create(const sdr_wls_params* p, int device, sdr_wls** out);
int sdr_wls_destroy(sdr_wls* h);
int sdr_wls_set_params(sdr_wls* h, const sdr_wls_params* p);
int sdr_wls_get_params(const sdr_wls* h, sdr_wls_params* p);
/* HIP stream the filter launches on (NULL = the HIP null stream); reset = its own stream */
int sdr_wls_set_stream(sdr_wls* h, void* stream);
int sdr_wls_reset_stream(sdr_wls* h);
void* sdr_wls_get_stream(const sdr_wls* h);
/* DisparityWLSFilter::getROI for a W x H map: roi = {x, y, w, h}. */
int sdr_wls_get_roi(const sdr_wls* h, int width, int height, int roi[4]);
/* DisparityWLSFilter::filter(disp_left, left_view, filtered, disp_right) on device, async on the
 * handle's stream: dense int16 maps [nframes][H][W], 8-bit gray guide (guide_stride bytes per
 * row, guide_frame_stride bytes per frame) -> filtered int16 [nframes][H][W].  d_conf
 * (nullable) receives getConfidenceMap() as float [nframes][H][W]. */
int sdr_wls_filter_device(sdr_wls* h, const int16_t* d_disp_left, const int16_t* d_disp_right,
                          const uint8_t* d_guide, int width, int height, size_t guide_stride,
                          size_t guide_frame_stride, int nframes, int16_t* d_out, float* d_conf);
/* Host-pointer version (synchronous). */
int sdr_wls_filter(sdr_wls* h, const int16_t* disp_left, const int16_t* disp_right,
                   const uint8_t* guide, int width, int height, size_t guide_stride,
                   int16_t* out, float* conf);
/* cv::ximgproc::fastGlobalSmootherFilter(guide, src, dst, lambda, sigma, attenuation, iters) on
 * nimg float images [nimg][h][w] sharing one 8-bit guide, in place, async on `stream`; solver
 * SDR_FGS_PCR or SDR_FGS_THOMAS.  SDR_FGS_THOMAS needs every pass's lambda * attenuation^k in
 * [0, 2^100] and allocates (stream-ordered per call, from the library's device memory pool)
 * 4 * (6 + 10 * num_iter) bytes a sample of
 * w x h rounded up to 4 each way: the coefficients of its 2 * num_iter passes (20 B a sample each)
 * and the pass layouts. */
int sdr_fgs_filter_device(const uint8_t* d_guide, size_t guide_stride, int width, int height,
                          double lambda, double sigma_color, double lambda_attenuation,
                          int num_iter, float* d_img, int nimg, int solver, void* stream);
/* Self-test of the reciprocal the SDR_FGS_THOMAS coefficient jobs use (v_rcp_f32 + one Newton
 * step, sdr_wls.hip fgs_rcp) against the IEEE quotient 1.0f / d, on the current device, for all
 * 2^23 mantissas of d in [2^e, 2^(e+1)), 0 <= e <= 126: *mismatches = how many differ (0 expected
 * for e <= 125, where 1/d is normal: the jobs' bit-exactness rests on it; SDR_FGS_THOMAS refuses
 * lambda > 2^100 so that its pivots stay below 2^126). Synchronous. */
int sdr_fgs_rcp_selftest(int e, unsigned int* mismatches);

/* ---- ingest in front of the path: StereoRectifier + SBS split ----
 * cv::initUndistortRectifyMap(K, dist, R, P, size, CV_16SC2, map1, map2)   stereo_rectifier.cpp:7-11
 * computed on the device (f64, OpenCV's scalar loop): map1 int16 [H][W][2], map2 uint16 [H][W]
 * (5-bit fractions, (v&31)*32 + (u&31)); host outputs.  dist has 0/4/5/8/12 coefficients; P is
 * row-major 3 x p_cols (p_cols 3 or 4, only the first 3 columns are used). */
int sdr_init_undistort_rectify_map(const double K[9], const double* dist, int ndist,
                                   const double R[9], const double* P, int p_cols, int width,
                                   int height, int device, int16_t* map1, uint16_t* map2);
/* cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0 on 8-bit images with 1 or
 * 3 channels, nframes frames (src/dst frame strides in bytes), async on `stream`. */
int sdr_remap_bilinear_device(const uint8_t* d_src, int src_width, int src_height,
                              size_t src_stride, size_t src_frame_stride, int channels,
                              const int16_t* d_map1, const uint16_t* d_map2, int width, int height,
                              uint8_t* d_dst, size_t dst_stride, size_t dst_frame_stride,
                              int nframes, void* stream);

typedef struct sdr_rectifier sdr_rectifier;
/* StereoRectifier(config) (stereo_rectifier.cpp:6-11): both eyes' maps built on `device`. */
int sdr_rectifier_create(const double K_left[9], const double* dist_left, int ndist_left,
                         const double R1[9], const double* P1, const double K_right[9],
                         const double* dist_right, int ndist_right, const double R2[9],
                         const double* P2, int p_cols, int width, int height, int device,
                         sdr_rectifier** out);
int sdr_rectifier_destroy(sdr_rectifier* h);
int sdr_rectifier_set_stream(sdr_rectifier* h, void* stream); /* NULL = the HIP null stream */
int sdr_rectifier_reset_stream(sdr_rectifier* h);                /* back to its own stream */
/* host copies of eye `which` (0 left, 1 right) maps */
int sdr_rectifier_get_maps(const sdr_rectifier* h, int which, int16_t* map1, uint16_t* map2);
/* StereoRectifier::rectify (stereo_rectifier.cpp:17-41) on device; either eye may be NULL. */
int sdr_rectify_device(sdr_rectifier* h, const uint8_t* d_left, const uint8_t* d_right,
                       size_t stride, size_t frame_stride, int channels, int nframes,
                       uint8_t* d_left_out, uint8_t* d_right_out, size_t out_stride,
                       size_t out_frame_stride);
/* Side-by-side BGR frames [nframes] of (2*width) x height (stereo_displayer.cpp:155-159): split +
 * rectify both eyes in one pass.  Outputs (each nullable, dense): rectified BGR [F][H][W][3] per
 * eye, and/or the class path's input BGR2GRAY + INTER_AREA 0.5x of the rectified eye
 * [F][H/2][W/2] (stereo_disparity.cpp:19-24), with OpenCV's intermediate u8 roundings. */
int sdr_rectify_sbs_device(sdr_rectifier* h, const uint8_t* d_sbs, size_t sbs_stride,
                           size_t sbs_frame_stride, int nframes, uint8_t* d_bgr_left,
                           uint8_t* d_bgr_right, uint8_t* d_small_left, uint8_t* d_small_right);

/* Class path from the half-size gray pair already on the device (after sdr_rectify_sbs_device),
 * async on the left matcher's stream: left/right matchers (+ WLS when wls != NULL) for nframes
 * dense [F][h][w] frames.  Outputs (device, dense): d_out float disparity in px (the value
 * computeDisparity returns), d_filtered int16 (nullable), d_conf float (nullable).  The right
 * matcher runs on a side stream owned by the left handle, forked from and joined back to the left
 * handle's stream with events (the call stays stream-ordered for the caller). */
int sdr_stereo_class_compute_device(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                                    const uint8_t* d_small_left, const uint8_t* d_small_right,
                                    int width, int height, int nframes, float* d_out,
                                    int16_t* d_filtered, float* d_conf);
/* The reference's per-frame pair computeDisparity -> computeDepth (stereo_displayer.cpp:161-162,
 * stereo_disparity.cpp:17-39,76-80) in one call: sdr_stereo_class_compute_device plus
 * reprojectImageTo3D(d_out, Q, handleMissing = false) -> d_xyz float32x3 [F][h][w][3], fused into
 * the WLS filter's last kernel when wls != NULL. */
int sdr_stereo_class_depth_device(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                                  const uint8_t* d_small_left, const uint8_t* d_small_right,
                                  int width, int height, int nframes, float* d_out,
                                  int16_t* d_filtered, float* d_conf, const double Q[16],
                                  float* d_xyz);

/* ---- point-cloud emit after the path, point_cloud/src/pcd_write.cpp ----
 * Points are pcl::PointXYZRGB as savePCDFileBinary lays them out: 16-byte records
 * {float x, y, z; uint32 rgba}. */
/* convertCVMatToPCL(xyz, left) (pcd_write.cpp:17-51): xyz float [F][H][W][3], bgr u8 3-channel
 * rows of bgr_stride bytes, frames bgr_frame_stride apart (0 = dense), or NULL -> organised cloud
 * [F][H*W]; non-finite points get NaN x/y/z.  Async on `stream`. */
int sdr_xyz_to_cloud_device(const float* d_xyz, const uint8_t* d_bgr, size_t bgr_stride,
                            size_t bgr_frame_stride, int width, int height, int nframes,
                            void* d_points, void* stream);
/* pcl::VoxelGrid<PointXYZRGB> with leaf (lx, ly, lz) (pcd_write.cpp:122-130) on n device points
 * -> d_out (capacity n) and *out_count.  PCL's int32-overflow case (leaf too small for the extent,
 * the reference's 5 mm leaf on millimetre clouds) copies the input through and sets *passthrough.
 * Synchronous on `stream` (the count is a host value).  Scratch: ~44 B a point plus the sort's
 * histograms, from a grow-only device arena a call leases and returns idle (one arena per call in
 * flight at once, kept for the process). */
int sdr_voxel_grid_device(const void* d_points, int n, float lx, float ly, float lz, void* d_out,
                          int* out_count, int* passthrough, void* stream);
/* pcl::io::savePCDFileBinary (pcd_write.cpp:141): header + width*height records (host memory).
 * sdr_pcd_header returns the header length (writing it to buf when buf != NULL). */
int sdr_pcd_header(int width, int height, char* buf, size_t cap);
int sdr_write_pcd_binary(const char* path, const void* points, int width, int height);

/* ---- display outputs: StereoDisparity::show_disparityMap / show_depthMap,
 * the live loop's JET overlay and StereoDisplayer::depth_coverage ----
 * Colour tables are 256 BGR triples (cv::applyColorMap's LUT); NULL = the built-in table of the
 * colormap the reference uses (TURBO for the depth map, JET for the overlay), generated from the
 * published colormap definitions by sdr_colormap_lut.  A display handle owns the EMA history
 * (prev_vis / prev_depth_vis of stereo_disparity.hpp:11) and a default range state. */
enum { SDR_COLORMAP_JET = 2, SDR_COLORMAP_TURBO = 20 }; /* cv::COLORMAP_* */
typedef struct sdr_display sdr_display;
int sdr_colormap_lut(int colormap, uint8_t* lut_bgr /* 768 bytes */);
int sdr_display_create(int device, sdr_display** out);
int sdr_display_destroy(sdr_display* h);
int sdr_display_set_stream(sdr_display* h, void* stream); /* NULL = the HIP null stream */
int sdr_display_reset_stream(sdr_display* h);              /* back to its own stream */
/* forget the EMA history and reset the handle's range state to {1000, 2000} */
int sdr_display_reset(sdr_display* h);
/* show_disparityMap (stereo_disparity.cpp:42-73) on nframes float disparities (px; `stride` and
 * `frame_stride` in ELEMENTS) -> d_vis u8 [F][H][W], frames in order through the EMA. */
int sdr_show_disparity_map_device(sdr_display* h, const float* d_disp, int width, int height,
                                  size_t stride, size_t frame_stride, int nframes,
                                  int num_disparities, uint8_t* d_vis);
/* show_depthMap (stereo_disparity.cpp:83-124) on computeDepth outputs (channels 3: Z is channel 2;
 * channels 1: Z itself), dense [F][H][W][channels] -> d_bgr u8 [F][H][W][3].  d_zrange: device
 * {zmin_smooth, zmax_smooth} (the reference's function-static doubles, shared by every caller
 * that passes the same pointer), NULL = the handle's own.  coverage_pct (host [F], nullable):
 * depth_coverage of each frame (stereo_displayer.cpp:105-118, columns >= 80); synchronises. */
int sdr_show_depth_map_device(sdr_display* h, const float* d_xyz, int width, int height,
                              int channels, int nframes, double* d_zrange, const uint8_t* lut_bgr,
                              uint8_t* d_bgr, double* coverage_pct);
/* StereoDisplayer::depth_coverage of xyz [F][H][W][3]: percent of Z in [0, 12000] among columns
 * >= col0 (80 in the reference), over all H*W pixels (host pct[F]; synchronous). */
int sdr_depth_coverage_device(sdr_display* h, const float* d_xyz, int width, int height,
                              int nframes, int col0, double* pct);
/* stereo_displayer.cpp:167-173: applyColorMap(vis, JET) -> d_heat (nullable) and
 * addWeighted(resize(left_rect, 0.5, INTER_AREA), 0.7, heat, 0.3, 0) -> d_overlay (nullable), from
 * the FULL-resolution rectified left BGR view (2*width x 2*height, left_stride bytes per row,
 * left_frame_stride bytes per frame, 0 = dense); vis/heat/overlay are [F][H][W](x3). */
int sdr_disparity_overlay_device(sdr_display* h, const uint8_t* d_vis, const uint8_t* d_left_bgr,
                                 size_t left_stride, size_t left_frame_stride, int width,
                                 int height, int nframes, const uint8_t* lut_bgr, uint8_t* d_heat,
                                 uint8_t* d_overlay);
/* Host-pointer versions (synchronous; `stride` in elements, out_stride in bytes).  zrange: host
 * {zmin_smooth, zmax_smooth} in/out, NULL = the handle's own state. */
int sdr_show_disparity_map(sdr_display* h, const float* disp, int width, int height, size_t stride,
                           int num_disparities, uint8_t* out, size_t out_stride);
int sdr_show_depth_map(sdr_display* h, const float* xyz, int width, int height, int channels,
                       double* zrange, uint8_t* out_bgr, double* coverage_pct);
int sdr_disparity_overlay(sdr_display* h, const uint8_t* vis, const uint8_t* left_bgr,
                          size_t left_stride, int width, int height, uint8_t* heat,
                          uint8_t* overlay);
/* StereoDisplayer::depth_coverage of a host xyz map [H][W][3] (synchronous); read-only like the
 * reference's: the handle's EMA history and range state are untouched. */
int sdr_depth_coverage(sdr_display* h, const float* xyz, int width, int height, int col0, double* pct);

/* Bytes of device scratch the handle holds for the given frame shape (for capacity planning);
 * 0 when compute would refuse the shape or parameters.  sdr_sgbm_scratch_bytes is the CV_8UC1
 * figure, sdr_sgbm_scratch_bytes_cn takes the channel count (1 or 3: colour input holds three
 * operand sets per image). */
size_t sdr_sgbm_scratch_bytes(const sdr_sgbm_params* p, int width, int height, int nframes);
size_t sdr_sgbm_scratch_bytes_cn(const sdr_sgbm_params* p, int width, int height, int channels,
                                 int nframes);

/* Timing with HIP events on the handle's stream.  level 1: per-stage timing of the last compute
 * (sdr_sgbm_last_timing: cost volume / path aggregation / LR+median+speckle, ms).  level 2 also
 * brackets every kernel launch; sdr_sgbm_kernel_time sums the launches of one SDR_KERNEL_* kind
 * (kind < 0: all) since the last reset. */
enum {
    SDR_KERNEL_PREFILTER = 0, SDR_KERNEL_COST = 1, SDR_KERNEL_PATHS = 2,
    SDR_KERNEL_WTA_LR = 3,   /* k_south_wta: top-to-bottom path fused with WTA/uniqueness/disp2 */
    SDR_KERNEL_MEDIAN = 4, SDR_KERNEL_SPECKLE = 5, SDR_KERNEL_REPROJECT = 6,
    SDR_KERNEL_LR_CHECK = 7, /* the LR-checked map materialised (debug stage 2 only since round 3) */
    SDR_KERNEL_SWEEP = 8,    /* k_sweep: batched MODE_HH's up pass (N, NE, NW) */
    /* the class path's WLS filter (sdr_stereo_class_*), recorded on the left matcher's handle */
    SDR_KERNEL_WLS_PREP = 9, /* k_wls_prep (or k_wls_disc + k_wls_conf past 4096 ROI columns) */
    SDR_KERNEL_FGS = 10,     /* one FGS pass: k_fgs_pcr, or k_fgs_th (SDR_FGS_THOMAS) */
    SDR_KERNEL_WLS_FINAL = 11, /* k_wls_final (+ /16 + computeDepth epilogue) */
    SDR_KERNEL_SWEEP_DOWN = 12, /* batched MODE_HH's down pass (SE, SW): timed apart from the up pass */
    SDR_KERNEL_FGS_COEF = 13 /* SDR_FGS_THOMAS: the coefficient jobs of a filter's passes (one launch) */
};
int sdr_sgbm_enable_timing(sdr_sgbm* h, int level);
int sdr_sgbm_last_timing(const sdr_sgbm* h, float* cost_ms, float* paths_ms, float* post_ms);
int sdr_sgbm_kernel_time(sdr_sgbm* h, int kind, int reset, float* total_ms, int* count);

/* Status of the handle's device batches since the last report (synchronises the handle's
 * stream).  A batched MODE_HH call (>= 8 frames, sdr_sgbm_compute_device*) runs row sweeps whose
 * workgroups wait on their neighbours; they assume every workgroup of the sweep is resident, i.e.
 * that this process has the device to itself (sweeps of one process are ordered among themselves).
 * If a wait still gives up (another process's persistent kernel holding CUs for about a second),
 * that batch's output frames are written as INVALID ((minDisparity-1)*16, the reprojection's
 * frame minima too) and SDR_ERR_DEVICE is returned once for the timeouts seen since the last
 * report -- by this call, or by the next compute call if it sees them first -- then SDR_OK again
 * (the device keeps a count, so copies of it still in flight cannot report a timeout twice).  The
 * host-pointer entry points compute one frame and never take the sweeps. */
int sdr_sgbm_last_status(sdr_sgbm* h);
/* Test hooks.  SDR_DEBUG_SWEEP_SPIN: polls a sweep's neighbour wait makes before it gives up
 * (<= 0: the default, about a second); a small value forces the failure path above. */
enum { SDR_DEBUG_SWEEP_SPIN = 1 };
int sdr_sgbm_debug_knob(sdr_sgbm* h, int knob, int value);

/* Device self-test of the cross-lane primitives the kernels rely on (DPP wave shifts,
 * permlane swaps); fills 4 failure counters, all zero on a healthy gfx950. */
int sdr_selftest_wave_ops(int* failures4);

/* The device's streaming rate: `iters` back-to-back copies of a `bytes` buffer, the fastest of
 * several access shapes (16-byte loads, 4 or 8 in flight per thread, plain or non-temporal
 * stores, 2-16 workgroups a CU), read + write bytes per second in GB/s.  bench.py records it
 * beside the dominant kernel's rate (box-to-box spread).  _ex fills gbs3 = {copy, read-only,
 * write-only}. */
int sdr_stream_probe(int device, size_t bytes, int iters, double* gbs);
int sdr_stream_probe_ex(int device, size_t bytes, int iters, double* gbs3);

/* Diagnostics: synchronously copy an internal buffer of the last compute to host memory.
 * stage 0 = cost volume C [F][H][W1][D] s16, 1 = WTA disparity before the LR check [F][H][W] s16,
 * 2 = after the LR check (computed from stages 1 and 5 on request: the pipeline's median computes
 * it per tile and never writes it), 3 = final (median + speckle), 4 = path costs L
 * [P-1][F][H][W1][D] s16 (every direction but top-to-bottom, whose L is consumed on chip by the
 * fused WTA pass), 5 = the right view's WTA keys [F][H][W] u32: (minS << 16 | 0xffff - x) of the
 * winning left pixel x (matched column) per right-view column, 0xffffffff where none (not built
 * when the LR check cannot fire), 6 = MODE_SGBM_3WAY's stripe-start cost rows [F][stripes][rows][W1][D]
 * s16 (rows = the largest stripe's count); stage 1 holds values only in the matched columns. */
int sdr_sgbm_debug_stage(const sdr_sgbm* h, int stage, void* host_dst, size_t bytes);

/* Page-locked host memory (the role of cv::cuda::HostMem): host buffers from sdr_host_alloc that
 * are passed to the host-pointer entry points are copied to and from by DMA directly, without
 * the staging copy pageable memory needs. */
int sdr_host_alloc(size_t bytes, void** out);
int sdr_host_free(void* p);

const char* sdr_last_error(void);
int sdr_abi_version(void);
/* Hash of the sources the library was built from (stereo_depth_ruler_amd/build.py source_hash):
 * the build and the smoke test compare it with the tree's sources. */
const char* sdr_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
