// stereo.hpp -- header-only C++ facade over the C ABI (sdr.h) with the reference's C++ surface:
//
//   sdr::StereoSGBM::create(...) / compute(L, R, disp)      <- cv::StereoSGBM
//       reference stereo_vision/src/stereo_disparity.cpp:5-9,27-28, point_cloud/src/pcd_write.cpp:102-111
//   sdr::reprojectImageTo3D(disp, xyz, Q, handleMissing)    <- cv::reprojectImageTo3D
//       stereo_disparity.cpp:78, pcd_write.cpp:116
//   sdr::ximgproc::createRightMatcher(left)                 <- cv::ximgproc::createRightMatcher
//   sdr::ximgproc::createDisparityWLSFilter(left)           <- cv::ximgproc::createDisparityWLSFilter
//       stereo_disparity.cpp:10-13,31,36
//   sdr::StereoDisparity                                     <- class StereoDisparity
//       stereo_vision/include/stereo_disparity.hpp:8-24
//   sdr::Display                                             <- show_disparityMap / show_depthMap,
//       the displayer's JET overlay and depth_coverage (stereo_displayer.cpp:105-118,164-173)
//
// sdr::Mat is a minimal owning image (rows, cols, OpenCV type code, row step) so that callers
// can switch from cv::Mat without OpenCV present; when OpenCV is available, wrap cv::Mat data
// pointers with sdr::Mat::view(...) at zero cost.  Errors throw sdr::Exception (cf. cv::Exception).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "sdr.h"

namespace sdr {

enum { CV_8UC1 = 0, CV_16SC1 = 3, CV_32FC1 = 5, CV_64FC1 = 6, CV_8UC3 = 16, CV_32FC3 = 21 };

inline size_t elem_size(int type) {
    switch (type) {
    case CV_8UC1: return 1;
    case CV_16SC1: return 2;
    case CV_32FC1: return 4;
    case CV_64FC1: return 8;
    case CV_8UC3: return 3;
    case CV_32FC3: return 12;
    default: throw std::invalid_argument("sdr::Mat: unsupported type");
    }
}

class Exception : public std::runtime_error {
public:
    Exception(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
    int code;
};

inline void check(int rc) {
    if (rc != SDR_OK) throw Exception(rc, sdr_last_error());
}

namespace detail {
// Page-locked blocks are expensive to allocate (the driver pins every page), and the reference's
// calls return fresh Mats per frame (StereoDisparity::computeDisparity, computeDepth): released
// blocks are kept here and handed to the next allocation of a similar size (best fit within 2x),
// up to kPinPoolBytes, so a per-frame Mat costs no pinning after the first frames.  The pool is
// never destroyed (Mats may outlive static destruction); the process exit releases its blocks.
struct PinPool {
    static constexpr size_t kPinPoolBytes = (size_t)512 << 20;
    std::mutex mu;
    std::multimap<size_t, void*> free_;
    size_t held = 0;
    void* get(size_t n, size_t* got) {
        {
            std::lock_guard<std::mutex> lk(mu);
            auto it = free_.lower_bound(n);
            if (it != free_.end() && it->first <= 2 * n) {
                void* p = it->second;
                *got = it->first;
                held -= it->first;
                free_.erase(it);
                return p;
            }
        }
        void* p = nullptr;
        if (sdr_host_alloc(n, &p) != SDR_OK) return nullptr;
        *got = n;
        return p;
    }
    void put(void* p, size_t n) {
        std::lock_guard<std::mutex> lk(mu);
        free_.emplace(n, p);
        held += n;
        while (held > kPinPoolBytes && !free_.empty()) {  // evict the largest blocks first
            auto it = std::prev(free_.end());
            held -= it->first;
            sdr_host_free(it->second);
            free_.erase(it);
        }
    }
};
inline PinPool& pin_pool() {
    static PinPool* pool = new PinPool();
    return *pool;
}
// a page-locked block of at least n bytes (nullptr if page-locked memory is unavailable)
inline std::shared_ptr<void> pinned_block(size_t n) {
    size_t got = 0;
    void* p = pin_pool().get(n, &got);
    if (!p) return nullptr;
    return std::shared_ptr<void>(p, [got](void* q) { pin_pool().put(q, got); });
}
}  // namespace detail

class Mat {
public:
    int rows = 0, cols = 0, type = CV_8UC1;
    size_t step = 0;  // bytes per row
    uint8_t* data = nullptr;

    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    static Mat view(int r, int c, int t, void* p, size_t step_bytes = 0) {
        Mat m;
        m.rows = r; m.cols = c; m.type = t;
        m.step = step_bytes ? step_bytes : (size_t)c * elem_size(t);
        m.data = (uint8_t*)p;
        return m;
    }
    // like cv::Mat::create: reallocates only when the shape or type changes.  The storage is
    // page-locked (sdr_host_alloc), so the engine's host-pointer calls DMA straight to and from
    // every Mat the facade allocates -- compute()'s disparity, reprojectImageTo3D's xyz,
    // computeDisparity's output -- with no staging copy; where page-locked memory is unavailable
    // (no HIP device) it falls back to ordinary memory, which the engine stages.
    void create(int r, int c, int t) {
        if (data && r == rows && c == cols && t == type) return;
        alloc(r, c, t, true);
    }
    // explicit page-locked storage (cv::cuda::HostMem(PAGE_LOCKED).createMatHeader()); throws if
    // it cannot be had
    static Mat page_locked(int r, int c, int t) {
        Mat m;
        m.rows = r; m.cols = c; m.type = t;
        m.step = (size_t)c * elem_size(t);
        auto b = detail::pinned_block(std::max<size_t>((size_t)r * m.step, 1));
        if (!b) throw Exception(SDR_ERR_NOMEM, std::string("page-locked allocation failed: ") + sdr_last_error());
        m.store_ = b;
        m.data = (uint8_t*)b.get();
        return m;
    }
    // ordinary (pageable) storage
    static Mat pageable(int r, int c, int t) {
        Mat m;
        m.alloc(r, c, t, false);
        return m;
    }
    bool empty() const { return !data || rows == 0 || cols == 0; }
    template <typename T> T* ptr(int y) { return (T*)(data + (size_t)y * step); }
    template <typename T> const T* ptr(int y) const { return (const T*)(data + (size_t)y * step); }
    template <typename T> T& at(int y, int x) { return ptr<T>(y)[x]; }
    Mat clone() const {
        Mat m(rows, cols, type);
        for (int y = 0; y < rows; y++) std::memcpy(m.ptr<uint8_t>(y), ptr<uint8_t>(y), (size_t)cols * elem_size(type));
        return m;
    }

private:
    void alloc(int r, int c, int t, bool pinned) {
        rows = r; cols = c; type = t;
        step = (size_t)c * elem_size(t);
        const size_t bytes = std::max<size_t>((size_t)r * step, 1);
        if (pinned) {
            if (auto b = detail::pinned_block(bytes)) {
                store_ = b;
                data = (uint8_t*)b.get();
                return;
            }
        }
        auto v = std::make_shared<std::vector<uint8_t>>(bytes);
        data = v->data();
        store_ = v;
    }
    std::shared_ptr<void> store_;
};

template <class T> using Ptr = std::shared_ptr<T>;

// Q (4x4, CV_64F or CV_32F) as 16 doubles
inline void q_of(const Mat& Q, double q[16]) {
    if (Q.rows != 4 || Q.cols != 4) throw Exception(SDR_ERR_ARG, "Q must be 4x4");
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            q[i * 4 + j] = Q.type == CV_64FC1 ? Q.ptr<double>(i)[j] : (double)Q.ptr<float>(i)[j];
}

class StereoSGBM {
public:
    enum { MODE_SGBM = SDR_MODE_SGBM, MODE_HH = SDR_MODE_HH, MODE_SGBM_3WAY = SDR_MODE_SGBM_3WAY,
           MODE_HH4 = SDR_MODE_HH4 };

    static Ptr<StereoSGBM> create(int minDisparity = 0, int numDisparities = 16, int blockSize = 3,
                                  int P1 = 0, int P2 = 0, int disp12MaxDiff = 0, int preFilterCap = 0,
                                  int uniquenessRatio = 0, int speckleWindowSize = 0,
                                  int speckleRange = 0, int mode = MODE_SGBM, int device = 0) {
        sdr_sgbm_params p;
        sdr_sgbm_params_default(&p);
        p.minDisparity = minDisparity; p.numDisparities = numDisparities; p.blockSize = blockSize;
        p.P1 = P1; p.P2 = P2; p.disp12MaxDiff = disp12MaxDiff; p.preFilterCap = preFilterCap;
        p.uniquenessRatio = uniquenessRatio; p.speckleWindowSize = speckleWindowSize;
        p.speckleRange = speckleRange; p.mode = mode;
        return Ptr<StereoSGBM>(new StereoSGBM(p, device));
    }
    static Ptr<StereoSGBM> create(const sdr_sgbm_params& p, int device = 0) {
        return Ptr<StereoSGBM>(new StereoSGBM(p, device));
    }
    ~StereoSGBM() { sdr_sgbm_destroy(h_); }
    StereoSGBM(const StereoSGBM&) = delete;
    StereoSGBM& operator=(const StereoSGBM&) = delete;

    // StereoMatcher::compute: CV_8UC1 or CV_8UC3 pair -> CV_16SC1 disparity (1/16 px); disp is
    // (re)allocated
    void compute(const Mat& left, const Mat& right, Mat& disparity) {
        if (left.rows != right.rows || left.cols != right.cols || left.type != right.type)
            throw Exception(SDR_ERR_ARG, "left and right images must have the same size and type");
        if ((left.type != CV_8UC1 && left.type != CV_8UC3) || left.step != right.step)
            throw Exception(SDR_ERR_TYPE, "8-bit 1- or 3-channel images with equal steps are required");
        disparity.create(left.rows, left.cols, CV_16SC1);
        check(sdr_sgbm_compute(h_, left.data, right.data, left.cols, left.rows,
                               left.type == CV_8UC3 ? 3 : 1, left.step, (int16_t*)disparity.data,
                               disparity.step / 2));
    }

    // compute -> convertTo(CV_32F, 1/16) -> reprojectImageTo3D(Q, handleMissingValues) in one call
    // (pcd_write.cpp:111-116), the float disparity kept on the device; xyz CV_32FC3
    void computeReproject(const Mat& left, const Mat& right, const Mat& Q, bool handleMissingValues,
                          Mat& disparity, Mat& xyz) {
        if (left.rows != right.rows || left.cols != right.cols || left.type != right.type)
            throw Exception(SDR_ERR_ARG, "left and right images must have the same size and type");
        if (left.type != CV_8UC1 || left.step != right.step)
            throw Exception(SDR_ERR_TYPE, "8-bit single-channel images with equal steps are required");
        double q[16];
        q_of(Q, q);
        disparity.create(left.rows, left.cols, CV_16SC1);
        xyz.create(left.rows, left.cols, CV_32FC3);
        check(sdr_sgbm_compute_reproject(h_, left.data, right.data, left.cols, left.rows, left.step,
                                         (int16_t*)disparity.data, disparity.step / 2, q,
                                         handleMissingValues ? 1 : 0, (float*)xyz.data, xyz.step / 4));
    }

    int getMinDisparity() const { return p_.minDisparity; }
    void setMinDisparity(int v) { p_.minDisparity = v; push(); }
    int getNumDisparities() const { return p_.numDisparities; }
    void setNumDisparities(int v) { p_.numDisparities = v; push(); }
    int getBlockSize() const { return p_.blockSize; }
    void setBlockSize(int v) { p_.blockSize = v; push(); }
    int getP1() const { return p_.P1; }
    void setP1(int v) { p_.P1 = v; push(); }
    int getP2() const { return p_.P2; }
    void setP2(int v) { p_.P2 = v; push(); }
    int getDisp12MaxDiff() const { return p_.disp12MaxDiff; }
    void setDisp12MaxDiff(int v) { p_.disp12MaxDiff = v; push(); }
    int getPreFilterCap() const { return p_.preFilterCap; }
    void setPreFilterCap(int v) { p_.preFilterCap = v; push(); }
    int getUniquenessRatio() const { return p_.uniquenessRatio; }
    void setUniquenessRatio(int v) { p_.uniquenessRatio = v; push(); }
    int getSpeckleWindowSize() const { return p_.speckleWindowSize; }
    void setSpeckleWindowSize(int v) { p_.speckleWindowSize = v; push(); }
    int getSpeckleRange() const { return p_.speckleRange; }
    void setSpeckleRange(int v) { p_.speckleRange = v; push(); }
    int getMode() const { return p_.mode; }
    void setMode(int v) { p_.mode = v; push(); }

    const sdr_sgbm_params& params() const { return p_; }
    sdr_sgbm* handle() const { return h_; }
    int device() const { return dev_; }

private:
    StereoSGBM(const sdr_sgbm_params& p, int device) : p_(p), dev_(device) {
        check(sdr_sgbm_create(&p_, device, &h_));
    }
    void push() { check(sdr_sgbm_set_params(h_, &p_)); }
    sdr_sgbm_params p_;
    sdr_sgbm* h_ = nullptr;
    int dev_ = 0;
};

// cv::reprojectImageTo3D(disparity CV_32F or CV_16S, _3dImage CV_32FC3, Q 4x4, handleMissing)
// convertTo: disp.convertTo(f, CV_32F, 1/16) as the reference does before reprojecting
inline void convertTo32F(const Mat& disp16, Mat& f, double scale) {
    if (disp16.type != CV_16SC1) throw Exception(SDR_ERR_TYPE, "convertTo32F expects CV_16S");
    f.create(disp16.rows, disp16.cols, CV_32FC1);
    const float a = (float)scale;
    for (int y = 0; y < disp16.rows; y++) {  // a plain loop per row: the compiler vectorises it
        const int16_t* __restrict__ s = disp16.ptr<int16_t>(y);
        float* __restrict__ d = f.ptr<float>(y);
        for (int x = 0; x < disp16.cols; x++) d[x] = (float)s[x] * a;
    }
}

inline void reprojectImageTo3D(const Mat& disparity, Mat& xyz, const Mat& Q,
                               bool handleMissingValues = false) {
    double q[16];
    q_of(Q, q);
    Mat f = disparity;
    if (disparity.type == CV_16SC1) {  // OpenCV reads CV_16S values as-is (no 1/16 scaling)
        f = Mat::pageable(disparity.rows, disparity.cols, CV_32FC1);
        for (int y = 0; y < disparity.rows; y++)
            for (int x = 0; x < disparity.cols; x++) f.ptr<float>(y)[x] = (float)disparity.ptr<int16_t>(y)[x];
    } else if (disparity.type != CV_32FC1) {
        throw Exception(SDR_ERR_TYPE, "disparity must be CV_32F or CV_16S");
    }
    xyz.create(disparity.rows, disparity.cols, CV_32FC3);
    check(sdr_reproject(f.ptr<float>(0), f.cols, f.rows, f.step / 4, q, handleMissingValues ? 1 : 0,
                        xyz.ptr<float>(0), xyz.step / 4));
}

namespace ximgproc {
// cv::ximgproc::createRightMatcher(matcher_left)
inline Ptr<StereoSGBM> createRightMatcher(const Ptr<StereoSGBM>& left) {
    sdr_sgbm_params r;
    sdr_right_matcher_params(&left->params(), &r);
    return StereoSGBM::create(r, left->device());
}

// cv::ximgproc::DisparityWLSFilter (stereo_disparity.cpp:11-13,31,36)
class DisparityWLSFilter {
public:
    DisparityWLSFilter(const sdr_wls_params& p, int device) : p_(p) { check(sdr_wls_create(&p_, device, &h_)); }
    ~DisparityWLSFilter() { sdr_wls_destroy(h_); }
    DisparityWLSFilter(const DisparityWLSFilter&) = delete;
    DisparityWLSFilter& operator=(const DisparityWLSFilter&) = delete;

    double getLambda() const { return p_.lambda; }
    void setLambda(double v) { p_.lambda = v; push(); }
    double getSigmaColor() const { return p_.sigma_color; }
    void setSigmaColor(double v) { p_.sigma_color = v; push(); }
    int getLRCthresh() const { return p_.lrc_thresh; }
    void setLRCthresh(int v) { p_.lrc_thresh = v; push(); }
    int getDepthDiscontinuityRadius() const { return p_.depth_discontinuity_radius; }
    void setDepthDiscontinuityRadius(int v) { p_.depth_discontinuity_radius = v; push(); }
    // engine extension: FGS line solver, SDR_FGS_THOMAS (default) or SDR_FGS_PCR (sdr.h)
    int getFgsSolver() const { return p_.fgs_solver; }
    void setFgsSolver(int v) { p_.fgs_solver = v; push(); }

    // filter(disparity_map_left CV_16S, left_view CV_8UC1, filtered CV_16S, disparity_map_right CV_16S)
    void filter(const Mat& dl, const Mat& left_view, Mat& filtered, const Mat& dr) {
        if (dl.type != CV_16SC1 || dr.type != CV_16SC1 || dl.rows != dr.rows || dl.cols != dr.cols)
            throw Exception(SDR_ERR_TYPE, "disparity maps must be CV_16S of equal size");
        if (left_view.type != CV_8UC1 || left_view.rows != dl.rows || left_view.cols != dl.cols)
            throw Exception(SDR_ERR_TYPE, "left_view must be CV_8UC1 of the disparity map's size");
        if (dl.step != (size_t)dl.cols * 2 || dr.step != (size_t)dr.cols * 2)
            throw Exception(SDR_ERR_ARG, "disparity maps must be continuous");
        filtered.create(dl.rows, dl.cols, CV_16SC1);
        conf_.create(dl.rows, dl.cols, CV_32FC1);
        check(sdr_wls_filter(h_, dl.ptr<int16_t>(0), dr.ptr<int16_t>(0), left_view.data, dl.cols,
                             dl.rows, left_view.step, filtered.ptr<int16_t>(0), conf_.ptr<float>(0)));
    }
    Mat getConfidenceMap() const { return conf_; }
    sdr_wls* handle() const { return h_; }

private:
    void push() { check(sdr_wls_set_params(h_, &p_)); }
    sdr_wls_params p_;
    sdr_wls* h_ = nullptr;
    Mat conf_;
};

// cv::ximgproc::createDisparityWLSFilter(matcher_left): also switches the left matcher to
// disp12MaxDiff = 1e6, speckleWindowSize = 0, uniquenessRatio = 0, as ximgproc does
inline Ptr<DisparityWLSFilter> createDisparityWLSFilter(const Ptr<StereoSGBM>& left) {
    sdr_sgbm_params m = left->params();
    sdr_wls_params p;
    sdr_wls_params_for_sgbm(&m, &p);
    left->setDisp12MaxDiff(m.disp12MaxDiff);
    left->setSpeckleWindowSize(m.speckleWindowSize);
    left->setUniquenessRatio(m.uniquenessRatio);
    return Ptr<DisparityWLSFilter>(new DisparityWLSFilter(p, left->device()));
}
}  // namespace ximgproc

// Display outputs on the engine: the EMA history of one StereoDisparity
// (prev_vis / prev_depth_vis, stereo_disparity.hpp:11), show_disparityMap / show_depthMap, the live
// loop's JET overlay and StereoDisplayer::depth_coverage (stereo_displayer.cpp:105-118,167-173).
class Display {
public:
    explicit Display(int device = 0) { check(sdr_display_create(device, &h_)); }
    ~Display() { sdr_display_destroy(h_); }
    Display(const Display&) = delete;
    Display& operator=(const Display&) = delete;

    // CV_32F disparity (px) -> CV_8UC1
    Mat show_disparityMap(const Mat& disparity, int numDisparities) {
        if (disparity.type != CV_32FC1) throw Exception(SDR_ERR_TYPE, "show_disparityMap expects CV_32F");
        Mat out(disparity.rows, disparity.cols, CV_8UC1);
        check(sdr_show_disparity_map(h_, disparity.ptr<float>(0), disparity.cols, disparity.rows,
                                     disparity.step / 4, numDisparities, out.data, out.step));
        return out;
    }
    // CV_32FC3 depth (Z = channel 2) or CV_32F Z -> CV_8UC3 (TURBO); zrange = {zmin, zmax} state
    Mat show_depthMap(const Mat& depth, double* zrange, double* coverage_pct = nullptr) {
        if (depth.type != CV_32FC3 && depth.type != CV_32FC1)
            throw Exception(SDR_ERR_TYPE, "show_depthMap expects CV_32FC3 or CV_32F");
        const int ch = depth.type == CV_32FC3 ? 3 : 1;
        if (depth.step != (size_t)depth.cols * 4 * ch) throw Exception(SDR_ERR_ARG, "depth must be continuous");
        Mat out(depth.rows, depth.cols, CV_8UC3);
        check(sdr_show_depth_map(h_, depth.ptr<float>(0), depth.cols, depth.rows, ch, zrange, out.data,
                                 coverage_pct));
        return out;
    }
    // applyColorMap(vis, JET) + addWeighted(resize(left_rect, 0.5, INTER_AREA), 0.7, heat, 0.3, 0)
    Mat overlay(const Mat& vis, const Mat& left_rect) {
        if (vis.type != CV_8UC1 || left_rect.type != CV_8UC3 || left_rect.rows != 2 * vis.rows ||
            left_rect.cols != 2 * vis.cols || vis.step != (size_t)vis.cols)
            throw Exception(SDR_ERR_TYPE, "overlay expects CV_8UC1 vis and a CV_8UC3 left view of twice its size");
        Mat out(vis.rows, vis.cols, CV_8UC3);
        check(sdr_disparity_overlay(h_, vis.data, left_rect.data, left_rect.step, vis.cols, vis.rows,
                                    nullptr, out.data));
        return out;
    }
    // StereoDisplayer::depth_coverage(depth_map): percent of Z in [0, 12000] in columns >= 80;
    // read-only (this Display's show_depthMap history is untouched)
    double depth_coverage(const Mat& depth) {
        if (depth.type != CV_32FC3 || depth.step != (size_t)depth.cols * 12)
            throw Exception(SDR_ERR_TYPE, "depth_coverage expects a continuous CV_32FC3 map");
        double pct = 0;
        check(sdr_depth_coverage(h_, depth.ptr<float>(0), depth.cols, depth.rows, 80, &pct));
        return pct;
    }
    sdr_display* handle() const { return h_; }

private:
    sdr_display* h_ = nullptr;
};

// class StereoDisparity (reference stereo_vision/include/stereo_disparity.hpp:8-24)
class StereoDisparity {
public:
    explicit StereoDisparity(const Mat& Q_matrix, int device = 0) : Q(Q_matrix.clone()) {
        // stereo_disparity.cpp:5-9: StereoSGBM::create(0, 80, 5, 8*5*5*3, 32*5*5*3, 1, 63, 12, 200, 2, 3WAY)
        matcher = StereoSGBM::create(0, 80, 5, 8 * 5 * 5 * 3, 32 * 5 * 5 * 3, 1, 63, 12, 200, 2,
                                     StereoSGBM::MODE_SGBM_3WAY, device);
        right_matcher = ximgproc::createRightMatcher(matcher);          // :10
        wls_filter = ximgproc::createDisparityWLSFilter(matcher);       // :11
        wls_filter->setLambda(8000.0);                                   // :12
        wls_filter->setSigmaColor(1.1);                                  // :13
    }
    // BGR 8UC3 rectified pair (full res) -> CV_32F disparity in px at half resolution
    Mat computeDisparity(const Mat& left, const Mat& right) {
        if (left.type != CV_8UC3 || right.type != CV_8UC3 || left.rows != right.rows ||
            left.cols != right.cols || left.step != right.step)
            throw Exception(SDR_ERR_TYPE, "computeDisparity expects two equal-size BGR images");
        Mat out(left.rows / 2, left.cols / 2, CV_32FC1);
        conf_map.create(left.rows / 2, left.cols / 2, CV_32FC1);
        check(sdr_stereo_class_compute(matcher->handle(), right_matcher->handle(),
                                       wls_filter->handle(), left.data, right.data, left.cols,
                                       left.rows, left.step, out.ptr<float>(0), out.step / 4,
                                       nullptr, nullptr, nullptr, conf_map.ptr<float>(0)));
        return out;
    }
    Mat computeDepth(const Mat& disparity) {  // stereo_disparity.cpp:76-80 (handleMissing=false)
        Mat depth;
        reprojectImageTo3D(disparity, depth, Q);
        return depth;
    }
    const Ptr<StereoSGBM> get_matcher() const { return matcher; }
    const Mat& getConfidenceMap() const { return conf_map; }  // wls_filter->getConfidenceMap() (:36)

    // stereo_disparity.cpp:42-73: gamma map with the EMA against this object's previous frame
    Mat show_disparityMap(const Mat& disparity) {
        return display().show_disparityMap(disparity, matcher->getNumDisparities());
    }
    // stereo_disparity.cpp:83-124: the range state is function-static in the reference, i.e. one
    // pair of doubles for every StereoDisparity of the process; so it is here
    Mat show_depthMap(const Mat& depth) {
        static double zrange[2] = {1000.0, 2000.0};
        return display().show_depthMap(depth, zrange);
    }

private:
    Display& display() {
        if (!display_) display_ = std::make_shared<Display>(matcher->device());
        return *display_;
    }
    Ptr<StereoSGBM> matcher, right_matcher;
    Ptr<ximgproc::DisparityWLSFilter> wls_filter;
    Mat Q, conf_map;
    Ptr<Display> display_;
};

}  // namespace sdr
