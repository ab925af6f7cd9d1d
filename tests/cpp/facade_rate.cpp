// facade_rate.cpp -- the reference's two host-memory call patterns through the C++ facade
// (include/sdr/stereo.hpp), timed frame by frame, and their outputs written for the parity test
// (tests/test_gpu_facade_rate.py) to compare with the oracle.
//
//   pcd      point_cloud/src/pcd_write.cpp:102-116 call for call: sgbm->compute(L, R, disp) ->
//            disp.convertTo(disp_f, CV_32F, 1/16) -> reprojectImageTo3D(disp_f, xyz, Q, true),
//            on 1280x720 gray pairs with the C2 parameters (d = 128, MODE_SGBM), outputs in
//            facade-allocated Mats (page-locked by Mat::create), inputs plain host memory (the
//            role of the cv::Mat cvtColor hands the reference)
//   class    stereo_vision/src/stereo_displayer.cpp:161-162: StereoDisparity::computeDisparity(
//            left BGR, right BGR) -> computeDepth(disparity), fresh Mats per frame as the reference
//            returns them
//
// usage: facade_rate <dir> <frames>; <dir> holds l.bin, r.bin (uint8 H x W gray), bl.bin, br.bin
// (uint8 H x W x 3 BGR) for W = 1280, H = 720 and q.bin (Q, 16 doubles); prints one JSON line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "sdr/stereo.hpp"

static std::vector<uint8_t> read_file(const std::string& p, size_t n) {
    std::vector<uint8_t> v(n);
    std::ifstream f(p, std::ios::binary);
    f.read((char*)v.data(), (std::streamsize)n);
    if (!f) {
        std::fprintf(stderr, "cannot read %s\n", p.c_str());
        std::exit(2);
    }
    return v;
}

static void write_mat(const std::string& p, const sdr::Mat& m) {
    std::ofstream f(p, std::ios::binary);
    for (int y = 0; y < m.rows; y++) f.write((const char*)m.ptr<uint8_t>(y), (std::streamsize)(m.cols * sdr::elem_size(m.type)));
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string dir = argv[1];
    const int frames = std::atoi(argv[2]);
    const int W = 1280, H = 720;
    std::vector<uint8_t> l = read_file(dir + "/l.bin", (size_t)W * H), r = read_file(dir + "/r.bin", (size_t)W * H);
    std::vector<uint8_t> bl = read_file(dir + "/bl.bin", (size_t)W * H * 3), br = read_file(dir + "/br.bin", (size_t)W * H * 3);
    const sdr::Mat L = sdr::Mat::view(H, W, sdr::CV_8UC1, l.data()), R = sdr::Mat::view(H, W, sdr::CV_8UC1, r.data());
    const sdr::Mat BL = sdr::Mat::view(H, W, sdr::CV_8UC3, bl.data()), BR = sdr::Mat::view(H, W, sdr::CV_8UC3, br.data());
    // Q (config/stereo.yaml, 16 doubles in q.bin)
    std::vector<uint8_t> qb = read_file(dir + "/q.bin", 16 * sizeof(double));
    sdr::Mat Q = sdr::Mat::pageable(4, 4, sdr::CV_64FC1);
    std::memcpy(Q.data, qb.data(), 16 * sizeof(double));

    auto sgbm = sdr::StereoSGBM::create(0, 128, 5, 600, 2400, 1, 63, 12, 200, 2, sdr::StereoSGBM::MODE_SGBM);
    sdr::Mat disp, disp_f, xyz;
    auto pcd = [&]() {  // pcd_write.cpp:111-116
        sgbm->compute(L, R, disp);
        sdr::convertTo32F(disp, disp_f, 1.0 / 16.0);
        sdr::reprojectImageTo3D(disp_f, xyz, Q, true);
    };
    sdr::StereoDisparity sd(Q);
    sdr::Mat cdisp, cdepth;
    auto cls = [&]() {  // stereo_displayer.cpp:161-162
        cdisp = sd.computeDisparity(BL, BR);
        cdepth = sd.computeDepth(cdisp);
    };
    auto rate = [&](auto&& fn) {
        for (int i = 0; i < 5; i++) fn();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < frames; i++) fn();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / frames;
        return s;
    };
    const double s_pcd = rate(pcd), s_cls = rate(cls);
    write_mat(dir + "/pcd_disp.bin", disp);
    write_mat(dir + "/pcd_xyz.bin", xyz);
    write_mat(dir + "/cls_disp.bin", cdisp);
    write_mat(dir + "/cls_depth.bin", cdepth);
    std::printf("{\"frames\": %d, \"pcd_separate\": {\"fps\": %.1f, \"Mpix_s\": %.1f, \"ms_per_frame\": %.3f}, "
                "\"class_computeDisparity_computeDepth\": {\"fps\": %.1f, \"Mpix_s_input\": %.1f, \"ms_per_frame\": %.3f}}\n",
                frames, 1 / s_pcd, W * H / s_pcd / 1e6, s_pcd * 1e3, 1 / s_cls, W * H / s_cls / 1e6, s_cls * 1e3);
    return 0;
}
