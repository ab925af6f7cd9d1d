// Exercises include/sdr/stereo.hpp the way the reference's C++ callers would
// (point_cloud/src/pcd_write.cpp:102-116, stereo_vision/src/stereo_disparity.cpp).
// usage: facade_test <W> <H> <left.bin> <right.bin> <bgr_left.bin> <bgr_right.bin> <outdir>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "sdr/stereo.hpp"

static std::vector<uint8_t> slurp(const char* p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}
static void dump(const std::string& p, const sdr::Mat& m) {
    std::ofstream f(p, std::ios::binary);
    for (int y = 0; y < m.rows; y++) f.write((const char*)m.ptr<uint8_t>(y), (std::streamsize)(m.cols * sdr::elem_size(m.type)));
}

int main(int argc, char** argv) {
    if (argc != 8) return 2;
    const int W = std::stoi(argv[1]), H = std::stoi(argv[2]);
    std::vector<uint8_t> l = slurp(argv[3]), r = slurp(argv[4]), bl = slurp(argv[5]), br = slurp(argv[6]);
    const std::string out = argv[7];
    try {
        // pcd_write.cpp path: SGBM (3WAY d=80) on gray, convertTo(1/16), reproject(handleMissing)
        sdr::Mat L = sdr::Mat::view(H, W, sdr::CV_8UC1, l.data()), R = sdr::Mat::view(H, W, sdr::CV_8UC1, r.data());
        auto sgbm = sdr::StereoSGBM::create(0, 80, 5, 8 * 5 * 5 * 3, 32 * 5 * 5 * 3, 1, 63, 12, 200, 2,
                                            sdr::StereoSGBM::MODE_SGBM_3WAY);
        sdr::Mat disp;
        sgbm->compute(L, R, disp);
        dump(out + "/disp.bin", disp);
        sdr::Mat Q(4, 4, sdr::CV_64FC1);
        const double q[16] = {1, 0, 0, -645.44378662109375, 0, 1, 0, -347.0967903137207,
                              0, 0, 0, 669.90015369541641, 0, 0, 0.00832541998100415, 0};
        for (int i = 0; i < 16; i++) Q.ptr<double>(i / 4)[i % 4] = q[i];
        sdr::Mat disp_float, xyz;
        sdr::convertTo32F(disp, disp_float, 1.0 / 16.0);
        sdr::reprojectImageTo3D(disp_float, xyz, Q, true);
        dump(out + "/xyz.bin", xyz);
        // the fused host call, into plain and into page-locked Mats: the same bytes
        sdr::Mat disp2, xyz2;
        sgbm->computeReproject(L, R, Q, true, disp2, xyz2);
        sdr::Mat disp3 = sdr::Mat::page_locked(H, W, sdr::CV_16SC1), xyz3 = sdr::Mat::page_locked(H, W, sdr::CV_32FC3);
        sdr::Mat Lp = sdr::Mat::page_locked(H, W, sdr::CV_8UC1), Rp = sdr::Mat::page_locked(H, W, sdr::CV_8UC1);
        std::memcpy(Lp.data, l.data(), l.size());
        std::memcpy(Rp.data, r.data(), r.size());
        sgbm->computeReproject(Lp, Rp, Q, true, disp3, xyz3);
        const size_t nd = (size_t)W * H * 2, nx = (size_t)W * H * 12;
        std::printf("fused_equal=%d\n", std::memcmp(disp2.data, disp.data, nd) == 0 &&
                                           std::memcmp(xyz2.data, xyz.data, nx) == 0 &&
                                           std::memcmp(disp3.data, disp.data, nd) == 0 &&
                                           std::memcmp(xyz3.data, xyz.data, nx) == 0);
        // class path: StereoDisparity(Q).computeDisparity(BGR, BGR) / computeDepth
        sdr::StereoDisparity sd(Q);
        sdr::Mat BL = sdr::Mat::view(H, W, sdr::CV_8UC3, bl.data()), BR = sdr::Mat::view(H, W, sdr::CV_8UC3, br.data());
        sdr::Mat df = sd.computeDisparity(BL, BR);
        dump(out + "/class_disp.bin", df);
        dump(out + "/class_conf.bin", sd.getConfidenceMap());
        sdr::Mat depth = sd.computeDepth(df);
        dump(out + "/class_depth.bin", depth);
        // display outputs (stereo_disparity.cpp:42-124, stereo_displayer.cpp:105-118,164-173): two
        // frames each, so the second goes through the EMA against the first
        for (int k = 0; k < 2; k++) {
            sdr::Mat vis = sd.show_disparityMap(df), dv = sd.show_depthMap(depth);
            dump(out + "/vis" + std::to_string(k) + ".bin", vis);
            dump(out + "/depthvis" + std::to_string(k) + ".bin", dv);
            if (k == 1) {
                sdr::Display disp_out;
                dump(out + "/overlay.bin", disp_out.overlay(vis, BL));
                std::printf("coverage=%.17g\n", disp_out.depth_coverage(depth));
            }
        }
        // the displayer's order on ONE Display: show_depthMap, depth_coverage, show_depthMap -- the
        // coverage call must leave the depth map's EMA history alone
        {
            sdr::Display dd;
            double zr[2] = {1000.0, 2000.0};
            for (int k = 0; k < 2; k++) {
                dump(out + "/dd_depthvis" + std::to_string(k) + ".bin", dd.show_depthMap(depth, zr));
                std::printf("dd_coverage%d=%.17g\n", k, dd.depth_coverage(depth));
            }
        }
        std::printf("numDisparities=%d\n", sd.get_matcher()->getNumDisparities());
        // error behaviour: numDisparities not divisible by 16 -> exception, like cv::Exception
        try {
            auto bad = sdr::StereoSGBM::create(0, 100, 5);
            bad->compute(L, R, disp);
            std::printf("ERROR: no exception\n");
            return 3;
        } catch (const sdr::Exception& e) {
            std::printf("exception code=%d\n", e.code);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "failed: %s\n", e.what());
        return 1;
    }
    return 0;
}
