/*
 * rectify_oracle.c -- CPU restatement of the ingest step before the hot path.
 * TEST INFRASTRUCTURE ONLY: the checker for the GPU kernels in stereo_depth_ruler_amd/csrc/sdr_rectify.hip.
 *
 *   cv::initUndistortRectifyMap(K, D, R, P, size, CV_16SC2, map1, map2)
 *       reference stereo_vision/src/stereo_rectifier.cpp:7-11   [OpenCV 4.6 calib3d/src/undistort.dispatch.cpp,
 *       undistort.simd.hpp initUndistortRectifyMapComputer, scalar loop]
 *   cv::remap(src, dst, map1, map2, INTER_LINEAR)  (BORDER_CONSTANT, value 0)
 *       stereo_rectifier.cpp:39-40   [OpenCV 4.6 imgproc/src/imgwarp.cpp remapBilinear with the
 *       fixed-point table of initInterTab2D(INTER_LINEAR, true)]
 *   frame(Rect(0,0,W/2,H)) / frame(Rect(W/2,0,W/2,H))  SBS split, stereo_displayer.cpp:155-156
 *
 * PARITY UNPINNED against OpenCV itself (absent from this image; the reference holds no fixtures).
 * Known divergence source: OpenCV's CPU-dispatched SIMD variant of the map loop (SSE2/AVX2 lanes,
 * FMA in v_muladd) rounds differently from the scalar loop restated here, so an OpenCV map entry can
 * differ by one 1/32-pixel step where u*32 or v*32 sits on a rounding boundary.  The remap itself is
 * exact integer arithmetic: identical for identical maps.
 *
 * Map formula (scalar loop, per row i, x accumulated column by column):
 *   iR = inv(P[:, :3] * R)  (3x3 closed-form inverse of cv::invert DECOMP_LU for n = 3)
 *   _x = i*iR01 + iR02, _y = i*iR11 + iR12, _w = i*iR21 + iR22;  per column: _x += iR00 ...
 *   w = 1/_w, x = _x*w, y = _y*w; r2 = x^2 + y^2;
 *   kr = (1 + ((k3 r2 + k2) r2 + k1) r2) / (1 + ((k6 r2 + k5) r2 + k4) r2)
 *   xd = x kr + p1 2xy + p2 (r2 + 2x^2) + s1 r2 + s2 r2^2;  yd = y kr + p1 (r2 + 2y^2) + p2 2xy + s3 r2 + s4 r2^2
 *   u = fx xd + u0, v = fy yd + v0  (no tilt: tauX = tauY = 0)
 *   iu = cvRound(u*32), iv = cvRound(v*32);  map1 = (iu >> 5, iv >> 5), map2 = (iv & 31)*32 + (iu & 31)
 * Remap per channel: w00 = (32-ax)(32-ay)*32, w01 = ax(32-ay)*32, w10 = (32-ax)ay*32, w11 = ax*ay*32
 *   (ax = map2 & 31, ay = map2 >> 5; the float table is exact for INTER_LINEAR), corners outside the
 *   source read 0, dst = sat_u8((sum + 2^14) >> 15).
 */
#include "rectify_oracle.h"

#include <math.h>
#include <string.h>

void orc_rectify_inv_matrix(const double K[9], const double R[9], const double P[12], int p_cols,
                            double iR[9]) {
    /* Ar = P.colRange(0,3) (3x3 or 3x4 input); M = Ar * R (gemm: sum over k from 0) */
    double A[9], M[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) A[r * 3 + c] = P[r * p_cols + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += A[r * 3 + k] * R[k * 3 + c];
            M[r * 3 + c] = s;
        }
    /* cv::invert(DECOMP_LU), n == 3: det3 then cofactors * (1/det) */
#define m(a, b) M[(a) * 3 + (b)]
    double d = m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) -
               m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
               m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
    if (d == 0.0) {
        memset(iR, 0, sizeof(double) * 9);
        return;
    }
    d = 1.0 / d;
    iR[0] = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) * d;
    iR[1] = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) * d;
    iR[2] = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) * d;
    iR[3] = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * d;
    iR[4] = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * d;
    iR[5] = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * d;
    iR[6] = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * d;
    iR[7] = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * d;
    iR[8] = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * d;
#undef m
    (void)K;
}

/* saturate_cast<int>(double) = cvRound: round half to even; out of int range saturates */
static int round_sat_int(double v) {
    const double r = nearbyint(v);
    if (r >= 2147483647.0) return 2147483647;
    if (r <= -2147483648.0) return (int)-2147483647 - 1;
    return (int)r;
}

void orc_init_undistort_rectify_map(const double K[9], const double* dist, int ndist,
                                    const double R[9], const double P[12], int p_cols, int W, int H,
                                    int16_t* map1, uint16_t* map2) {
    double iR[9];
    orc_rectify_inv_matrix(K, R, P, p_cols, iR);
    double k[14] = {0};
    for (int i = 0; i < ndist && i < 14; i++) k[i] = dist[i];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6],
                 k6 = k[7], s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
    const double u0 = K[2], v0 = K[5], fx = K[0], fy = K[4];
    for (int i = 0; i < H; i++) {
        double _x = i * iR[1] + iR[2], _y = i * iR[4] + iR[5], _w = i * iR[7] + iR[8];
        for (int j = 0; j < W; j++, _x += iR[0], _y += iR[3], _w += iR[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
            const double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
            /* matTilt = identity: vecTilt = (xd, yd, 1), invProj = 1 */
            const double u = fx * 1.0 * xd + u0;
            const double v = fy * 1.0 * yd + v0;
            const int iu = round_sat_int(u * 32), iv = round_sat_int(v * 32);
            const size_t o = (size_t)i * W + j;
            map1[2 * o] = (int16_t)(iu >> 5);
            map1[2 * o + 1] = (int16_t)(iv >> 5);
            map2[o] = (uint16_t)((iv & 31) * 32 + (iu & 31));
        }
    }
}

void orc_remap_bilinear_u8(const uint8_t* src, int sw, int sh, size_t sstride, int cn,
                           const int16_t* map1, const uint16_t* map2, int dw, int dh,
                           uint8_t* dst, size_t dstride) {
    for (int y = 0; y < dh; y++) {
        uint8_t* D = dst + (size_t)y * dstride;
        for (int x = 0; x < dw; x++) {
            const size_t o = (size_t)y * dw + x;
            const int sx = map1[2 * o], sy = map1[2 * o + 1];
            const int ax = map2[o] & 31, ay = map2[o] >> 5;
            const int w[4] = {(32 - ax) * (32 - ay) * 32, ax * (32 - ay) * 32, (32 - ax) * ay * 32,
                              ax * ay * 32};
            const int xs[2] = {sx, sx + 1}, ys[2] = {sy, sy + 1};
            for (int c = 0; c < cn; c++) {
                int acc = 0;
                for (int q = 0; q < 4; q++) {
                    const int xx = xs[q & 1], yy = ys[q >> 1];
                    const int v = (xx >= 0 && xx < sw && yy >= 0 && yy < sh)
                                      ? src[(size_t)yy * sstride + (size_t)xx * cn + c] : 0;
                    acc += v * w[q];
                }
                int r = (acc + (1 << 14)) >> 15;
                D[(size_t)x * cn + c] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
            }
        }
    }
}
