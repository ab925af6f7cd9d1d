// sdr_rectify.hip -- the ingest step in front of the hot path:
//   StereoRectifier(config): cv::initUndistortRectifyMap(K, D, R1/R2, P1/P2, size, CV_16SC2)
//       reference stereo_vision/src/stereo_rectifier.cpp:6-11
//   StereoRectifier::rectify: cv::remap(src, dst, map1, map2, INTER_LINEAR)   stereo_rectifier.cpp:39-40
//   side-by-side split frame(Rect(0,0,W/2,H)) | frame(Rect(W/2,0,W/2,H))    stereo_displayer.cpp:155-156
// restating OpenCV 4.6 the way oracle/rectify_oracle.c does (the checker; parity with OpenCV unpinned).
//
// Kernels:
//   k_init_map       one thread per map row: the scalar loop of initUndistortRectifyMapComputer,
//                    f64, contraction off, x/y/w accumulated column by column as OpenCV does
//   k_remap          cv::remap INTER_LINEAR, BORDER_CONSTANT 0, fixed-point (15-bit) weights that
//                    are exact for bilinear, so the integer sum matches OpenCV's table bit for bit;
//                    one thread per output pixel (maps 6 B/px, source gathers served by L2)
//   k_sbs_ingest     fused per-frame ingest of a side-by-side frame: split -> remap both eyes ->
//                    (a) rectified BGR (optional, display/colour) and/or
//                    (b) BGR2GRAY + INTER_AREA 0.5x of the rectified eye (the class path's
//                        stereo_disparity.cpp:19-24 pre-steps), each rounding kept as OpenCV does
#include "../../include/sdr/sdr.h"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <string>

#pragma clang fp contract(off)

namespace sdr {

struct MapParams {
    double ir[9];
    double k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4;
    double u0, v0, fx, fy;
};

__device__ __forceinline__ int round_sat_int(double v) {
    const double r = rint(v);
    if (r >= 2147483647.0) return 2147483647;
    if (r <= -2147483648.0) return (int)-2147483647 - 1;
    return (int)r;
}

__global__ __launch_bounds__(64) void k_init_map(MapParams m, int W, int H, int16_t* __restrict__ map1,
                                                 uint16_t* __restrict__ map2) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= H) return;
    const double* ir = m.ir;
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
        const double w = 1. / _w, x = _x * w, y = _y * w;
        const double x2 = x * x, y2 = y * y;
        const double r2 = x2 + y2, _2xy = 2 * x * y;
        const double kr = (1 + ((m.k3 * r2 + m.k2) * r2 + m.k1) * r2) /
                          (1 + ((m.k6 * r2 + m.k5) * r2 + m.k4) * r2);
        const double xd = (x * kr + m.p1 * _2xy + m.p2 * (r2 + 2 * x2) + m.s1 * r2 + m.s2 * r2 * r2);
        const double yd = (y * kr + m.p1 * (r2 + 2 * y2) + m.p2 * _2xy + m.s3 * r2 + m.s4 * r2 * r2);
        const double u = m.fx * 1.0 * xd + m.u0;
        const double v = m.fy * 1.0 * yd + m.v0;
        const int iu = round_sat_int(u * 32), iv = round_sat_int(v * 32);
        const size_t o = (size_t)i * W + j;
        *(uint32_t*)(map1 + 2 * o) = (uint32_t)(uint16_t)(int16_t)(iu >> 5) |
                                     ((uint32_t)(uint16_t)(int16_t)(iv >> 5) << 16);
        map2[o] = (uint16_t)((iv & 31) * 32 + (iu & 31));
    }
}

// one remapped pixel: cn channels of the source at map entry (sx, sy, frac) -> out[0..cn)
template <int CN>
__device__ __forceinline__ void remap_px(const uint8_t* __restrict__ src, int sw, int sh,
                                         size_t sstride, uint32_t m1, uint32_t m2, int* out) {
    const int sx = (int)(int16_t)(m1 & 0xffff), sy = (int)(int16_t)(m1 >> 16);
    const int ax = (int)(m2 & 31), ay = (int)(m2 >> 5) & 31;
    const int w00 = (32 - ax) * (32 - ay) * 32, w01 = ax * (32 - ay) * 32;
    const int w10 = (32 - ax) * ay * 32, w11 = ax * ay * 32;
    const bool x0 = sx >= 0 && sx < sw, x1 = sx + 1 >= 0 && sx + 1 < sw;
    const bool y0 = sy >= 0 && sy < sh, y1 = sy + 1 >= 0 && sy + 1 < sh;
    // every tap is loaded from a clamped, valid address and masked afterwards (BORDER_CONSTANT 0):
    // loads under a condition made the compiler branch around each one and wait for it there
    const int cx0 = min(max(sx, 0), sw - 1), cx1 = min(max(sx + 1, 0), sw - 1);
    const int cy0 = min(max(sy, 0), sh - 1), cy1 = min(max(sy + 1, 0), sh - 1);
    const uint8_t* r0 = src + (size_t)cy0 * sstride;
    const uint8_t* r1 = src + (size_t)cy1 * sstride;
    int t[4][CN];
#pragma unroll
    for (int c = 0; c < CN; c++) {
        t[0][c] = r0[cx0 * CN + c];
        t[1][c] = r0[cx1 * CN + c];
        t[2][c] = r1[cx0 * CN + c];
        t[3][c] = r1[cx1 * CN + c];
    }
#pragma unroll
    for (int c = 0; c < CN; c++) {
        const int v00 = (x0 && y0) ? t[0][c] : 0;
        const int v01 = (x1 && y0) ? t[1][c] : 0;
        const int v10 = (x0 && y1) ? t[2][c] : 0;
        const int v11 = (x1 && y1) ? t[3][c] : 0;
        const int acc = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
        out[c] = min(max((acc + (1 << 14)) >> 15, 0), 255);
    }
}

template <int CN>
__global__ __launch_bounds__(256) void k_remap(const uint8_t* __restrict__ src, int sw, int sh,
                                               size_t sstride, size_t sfstride,
                                               const int16_t* __restrict__ map1,
                                               const uint16_t* __restrict__ map2, int dw, int dh,
                                               uint8_t* __restrict__ dst, size_t dstride,
                                               size_t dfstride) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= dw || y >= dh) return;
    const size_t o = (size_t)y * dw + x;
    int v[CN];
    remap_px<CN>(src + (size_t)blockIdx.z * sfstride, sw, sh, sstride, ((const uint32_t*)map1)[o],
                 map2[o], v);
    uint8_t* d = dst + (size_t)blockIdx.z * dfstride + (size_t)y * dstride + (size_t)x * CN;
#pragma unroll
    for (int c = 0; c < CN; c++) d[c] = (uint8_t)v[c];
}

// remap_px<3> with each source row's two taps fetched as one 6-byte span (a dword and a short at
// byte 3 * cx, cx = clamp(sx, 0, sw - 2): both taps of an interior pixel, and every valid tap of
// an edge one, lie inside it, and it never leaves the row) instead of six byte loads; a tap's
// bytes are picked by its position in the span, invalid taps masked as before.  Needs sw >= 2.
__device__ __forceinline__ uint64_t bgr_span(const uint8_t* p) {
    uint32_t lo;
    uint16_t hi;
    __builtin_memcpy(&lo, p, 4);
    __builtin_memcpy(&hi, p + 4, 2);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void remap_px_bgr_span(const uint8_t* __restrict__ src, int sw, int sh, size_t sstride,
                                                  uint32_t m1, uint32_t m2, int* out) {
    const int sx = (int)(int16_t)(m1 & 0xffff), sy = (int)(int16_t)(m1 >> 16);
    const int ax = (int)(m2 & 31), ay = (int)(m2 >> 5) & 31;
    const int w00 = (32 - ax) * (32 - ay) * 32, w01 = ax * (32 - ay) * 32;
    const int w10 = (32 - ax) * ay * 32, w11 = ax * ay * 32;
    const bool x0 = sx >= 0 && sx < sw, x1 = sx + 1 >= 0 && sx + 1 < sw;
    const bool y0 = sy >= 0 && sy < sh, y1 = sy + 1 >= 0 && sy + 1 < sh;
    const int cx = min(max(sx, 0), sw - 2);
    const int cy0 = min(max(sy, 0), sh - 1), cy1 = min(max(sy + 1, 0), sh - 1);
    const uint64_t s0 = bgr_span(src + (size_t)cy0 * sstride + 3 * cx);
    const uint64_t s1 = bgr_span(src + (size_t)cy1 * sstride + 3 * cx);
    // bit offsets of the two taps in the span (a masked tap's offset is any valid one)
    const int b0 = 24 * min(max(sx - cx, 0), 1), b1 = 24 * min(max(sx + 1 - cx, 0), 1);
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int v00 = (x0 && y0) ? (int)((s0 >> (b0 + 8 * c)) & 0xff) : 0;
        const int v01 = (x1 && y0) ? (int)((s0 >> (b1 + 8 * c)) & 0xff) : 0;
        const int v10 = (x0 && y1) ? (int)((s1 >> (b0 + 8 * c)) & 0xff) : 0;
        const int v11 = (x1 && y1) ? (int)((s1 >> (b1 + 8 * c)) & 0xff) : 0;
        const int acc = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
        out[c] = min(max((acc + (1 << 14)) >> 15, 0), 255);
    }
}

__device__ __forceinline__ int bgr2gray(int b, int g, int r) {
    return (b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14;
}

struct SbsArgs {
    const uint8_t* sbs;        // [F][H][2W][3]
    size_t sstride, sfstride;  // bytes
    const int16_t* map1[2];    // per eye [H][W][2]
    const uint16_t* map2[2];
    int W, H;                  // one eye
    uint8_t* bgr[2];           // nullable [F][H][W][3]
    uint8_t* small[2];         // nullable [F][H/2][W/2]
};

// one thread per 2x2 block of rectified output (= one half-size gray pixel), blockIdx.z = frame*2+eye
__global__ __launch_bounds__(256) void k_sbs_ingest(SbsArgs a) {
    const int x2 = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y2 = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int eye = blockIdx.z & 1, f = blockIdx.z >> 1;
    const int W = a.W, H = a.H, w2 = W >> 1, h2 = H >> 1;
    const int nbx = (W + 1) >> 1, nby = (H + 1) >> 1;  // 2x2 blocks covering odd sizes too
    if (x2 >= nbx || y2 >= nby) return;
    const uint8_t* src = a.sbs + (size_t)f * a.sfstride + (size_t)eye * W * 3;
    const uint32_t* m1 = (const uint32_t*)a.map1[eye];
    const uint16_t* m2 = a.map2[eye];
    uint8_t* bgr = a.bgr[eye] ? a.bgr[eye] + (size_t)f * W * H * 3 : nullptr;
    int gsum = 0;
    // the block's four map entries first (clamped to the image: an odd size's missing pixels are
    // computed on a duplicate and dropped), then every gather, all unconditional
    uint32_t e1[4], e2[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const size_t o = (size_t)min(2 * y2 + (q >> 1), H - 1) * W + min(2 * x2 + (q & 1), W - 1);
        e1[q] = m1[o];
        e2[q] = m2[o];
    }
    int v[4][3];
#pragma unroll
    for (int q = 0; q < 4; q++) remap_px_bgr_span(src, W, H, a.sstride, e1[q], e2[q], v[q]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int x = 2 * x2 + (q & 1), y = 2 * y2 + (q >> 1);
        if (x >= W || y >= H) continue;
        if (bgr) {
            uint8_t* d = bgr + ((size_t)y * W + x) * 3;
            d[0] = (uint8_t)v[q][0];
            d[1] = (uint8_t)v[q][1];
            d[2] = (uint8_t)v[q][2];
        }
        gsum += bgr2gray(v[q][0], v[q][1], v[q][2]);
    }
    if (a.small[eye] && x2 < w2 && y2 < h2)
        a.small[eye][(size_t)f * w2 * h2 + (size_t)y2 * w2 + x2] = (uint8_t)((gsum + 2) >> 2);
}

}  // namespace sdr

// ===========================================================================================
// C ABI (include/sdr/sdr.h)
// ===========================================================================================
struct sdr_rectifier {
    int device = 0, W = 0, H = 0;
    hipStream_t stream = nullptr, own_stream = nullptr;
    sdr::Buf map1[2], map2[2];
};

namespace {

#define RECT_HIP(call)                                                                          \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return sdr::set_error(SDR_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// iR = inv(P[:, :3] * R): gemm with sums from k = 0, then cv::invert(DECOMP_LU)'s closed form
// for n = 3 (det3, cofactors times 1/det); host f64, the same expression order as the oracle
int make_map_params(const double K[9], const double* dist, int ndist, const double R[9],
                    const double* P, int p_cols, sdr::MapParams* m) {
    if (!K || !R || !P || (ndist > 0 && !dist)) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (p_cols != 3 && p_cols != 4) return sdr::set_error(SDR_ERR_ARG, "P must be 3x3 or 3x4");
    if (!(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8 || ndist == 12 || ndist == 14))
        return sdr::set_error(SDR_ERR_ARG, "distortion must have 4, 5, 8, 12 or 14 coefficients");
    double A[9], M[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) A[r * 3 + c] = P[r * p_cols + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += A[r * 3 + k] * R[k * 3 + c];
            M[r * 3 + c] = s;
        }
#define mm(a, b) M[(a) * 3 + (b)]
    double d = mm(0, 0) * (mm(1, 1) * mm(2, 2) - mm(1, 2) * mm(2, 1)) -
               mm(0, 1) * (mm(1, 0) * mm(2, 2) - mm(1, 2) * mm(2, 0)) +
               mm(0, 2) * (mm(1, 0) * mm(2, 1) - mm(1, 1) * mm(2, 0));
    double* iR = m->ir;
    if (d == 0.0) {
        for (int i = 0; i < 9; i++) iR[i] = 0.0;
    } else {
        d = 1.0 / d;
        iR[0] = (mm(1, 1) * mm(2, 2) - mm(1, 2) * mm(2, 1)) * d;
        iR[1] = (mm(0, 2) * mm(2, 1) - mm(0, 1) * mm(2, 2)) * d;
        iR[2] = (mm(0, 1) * mm(1, 2) - mm(0, 2) * mm(1, 1)) * d;
        iR[3] = (mm(1, 2) * mm(2, 0) - mm(1, 0) * mm(2, 2)) * d;
        iR[4] = (mm(0, 0) * mm(2, 2) - mm(0, 2) * mm(2, 0)) * d;
        iR[5] = (mm(0, 2) * mm(1, 0) - mm(0, 0) * mm(1, 2)) * d;
        iR[6] = (mm(1, 0) * mm(2, 1) - mm(1, 1) * mm(2, 0)) * d;
        iR[7] = (mm(0, 1) * mm(2, 0) - mm(0, 0) * mm(2, 1)) * d;
        iR[8] = (mm(0, 0) * mm(1, 1) - mm(0, 1) * mm(1, 0)) * d;
    }
#undef mm
    double k[14] = {0};
    for (int i = 0; i < ndist; i++) k[i] = dist[i];
    m->k1 = k[0]; m->k2 = k[1]; m->p1 = k[2]; m->p2 = k[3]; m->k3 = k[4]; m->k4 = k[5];
    m->k5 = k[6]; m->k6 = k[7]; m->s1 = k[8]; m->s2 = k[9]; m->s3 = k[10]; m->s4 = k[11];
    if (k[12] != 0.0 || k[13] != 0.0)
        return sdr::set_error(SDR_ERR_ARG, "tilted-sensor coefficients (tauX, tauY) are not supported");
    m->u0 = K[2]; m->v0 = K[5]; m->fx = K[0]; m->fy = K[4];
    return SDR_OK;
}

int enqueue_init_map(const sdr::MapParams& m, int W, int H, int16_t* map1, uint16_t* map2,
                     hipStream_t st) {
    hipLaunchKernelGGL(sdr::k_init_map, dim3((H + 63) / 64), dim3(64), 0, st, m, W, H, map1, map2);
    RECT_HIP(hipGetLastError());
    return SDR_OK;
}

}  // namespace

extern "C" {

int sdr_init_undistort_rectify_map(const double K[9], const double* dist, int ndist, const double R[9],
                                   const double* P, int p_cols, int W, int H, int device,
                                   int16_t* map1, uint16_t* map2) {
    if (!map1 || !map2 || W <= 0 || H <= 0) return sdr::set_error(SDR_ERR_ARG, "bad map arguments");
    if (W > 32767 || H > 32767) return sdr::set_error(SDR_ERR_SIZE, "CV_16SC2 maps need size < 32768");
    sdr::MapParams m;
    int rc = make_map_params(K, dist, ndist, R, P, p_cols, &m);
    if (rc) return rc;
    RECT_HIP(hipSetDevice(device));
    const size_t px = (size_t)W * H;
    int16_t* d1 = nullptr;
    uint16_t* d2 = nullptr;
    RECT_HIP(hipMalloc((void**)&d1, px * 4));
    if (hipMalloc((void**)&d2, px * 2) != hipSuccess) {
        (void)hipFree(d1);
        return sdr::set_error(SDR_ERR_NOMEM, "hipMalloc failed");
    }
    rc = enqueue_init_map(m, W, H, d1, d2, nullptr);
    if (!rc && hipMemcpy(map1, d1, px * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = SDR_ERR_DEVICE;
    if (!rc && hipMemcpy(map2, d2, px * 2, hipMemcpyDeviceToHost) != hipSuccess) rc = SDR_ERR_DEVICE;
    (void)hipFree(d1);
    (void)hipFree(d2);
    if (rc == SDR_ERR_DEVICE) return sdr::set_error(rc, "map copy failed");
    return rc;
}

int sdr_rectifier_create(const double K_left[9], const double* dist_left, int ndist_left,
                         const double R1[9], const double* P1, const double K_right[9],
                         const double* dist_right, int ndist_right, const double R2[9],
                         const double* P2, int p_cols, int W, int H, int device,
                         sdr_rectifier** out) {
    if (!out || W <= 0 || H <= 0) return sdr::set_error(SDR_ERR_ARG, "bad rectifier arguments");
    if (W > 32767 || H > 32767) return sdr::set_error(SDR_ERR_SIZE, "CV_16SC2 maps need size < 32768");
    sdr::MapParams ml, mr;
    int rc;
    if ((rc = make_map_params(K_left, dist_left, ndist_left, R1, P1, p_cols, &ml))) return rc;
    if ((rc = make_map_params(K_right, dist_right, ndist_right, R2, P2, p_cols, &mr))) return rc;
    RECT_HIP(hipSetDevice(device));
    sdr_rectifier* h = new sdr_rectifier();
    h->device = device;
    h->W = W;
    h->H = H;
    const size_t px = (size_t)W * H;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return sdr::set_error(SDR_ERR_DEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    for (int e = 0; e < 2 && !rc; e++) {
        if ((rc = sdr::ensure(h->map1[e], px * 4))) break;
        if ((rc = sdr::ensure(h->map2[e], px * 2))) break;
        rc = enqueue_init_map(e ? mr : ml, W, H, (int16_t*)h->map1[e].p, (uint16_t*)h->map2[e].p,
                              h->stream);
    }
    if (!rc && hipStreamSynchronize(h->stream) != hipSuccess)
        rc = sdr::set_error(SDR_ERR_DEVICE, "map build failed");
    if (rc) {
        sdr_rectifier_destroy(h);
        return rc;
    }
    *out = h;
    return SDR_OK;
}

int sdr_rectifier_destroy(sdr_rectifier* h) {
    if (!h) return SDR_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (int e = 0; e < 2; e++) {
        if (h->map1[e].p) (void)hipFree(h->map1[e].p);
        if (h->map2[e].p) (void)hipFree(h->map2[e].p);
    }
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return SDR_OK;
}

int sdr_rectifier_set_stream(sdr_rectifier* h, void* stream) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = (hipStream_t)stream;  // NULL = the HIP null (legacy default) stream
    return SDR_OK;
}

int sdr_rectifier_reset_stream(sdr_rectifier* h) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = h->own_stream;
    return SDR_OK;
}

int sdr_rectifier_get_maps(const sdr_rectifier* h, int which, int16_t* map1, uint16_t* map2) {
    if (!h || (which != 0 && which != 1)) return sdr::set_error(SDR_ERR_ARG, "bad arguments");
    RECT_HIP(hipSetDevice(h->device));
    RECT_HIP(hipStreamSynchronize(h->stream));
    const size_t px = (size_t)h->W * h->H;
    if (map1) RECT_HIP(hipMemcpy(map1, h->map1[which].p, px * 4, hipMemcpyDeviceToHost));
    if (map2) RECT_HIP(hipMemcpy(map2, h->map2[which].p, px * 2, hipMemcpyDeviceToHost));
    return SDR_OK;
}

int sdr_remap_bilinear_device(const uint8_t* src, int sw, int sh, size_t sstride, size_t sfstride,
                              int channels, const int16_t* map1, const uint16_t* map2, int dw,
                              int dh, uint8_t* dst, size_t dstride, size_t dfstride, int nframes,
                              void* stream) {
    if (!src || !map1 || !map2 || !dst) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || nframes <= 0)
        return sdr::set_error(SDR_ERR_ARG, "bad size");
    if (channels != 1 && channels != 3) return sdr::set_error(SDR_ERR_TYPE, "channels must be 1 or 3");
    if (sstride < (size_t)sw * channels || dstride < (size_t)dw * channels)
        return sdr::set_error(SDR_ERR_ARG, "bad stride");
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, nframes);
    if (channels == 1)
        hipLaunchKernelGGL(sdr::k_remap<1>, grid, dim3(256), 0, st, src, sw, sh, sstride, sfstride,
                           map1, map2, dw, dh, dst, dstride, dfstride);
    else
        hipLaunchKernelGGL(sdr::k_remap<3>, grid, dim3(256), 0, st, src, sw, sh, sstride, sfstride,
                           map1, map2, dw, dh, dst, dstride, dfstride);
    RECT_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_rectify_device(sdr_rectifier* h, const uint8_t* d_left, const uint8_t* d_right,
                       size_t stride, size_t frame_stride, int channels, int nframes,
                       uint8_t* d_left_out, uint8_t* d_right_out, size_t out_stride,
                       size_t out_frame_stride) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    RECT_HIP(hipSetDevice(h->device));
    int rc;
    const uint8_t* in[2] = {d_left, d_right};
    uint8_t* outp[2] = {d_left_out, d_right_out};
    for (int e = 0; e < 2; e++) {
        if (!in[e] && !outp[e]) continue;
        if ((rc = sdr_remap_bilinear_device(in[e], h->W, h->H, stride, frame_stride, channels,
                                            (const int16_t*)h->map1[e].p,
                                            (const uint16_t*)h->map2[e].p, h->W, h->H, outp[e],
                                            out_stride, out_frame_stride, nframes, h->stream)))
            return rc;
    }
    return SDR_OK;
}

int sdr_rectify_sbs_device(sdr_rectifier* h, const uint8_t* d_sbs, size_t sbs_stride,
                           size_t sbs_frame_stride, int nframes, uint8_t* d_bgr_left,
                           uint8_t* d_bgr_right, uint8_t* d_small_left, uint8_t* d_small_right) {
    if (!h || !d_sbs) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (nframes <= 0 || sbs_stride < (size_t)h->W * 6 ||
        (nframes > 1 && sbs_frame_stride < sbs_stride * h->H))
        return sdr::set_error(SDR_ERR_ARG, "bad SBS stride (frame must be (2*W) x H BGR)");
    if ((d_small_left || d_small_right) && ((h->W & 1) || (h->H & 1)))
        return sdr::set_error(SDR_ERR_SIZE, "INTER_AREA 0.5x needs even width and height");
    if (h->W < 2) return sdr::set_error(SDR_ERR_SIZE, "the SBS ingest needs eyes at least 2 pixels wide");
    RECT_HIP(hipSetDevice(h->device));
    sdr::SbsArgs a{};
    a.sbs = d_sbs;
    a.sstride = sbs_stride;
    a.sfstride = sbs_frame_stride;
    a.W = h->W;
    a.H = h->H;
    for (int e = 0; e < 2; e++) {
        a.map1[e] = (const int16_t*)h->map1[e].p;
        a.map2[e] = (const uint16_t*)h->map2[e].p;
    }
    a.bgr[0] = d_bgr_left;
    a.bgr[1] = d_bgr_right;
    a.small[0] = d_small_left;
    a.small[1] = d_small_right;
    dim3 grid(((h->W + 1) / 2 + 63) / 64, ((h->H + 1) / 2 + 3) / 4, 2 * nframes);
    hipLaunchKernelGGL(sdr::k_sbs_ingest, grid, dim3(256), 0, h->stream, a);
    RECT_HIP(hipGetLastError());
    return SDR_OK;
}

}  // extern "C"
