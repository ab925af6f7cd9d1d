// sdr_display.hip -- the reference's display outputs on the device.
//
//   show_disparityMap  stereo_vision/src/stereo_disparity.cpp:42-73
//       disparity > 0 mask, x 1/numDisparities, pow 0.6, x255 -> u8, EMA 0.63 with prev_vis
//   show_depthMap      stereo_disparity.cpp:83-124
//       Z channel, masked min/max of Z in (0, 10000), EMA 0.9/0.1 of the range (function-static
//       doubles in the reference), convertTo(8U, 255/(zmax-zmin), -255 zmin/(zmax-zmin)),
//       applyColorMap(TURBO), EMA 0.63 with prev_depth_vis
//   overlay            stereo_vision/src/stereo_displayer.cpp:167-173
//       applyColorMap(JET) of the display disparity, resize(left_rect, 0.5, INTER_AREA),
//       addWeighted(0.7, 0.3)
//   depth_coverage     stereo_displayer.cpp:105-118
//       share of pixels with Z in [0, 12000] (not NaN) in columns >= 80, over all pixels
//
// All of it is bandwidth-trivial per-pixel work; the only cross-pixel steps are the per-frame
// min/max/count reduction (wave minimum + one atomic per wave) and the range recurrence, a
// single-lane kernel that keeps the smoothing state on the device so the sequence stays
// asynchronous.  Batches of F frames are handled in frame order: the EMA state of pixel i is
// carried through the frames by the thread that owns pixel i.  The rounding rules follow
// oracle/display_oracle.c (recorded OpenCV assumptions there).
#include "../../include/sdr/sdr.h"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>

namespace sdr {
namespace {

struct Lut {
    uint8_t v[768];
};

// cvRound + saturate_cast<uchar> on a float: NaN and |v| >= 2^31 are x86's integer indefinite
// (INT_MIN), i.e. 0 after saturation
__device__ __forceinline__ uint8_t cvround_u8(float v) {
    if (!(v > -2147483648.f && v < 2147483648.f)) return 0;
    const int r = (int)__builtin_rintf(v);
    return (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
}
__device__ __forceinline__ uint8_t add_weighted(uint8_t a, float alpha, uint8_t b, float beta) {
    return cvround_u8(__builtin_fmaf((float)a, alpha, (float)b * beta) + 0.f);
}

__device__ __forceinline__ void lut_to_lds(const Lut& lut, uint8_t* s) {
    for (int i = threadIdx.x; i < 768; i += blockDim.x) s[i] = lut.v[i];
    __syncthreads();
}

#pragma clang fp contract(off)

// show_disparityMap over F frames: vis[f] = EMA(prev, gamma(disp[f])); prev carried per pixel
__global__ __launch_bounds__(256) void k_disp_vis(const float* __restrict__ disp, size_t stride,
                                                  size_t fstride, int W, int H, int F, float scale,
                                                  uint8_t* __restrict__ prev, int has_prev,
                                                  uint8_t* __restrict__ vis) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t i = (size_t)y * W + x;
    const size_t px = (size_t)W * H;
    uint8_t p = has_prev ? prev[i] : 0;
    bool hp = has_prev != 0;
    for (int f = 0; f < F; f++) {
        const float d = disp[(size_t)f * fstride + (size_t)y * stride + x];
        const float n01 = (d > 0.f ? d : 0.f) * scale;
        const float g = (float)pow((double)n01, 0.6);
        uint8_t s = cvround_u8(g * 255.0f);
        if (hp) s = add_weighted(p, 0.63f, s, 1.0f - 0.63f);
        vis[(size_t)f * px + i] = s;
        p = s;
        hp = true;
    }
    prev[i] = p;
}

// per-frame {min bits, max bits, coverage count} of the Z channel; valid Z > 0, so the float
// bits order like the values
struct ZStats {
    uint32_t zmin, zmax, count, pad;
};

__global__ void k_zstats_init(ZStats* st, int F) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < F) st[f] = ZStats{0xffffffffu, 0u, 0u, 0u};
}

__global__ __launch_bounds__(256) void k_zstats(const float* __restrict__ xyz, int channels, int W,
                                                int H, int col0, ZStats* __restrict__ st) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    uint32_t mn = 0xffffffffu, mx = 0u, cnt = 0u;
    if (x < W) {
        const float z = xyz[(((size_t)f * H + y) * W + x) * channels + (channels == 3 ? 2 : 0)];
        if (z > 0.f && z < 10000.f) {  // (Z > 0) & (Z < 10000) & (Z == Z)
            mn = mx = __float_as_uint(z);
        }
        cnt = (x >= col0 && z >= 0.f && z <= 12000.f) ? 1u : 0u;  // NaN fails both compares
    }
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        cnt += (uint32_t)__shfl_xor((int)cnt, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (mn != 0xffffffffu) {
            atomicMin(&st[f].zmin, mn);
            atomicMax(&st[f].zmax, mx);
        }
        if (cnt) atomicAdd(&st[f].count, cnt);
    }
}

// the show_depthMap range recurrence over the F frames, in order (one lane)
__global__ void k_zrange(const ZStats* __restrict__ st, int F, double* __restrict__ zr,
                         float2* __restrict__ ab) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double zmin = zr[0], zmax = zr[1];
    for (int f = 0; f < F; f++) {
        double lo = 0.0, hi = 0.0;
        if (st[f].zmin != 0xffffffffu) {
            lo = (double)__uint_as_float(st[f].zmin);
            hi = (double)__uint_as_float(st[f].zmax);
        }
        if (!(hi > lo)) {
            lo = 1000.0;
            hi = 2000.0;
        }
        const double a = 0.1;
        zmin = (1.0 - a) * zmin + a * lo;
        zmax = (1.0 - a) * zmax + a * hi;
        zmin = fmax(0.0, fmin(zmin, 10000.0));
        zmax = fmax(zmin + 1.0, fmin(zmax, 10000.0));
        ab[f] = make_float2((float)(255.0 / (zmax - zmin)), (float)(-255.0 * zmin / (zmax - zmin)));
    }
    zr[0] = zmin;
    zr[1] = zmax;
}

// show_depthMap's per-pixel part over F frames: TURBO(u8(Z)) with the EMA carried per pixel
__global__ __launch_bounds__(256) void k_depth_vis(const float* __restrict__ xyz, int channels, int W,
                                                   int H, int F, const float2* __restrict__ ab, Lut lut,
                                                   uint8_t* __restrict__ prev, int has_prev,
                                                   uint8_t* __restrict__ out) {
    __shared__ uint8_t sl[768];
    lut_to_lds(lut, sl);
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const size_t i = (size_t)y * W + x;
    const size_t px = (size_t)W * H;
    uint8_t p0 = 0, p1 = 0, p2 = 0;
    if (has_prev) {
        p0 = prev[3 * i];
        p1 = prev[3 * i + 1];
        p2 = prev[3 * i + 2];
    }
    bool hp = has_prev != 0;
    for (int f = 0; f < F; f++) {
        const float z = xyz[((size_t)f * px + i) * channels + (channels == 3 ? 2 : 0)];
        const float2 k = ab[f];
        const int v = cvround_u8(__builtin_fmaf(z, k.x, k.y));
        uint8_t c0 = sl[3 * v], c1 = sl[3 * v + 1], c2 = sl[3 * v + 2];
        if (hp) {
            c0 = add_weighted(p0, 0.63f, c0, 1.0f - 0.63f);
            c1 = add_weighted(p1, 0.63f, c1, 1.0f - 0.63f);
            c2 = add_weighted(p2, 0.63f, c2, 1.0f - 0.63f);
        }
        uint8_t* o = out + ((size_t)f * px + i) * 3;
        o[0] = c0;
        o[1] = c1;
        o[2] = c2;
        p0 = c0;
        p1 = c1;
        p2 = c2;
        hp = true;
    }
    prev[3 * i] = p0;
    prev[3 * i + 1] = p1;
    prev[3 * i + 2] = p2;
}

// applyColorMap(vis, JET) + addWeighted(resize(left_rect, 0.5, INTER_AREA), 0.7, heat, 0.3, 0):
// left is the FULL-resolution rectified BGR view (2W x 2H), area-halved on the fly
__global__ __launch_bounds__(256) void k_overlay(const uint8_t* __restrict__ vis, const uint8_t* __restrict__ left,
                                                 size_t lstride, size_t lfstride, int W, int H, Lut lut,
                                                 uint8_t* __restrict__ heat, uint8_t* __restrict__ overlay) {
    __shared__ uint8_t sl[768];
    lut_to_lds(lut, sl);
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= W) return;
    const size_t px = (size_t)W * H;
    const size_t i = (size_t)f * px + (size_t)y * W + x;
    const int v = vis[i];
    const uint8_t* a = left + (size_t)f * lfstride + (size_t)(2 * y) * lstride + 6 * x;
    const uint8_t* b = a + lstride;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const uint8_t hc = sl[3 * v + c];
        const uint8_t lc = (uint8_t)((a[c] + a[3 + c] + b[c] + b[3 + c] + 2) >> 2);
        if (heat) heat[3 * i + c] = hc;
        if (overlay) overlay[3 * i + c] = add_weighted(lc, 0.7f, hc, 0.3f);
    }
}

#pragma clang fp contract(on)

}  // namespace

// host-side table of a colormap from its published definition (oracle/display_oracle.c restates
// the same formulas independently; tests/test_display.py compares the two)
static int colormap_lut(int cmap, uint8_t* lut) {
    auto clamp01 = [](double v) { return v < 0 ? 0.0 : v > 1 ? 1.0 : v; };
    for (int i = 0; i < 256; i++) {
        const double x = i / 255.0;
        double r, g, b;
        if (cmap == SDR_COLORMAP_JET) {
            r = clamp01(1.5 - std::fabs(4.0 * x - 3.0));
            g = clamp01(1.5 - std::fabs(4.0 * x - 2.0));
            b = clamp01(1.5 - std::fabs(4.0 * x - 1.0));
        } else if (cmap == SDR_COLORMAP_TURBO) {  // Google's Turbo polynomial (2019)
            r = clamp01(0.13572138 + x * (4.61539260 + x * (-42.66032258 + x * (132.13108234 + x * (-152.94239396 + x * 59.28637943)))));
            g = clamp01(0.09140261 + x * (2.19418839 + x * (4.84296658 + x * (-14.18503333 + x * (4.27729857 + x * 2.82956604)))));
            b = clamp01(0.10667330 + x * (12.64194608 + x * (-60.58204836 + x * (110.36276771 + x * (-89.90310912 + x * 27.34824973)))));
        } else {
            return -1;
        }
        lut[3 * i] = (uint8_t)std::floor(255.0 * b + 0.5);
        lut[3 * i + 1] = (uint8_t)std::floor(255.0 * g + 0.5);
        lut[3 * i + 2] = (uint8_t)std::floor(255.0 * r + 0.5);
    }
    return 0;
}

}  // namespace sdr

struct sdr_display {
    int device = 0;
    hipStream_t stream = nullptr, own_stream = nullptr;
    sdr::Buf prev_vis, prev_depth, zrange, stats, ab, stage_in, stage_out, stage_left, stage_vis, stage_zr;
    int vis_w = 0, vis_h = 0;      // prev_vis size (0 = empty)
    int depth_w = 0, depth_h = 0;  // prev_depth_vis size
    sdr::Lut turbo{}, jet{};
    double zinit[2] = {1000.0, 2000.0};
};

namespace {
int dfail(int code, const char* msg) { return sdr::set_error(code, msg); }
#define SDR_DHIP(call)                                                              \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) return dfail(SDR_ERR_DEVICE, hipGetErrorString(e_)); \
    } while (0)

// static double zmin_smooth = 1000.0, zmax_smooth = 2000.0: the copy is ordered on the handle's
// current stream, from memory the handle owns (a pageable source may be read after the call)
int reset_zrange(sdr_display* h) {
    SDR_DHIP(hipMemcpyAsync(h->zrange.p, h->zinit, sizeof(h->zinit), hipMemcpyHostToDevice, h->stream));
    return SDR_OK;
}

sdr::Lut lut_or(const uint8_t* user, const sdr::Lut& dflt) {
    if (!user) return dflt;
    sdr::Lut l;
    std::memcpy(l.v, user, 768);
    return l;
}

// the shared part of show_depthMap: stats -> range recurrence -> TURBO + EMA
int depth_map(sdr_display* h, const float* d_xyz, int W, int H, int channels, int F, double* d_zr,
              const uint8_t* lut, uint8_t* d_out, int col0) {
    int rc;
    const size_t px = (size_t)W * H;
    if ((rc = sdr::ensure(h->stats, (size_t)F * sizeof(sdr::ZStats)))) return rc;
    if ((rc = sdr::ensure(h->ab, (size_t)F * sizeof(float2)))) return rc;
    const bool same = h->depth_w == W && h->depth_h == H;
    if (!same) {
        if ((rc = sdr::ensure(h->prev_depth, px * 3))) return rc;
    }
    sdr::ZStats* st = (sdr::ZStats*)h->stats.p;
    hipLaunchKernelGGL(sdr::k_zstats_init, dim3((F + 63) / 64), dim3(64), 0, h->stream, st, F);
    hipLaunchKernelGGL(sdr::k_zstats, dim3((W + 255) / 256, H, F), dim3(256), 0, h->stream, d_xyz, channels,
                       W, H, col0, st);
    hipLaunchKernelGGL(sdr::k_zrange, dim3(1), dim3(64), 0, h->stream, st, F,
                       d_zr ? d_zr : (double*)h->zrange.p, (float2*)h->ab.p);
    if (d_out) {
        hipLaunchKernelGGL(sdr::k_depth_vis, dim3((W + 255) / 256, H), dim3(256), 0, h->stream, d_xyz,
                           channels, W, H, F, (const float2*)h->ab.p, lut_or(lut, h->turbo),
                           (uint8_t*)h->prev_depth.p, same ? 1 : 0, d_out);
        h->depth_w = W;
        h->depth_h = H;
    }
    SDR_DHIP(hipGetLastError());
    return SDR_OK;
}

int read_coverage(sdr_display* h, int W, int H, int F, double* pct) {
    if (!pct) return SDR_OK;
    sdr::ZStats tmp[64];
    for (int f0 = 0; f0 < F; f0 += 64) {
        const int n = F - f0 < 64 ? F - f0 : 64;
        SDR_DHIP(hipMemcpyAsync(tmp, (sdr::ZStats*)h->stats.p + f0, n * sizeof(sdr::ZStats),
                                hipMemcpyDeviceToHost, h->stream));
        SDR_DHIP(hipStreamSynchronize(h->stream));
        for (int k = 0; k < n; k++) pct[f0 + k] = ((double)tmp[k].count / ((double)W * H)) * 100;
    }
    return SDR_OK;
}
}  // namespace

extern "C" {

int sdr_colormap_lut(int colormap, uint8_t* lut_bgr) {
    if (!lut_bgr) return dfail(SDR_ERR_ARG, "null argument");
    return sdr::colormap_lut(colormap, lut_bgr) ? dfail(SDR_ERR_ARG, "unknown colormap") : SDR_OK;
}

int sdr_display_create(int device, sdr_display** out) {
    if (!out) return dfail(SDR_ERR_ARG, "null argument");
    *out = nullptr;
    int ndev = 0;
    SDR_DHIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return dfail(SDR_ERR_DEVICE, "invalid device index");
    SDR_DHIP(hipSetDevice(device));
    sdr_display* h = new sdr_display();
    h->device = device;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return dfail(SDR_ERR_DEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    sdr::colormap_lut(SDR_COLORMAP_TURBO, h->turbo.v);
    sdr::colormap_lut(SDR_COLORMAP_JET, h->jet.v);
    int rc = sdr::ensure(h->zrange, 2 * sizeof(double));
    // blocking copy: later work may run on any stream the caller sets
    if (!rc && hipMemcpy(h->zrange.p, h->zinit, sizeof(h->zinit), hipMemcpyHostToDevice) != hipSuccess)
        rc = dfail(SDR_ERR_DEVICE, "hipMemcpy failed");
    if (rc) {
        sdr_display_destroy(h);
        return rc;
    }
    *out = h;
    return SDR_OK;
}

int sdr_display_destroy(sdr_display* h) {
    if (!h) return SDR_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (sdr::Buf* b : {&h->prev_vis, &h->prev_depth, &h->zrange, &h->stats, &h->ab, &h->stage_in,
                        &h->stage_out, &h->stage_left, &h->stage_vis, &h->stage_zr})
        if (b->p) (void)hipFree(b->p);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return SDR_OK;
}

int sdr_display_set_stream(sdr_display* h, void* stream) {
    if (!h) return dfail(SDR_ERR_ARG, "null handle");
    h->stream = (hipStream_t)stream;  // NULL = the HIP null stream (torch's default stream)
    return SDR_OK;
}

int sdr_display_reset_stream(sdr_display* h) {
    if (!h) return dfail(SDR_ERR_ARG, "null handle");
    h->stream = h->own_stream;
    return SDR_OK;
}

int sdr_display_reset(sdr_display* h) {
    if (!h) return dfail(SDR_ERR_ARG, "null handle");
    (void)hipSetDevice(h->device);
    h->vis_w = h->vis_h = h->depth_w = h->depth_h = 0;
    return reset_zrange(h);
}

int sdr_show_disparity_map_device(sdr_display* h, const float* d_disp, int W, int H, size_t stride,
                                  size_t frame_stride, int F, int num_disparities, uint8_t* d_vis) {
    if (!h || !d_disp || !d_vis) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0 || stride < (size_t)W) return dfail(SDR_ERR_ARG, "bad size");
    SDR_DHIP(hipSetDevice(h->device));
    const bool same = h->vis_w == W && h->vis_h == H;
    int rc;
    if (!same && (rc = sdr::ensure(h->prev_vis, (size_t)W * H))) return rc;
    // 1.0f / std::max(1, numDisp) in float, then convertTo's (float) scale
    const float scale = 1.0f / (float)(num_disparities > 1 ? num_disparities : 1);
    hipLaunchKernelGGL(sdr::k_disp_vis, dim3((W + 255) / 256, H), dim3(256), 0, h->stream, d_disp, stride,
                       F > 1 ? frame_stride : 0, W, H, F, scale, (uint8_t*)h->prev_vis.p, same ? 1 : 0, d_vis);
    h->vis_w = W;
    h->vis_h = H;
    SDR_DHIP(hipGetLastError());
    return SDR_OK;
}

int sdr_show_depth_map_device(sdr_display* h, const float* d_xyz, int W, int H, int channels, int F,
                              double* d_zrange, const uint8_t* lut_bgr, uint8_t* d_bgr,
                              double* coverage_pct) {
    if (!h || !d_xyz || !d_bgr) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0) return dfail(SDR_ERR_ARG, "bad size");
    if (channels != 1 && channels != 3) return dfail(SDR_ERR_TYPE, "depth must have 1 or 3 channels");
    SDR_DHIP(hipSetDevice(h->device));
    int rc = depth_map(h, d_xyz, W, H, channels, F, d_zrange, lut_bgr, d_bgr, 80);
    if (rc) return rc;
    return read_coverage(h, W, H, F, coverage_pct);
}

int sdr_depth_coverage_device(sdr_display* h, const float* d_xyz, int W, int H, int F, int col0,
                              double* pct) {
    if (!h || !d_xyz || !pct) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0) return dfail(SDR_ERR_ARG, "bad size");
    SDR_DHIP(hipSetDevice(h->device));
    int rc;
    if ((rc = sdr::ensure(h->stats, (size_t)F * sizeof(sdr::ZStats)))) return rc;
    sdr::ZStats* st = (sdr::ZStats*)h->stats.p;
    hipLaunchKernelGGL(sdr::k_zstats_init, dim3((F + 63) / 64), dim3(64), 0, h->stream, st, F);
    hipLaunchKernelGGL(sdr::k_zstats, dim3((W + 255) / 256, H, F), dim3(256), 0, h->stream, d_xyz, 3, W, H,
                       col0, st);
    SDR_DHIP(hipGetLastError());
    return read_coverage(h, W, H, F, pct);
}

int sdr_disparity_overlay_device(sdr_display* h, const uint8_t* d_vis, const uint8_t* d_left_bgr,
                                 size_t left_stride, size_t left_frame_stride, int W, int H, int F,
                                 const uint8_t* lut_bgr, uint8_t* d_heat, uint8_t* d_overlay) {
    if (!h || !d_vis || (!d_heat && !d_overlay) || (d_overlay && !d_left_bgr))
        return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0) return dfail(SDR_ERR_ARG, "bad size");
    if (d_left_bgr && left_stride < (size_t)W * 6) return dfail(SDR_ERR_ARG, "left_stride < 3 * (2 * width)");
    SDR_DHIP(hipSetDevice(h->device));
    hipLaunchKernelGGL(sdr::k_overlay, dim3((W + 255) / 256, H, F), dim3(256), 0, h->stream, d_vis,
                       d_left_bgr, left_stride, left_frame_stride ? left_frame_stride : left_stride * 2 * H,
                       W, H, lut_or(lut_bgr, h->jet), d_heat, d_overlay);
    SDR_DHIP(hipGetLastError());
    return SDR_OK;
}

// ---- host-pointer versions (the C++ facade's cv::Mat-style calls; synchronous) ----

int sdr_show_disparity_map(sdr_display* h, const float* disp, int W, int H, size_t stride,
                           int num_disparities, uint8_t* out, size_t out_stride) {
    if (!h || !disp || !out) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || stride < (size_t)W || out_stride < (size_t)W) return dfail(SDR_ERR_ARG, "bad size");
    SDR_DHIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = sdr::ensure(h->stage_in, px * 4)) || (rc = sdr::ensure(h->stage_vis, px))) return rc;
    SDR_DHIP(hipMemcpy2DAsync(h->stage_in.p, W * 4, disp, stride * 4, W * 4, H, hipMemcpyHostToDevice, h->stream));
    if ((rc = sdr_show_disparity_map_device(h, (const float*)h->stage_in.p, W, H, W, px, 1, num_disparities,
                                            (uint8_t*)h->stage_vis.p)))
        return rc;
    SDR_DHIP(hipMemcpy2DAsync(out, out_stride, h->stage_vis.p, W, W, H, hipMemcpyDeviceToHost, h->stream));
    SDR_DHIP(hipStreamSynchronize(h->stream));
    return SDR_OK;
}

int sdr_show_depth_map(sdr_display* h, const float* xyz, int W, int H, int channels, double* zrange,
                       uint8_t* out_bgr, double* coverage_pct) {
    if (!h || !xyz || !out_bgr) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0) return dfail(SDR_ERR_ARG, "bad size");
    if (channels != 1 && channels != 3) return dfail(SDR_ERR_TYPE, "depth must have 1 or 3 channels");
    SDR_DHIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = sdr::ensure(h->stage_in, px * 4 * channels)) || (rc = sdr::ensure(h->stage_out, px * 3)) ||
        (rc = sdr::ensure(h->stage_zr, 2 * sizeof(double))))
        return rc;
    double* dzr = nullptr;
    SDR_DHIP(hipMemcpyAsync(h->stage_in.p, xyz, px * 4 * channels, hipMemcpyHostToDevice, h->stream));
    if (zrange) {  // caller-owned range state (the reference's function-static doubles)
        dzr = (double*)h->stage_zr.p;
        SDR_DHIP(hipMemcpyAsync(dzr, zrange, 2 * sizeof(double), hipMemcpyHostToDevice, h->stream));
    }
    if ((rc = sdr_show_depth_map_device(h, (const float*)h->stage_in.p, W, H, channels, 1, dzr, nullptr,
                                        (uint8_t*)h->stage_out.p, coverage_pct)))
        return rc;
    SDR_DHIP(hipMemcpyAsync(out_bgr, h->stage_out.p, px * 3, hipMemcpyDeviceToHost, h->stream));
    if (zrange) SDR_DHIP(hipMemcpyAsync(zrange, dzr, 2 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SDR_DHIP(hipStreamSynchronize(h->stream));
    return SDR_OK;
}

int sdr_depth_coverage(sdr_display* h, const float* xyz, int W, int H, int col0, double* pct) {
    if (!h || !xyz || !pct) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0) return dfail(SDR_ERR_ARG, "bad size");
    SDR_DHIP(hipSetDevice(h->device));
    int rc;
    if ((rc = sdr::ensure(h->stage_in, (size_t)W * H * 12))) return rc;
    SDR_DHIP(hipMemcpyAsync(h->stage_in.p, xyz, (size_t)W * H * 12, hipMemcpyHostToDevice, h->stream));
    // statistics only: the handle's EMA history and range state are not touched
    return sdr_depth_coverage_device(h, (const float*)h->stage_in.p, W, H, 1, col0, pct);
}

int sdr_disparity_overlay(sdr_display* h, const uint8_t* vis, const uint8_t* left_bgr, size_t left_stride,
                          int W, int H, uint8_t* heat, uint8_t* overlay) {
    if (!h || !vis || !left_bgr || (!heat && !overlay)) return dfail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || left_stride < (size_t)W * 6) return dfail(SDR_ERR_ARG, "bad size");
    SDR_DHIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    int rc;
    if ((rc = sdr::ensure(h->stage_vis, px)) || (rc = sdr::ensure(h->stage_left, px * 12)) ||
        (rc = sdr::ensure(h->stage_out, px * 6)))
        return rc;
    uint8_t* dh = (uint8_t*)h->stage_out.p;
    uint8_t* dov = dh + px * 3;
    SDR_DHIP(hipMemcpyAsync(h->stage_vis.p, vis, px, hipMemcpyHostToDevice, h->stream));
    SDR_DHIP(hipMemcpy2DAsync(h->stage_left.p, (size_t)W * 6, left_bgr, left_stride, (size_t)W * 6, 2 * H,
                              hipMemcpyHostToDevice, h->stream));
    if ((rc = sdr_disparity_overlay_device(h, (const uint8_t*)h->stage_vis.p, (const uint8_t*)h->stage_left.p,
                                           (size_t)W * 6, 0, W, H, 1, nullptr, dh, dov)))
        return rc;
    if (heat) SDR_DHIP(hipMemcpyAsync(heat, dh, px * 3, hipMemcpyDeviceToHost, h->stream));
    if (overlay) SDR_DHIP(hipMemcpyAsync(overlay, dov, px * 3, hipMemcpyDeviceToHost, h->stream));
    SDR_DHIP(hipStreamSynchronize(h->stream));
    return SDR_OK;
}

}  // extern "C"
