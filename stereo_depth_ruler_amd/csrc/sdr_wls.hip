// sdr_wls.hip -- the class path's post-filter on the GPU:
//   cv::ximgproc::createDisparityWLSFilter(matcher)    stereo_vision/src/stereo_disparity.cpp:11-13
//   wls_filter->filter(disp_left, left_small, filtered, disp_right)               :31
//   wls_filter->getConfidenceMap()                                                :36
// restating opencv_contrib 4.6 ximgproc disparity_filters.cpp + fgs_filter.cpp as the oracle
// does (oracle/wls_oracle.c, the checker; parity against OpenCV itself is unpinned there).
//
// Kernels (all float work with contraction off and IEEE division, so every rounding matches the
// oracle's operation order bit for bit; the FGS weight table is computed once on the host with
// the same expf the oracle uses):
//   k_wls_disc     depth-discontinuity map of the RIGHT view over its ROI: 1 - roll_off * var
//                  of a (2r+1)^2 box, BORDER_REFLECT_101 inside the ROI, sums in int64/double
//   k_wls_conf     left discontinuity (inline) + discontinuity-aware LR check -> confidence
//                  x255 (full map for getConfidenceMap) and the two FGS inputs conf*d, conf,
//                  compacted to the ROI
//   k_fgs_lines    one FGS pass (rows or columns) = one tridiagonal Thomas solve per line for
//                  BOTH inputs at once (the elimination coefficients depend only on the guide
//                  and lambda).  A wave owns 64 lines; the lines are walked in 64-element chunks
//                  staged through LDS with coalesced loads (rows and columns alike), so the
//                  serial per-line recurrence reads LDS, never HBM
//   k_wls_final    FGS(conf*d) / FGS(conf) -> saturate_cast<short>, 16*(min_disp-1) outside ROI
#include "../../include/sdr/sdr.h"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#pragma clang fp contract(off)

namespace sdr {

constexpr int kFgsLevels = 65026;  // 255^2 + 1 squared differences of two 8-bit gray levels

__device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

// 1 - roll_off * (boxmean(d^2) - boxmean(d)^2), clamped at 0, at ROI pixel (i, j) of map d
// (ComputeDepthDisc: convertTo(CV_32F), multiply, boxFilter(CV_32F) x2 with double row sums)
__device__ __forceinline__ float disc_at(const int16_t* __restrict__ d, int W, int rx, int ry,
                                         int rw, int rh, int i, int j, int radius, double scale,
                                         float roll_off) {
    long long s = 0, s2 = 0;
    for (int a = -radius; a <= radius; a++) {
        const int ii = reflect101(i + a, rh);
        const int16_t* row = d + (size_t)(ry + ii) * W + rx;
        for (int b = -radius; b <= radius; b++) {
            const long long v = row[reflect101(j + b, rw)];
            s += v;
            s2 += v * v;
        }
    }
    const float mean = (float)((double)s * scale);
    const float msq = (float)((double)s2 * scale);
    const float var = msq - mean * mean;
    const float c = 1.0f - roll_off * var;
    return c > 0.0f ? c : 0.0f;
}

struct WlsGeom {
    int W, H;
    int rx, ry, rw, rh;      // left ROI
    int rrx;                 // right ROI x (same y, w, h)
    int radius;
    double scale;            // 1 / (2r+1)^2
    float roll_off;
    int lrc_thresh;
    int fill;                // 16 * (min_disp - 1)
};

__global__ __launch_bounds__(256) void k_wls_disc(const int16_t* __restrict__ dr, WlsGeom g,
                                                  float* __restrict__ rdisc) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (j >= g.rw || i >= g.rh) return;
    const size_t fo = (size_t)blockIdx.z * g.W * g.H;
    rdisc[fo + (size_t)(g.ry + i) * g.W + g.rrx + j] =
        disc_at(dr + fo, g.W, g.rrx, g.ry, g.rw, g.rh, i, j, g.radius, g.scale, g.roll_off);
}

// ComputeDiscontinuityAwareLRC + confidence_map = 255 * map; A = conf * d, B = conf (ROI-compact)
__global__ __launch_bounds__(256) void k_wls_conf(const int16_t* __restrict__ dl,
                                                  const int16_t* __restrict__ dr,
                                                  const float* __restrict__ rdisc, WlsGeom g,
                                                  float* __restrict__ conf_full,
                                                  float* __restrict__ A, float* __restrict__ B) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const size_t fo = (size_t)blockIdx.z * g.W * g.H;
    const size_t o = fo + (size_t)y * g.W + x;
    const int j = x - g.rx, i = y - g.ry;
    const bool in_roi = j >= 0 && j < g.rw && i >= 0 && i < g.rh;
    float c = 1.0f;
    int v = 0;
    if (in_roi) {
        c = disc_at(dl + fo, g.W, g.rx, g.ry, g.rw, g.rh, i, j, g.radius, g.scale, g.roll_off);
        v = dl[o];
        const int ridx = x - (v >> 4);
        if (ridx >= g.rrx && ridx < g.rrx + g.rw) {
            const size_t ro = fo + (size_t)y * g.W + ridx;
            if (abs(v + (int)dr[ro]) < g.lrc_thresh) {
                const float rc = rdisc[ro];
                c = c < rc ? c : rc;
            } else {
                c = 0.0f;
            }
        }
    }
    const float conf = 255.0f * c;
    if (conf_full) conf_full[o] = conf;
    if (in_roi) {
        const size_t co = (size_t)blockIdx.z * g.rw * g.rh + (size_t)i * g.rw + j;
        A[co] = conf * (float)v;
        B[co] = conf;
    }
}

// FGS line solve, per line of n samples with weights C[k] = lut[(g[k] - g[k+1])^2] (0 at the
// last sample):  (1 - lam*(C[k-1] + C[k])) u_k + lam*C[k-1] u_{k-1} + lam*C[k] u_{k+1} = f_k
// (C = -w <= 0), Thomas forward elimination then back substitution, in the oracle's order:
//   k=0:  den = 1 - lam*C0;  t0 = lam*C0 / den;  u0 = u0 / den
//   k>0:  a = lam*C[k-1];  c = lam*C[k];  den = (1 - c) - a*(1 + t[k-1]);
//         t[k] = c / den;  u_k = (u_k - a*u_{k-1}) / den
//   back: u_k = u_k - t[k]*u_{k+1}
// ROWS: line l = row l (element k at l*pitch + k); else line l = column l (element at k*pitch + l).
constexpr int kChunk = 64;
constexpr int kTilePitch = kChunk + 1;  // conflict-free row reads of the [line][k] tile

template <bool ROWS>
__global__ __launch_bounds__(64) void k_fgs_lines(const uint8_t* __restrict__ guide,
                                                  size_t gstride, size_t gfstride,
                                                  const float* __restrict__ lut, float* U0,
                                                  float* U1, float* T, int nimg, int w, int h,
                                                  float lam) {
    __shared__ float sU0[kChunk * kTilePitch];
    __shared__ float sU1[kChunk * kTilePitch];
    // the weights C[k] and the coefficients t[k] share a tile: iteration k reads C[k], then
    // writes t[k] over it
    __shared__ float sT[kChunk * kTilePitch];
    float* sC = sT;
    const int lane = threadIdx.x;
    const int nlines = ROWS ? h : w;
    const int n = ROWS ? w : h;
    const int l0 = blockIdx.x * kChunk;
    const int f = blockIdx.y;
    const uint8_t* gf = guide + (size_t)f * gfstride;
    const size_t fo = (size_t)f * w * h;
    float* u0 = U0 + fo;
    float* u1 = nimg > 1 ? U1 + fo : nullptr;
    float* t = T + fo;
    const int nl = min(kChunk, nlines - l0);
    auto eidx = [&](int l, int k) -> size_t {
        return ROWS ? (size_t)l * w + k : (size_t)k * w + l;
    };
    auto gval = [&](int l, int k) -> int {
        return ROWS ? gf[(size_t)l * gstride + k] : gf[(size_t)k * gstride + l];
    };
    const bool active = lane < nl;
    // forward elimination, chunk by chunk
    float cprev = 0.0f, tprev = 0.0f, p0 = 0.0f, p1 = 0.0f;
    for (int k0 = 0; k0 < n; k0 += kChunk) {
        const int nk = min(kChunk, n - k0);
        // stage U (and C) tiles [line][k]: each pass loads 64 consecutive addresses
        for (int r = 0; r < kChunk; r++) {
            int l, k;
            if (ROWS) { l = r; k = lane; } else { l = lane; k = r; }
            if (l < nl && k < nk) {
                const int gl = l0 + l, gk = k0 + k;
                const size_t e = eidx(gl, gk);
                sU0[l * kTilePitch + k] = u0[e];
                if (u1) sU1[l * kTilePitch + k] = u1[e];
                float cw = 0.0f;
                if (gk + 1 < n) {
                    const int dv = gval(gl, gk) - gval(gl, gk + 1);
                    cw = lut[dv * dv];
                }
                sC[l * kTilePitch + k] = cw;
            }
        }
        __syncthreads();
        if (active) {
            float* r0 = sU0 + lane * kTilePitch;
            float* r1 = sU1 + lane * kTilePitch;
            float* rt = sT + lane * kTilePitch;
            const float* rc = sC + lane * kTilePitch;
            int k = 0;
            if (k0 == 0) {
                cprev = rc[0];
                const float c0 = lam * cprev;
                const float den = 1.0f - c0;
                tprev = c0 / den;
                rt[0] = tprev;
                p0 = r0[0] / den;
                r0[0] = p0;
                if (u1) { p1 = r1[0] / den; r1[0] = p1; }
                k = 1;
            }
            for (; k < nk; k++) {
                const float a = lam * cprev;
                const float ck = rc[k];
                const float c = lam * ck;
                const float den = (1.0f - c) - a * (1.0f + tprev);
                tprev = c / den;
                rt[k] = tprev;
                p0 = (r0[k] - a * p0) / den;
                r0[k] = p0;
                if (u1) { p1 = (r1[k] - a * p1) / den; r1[k] = p1; }
                cprev = ck;
            }
        }
        __syncthreads();
        for (int r = 0; r < kChunk; r++) {
            int l, k;
            if (ROWS) { l = r; k = lane; } else { l = lane; k = r; }
            if (l < nl && k < nk) {
                const size_t e = eidx(l0 + l, k0 + k);
                u0[e] = sU0[l * kTilePitch + k];
                if (u1) u1[e] = sU1[l * kTilePitch + k];
                t[e] = sT[l * kTilePitch + k];
            }
        }
        __syncthreads();
    }
    // back substitution, chunks in reverse (the last chunk is re-read from L2)
    float q0 = 0.0f, q1 = 0.0f;
    const int last0 = ((n - 1) / kChunk) * kChunk;
    for (int k0 = last0; k0 >= 0; k0 -= kChunk) {
        const int nk = min(kChunk, n - k0);
        for (int r = 0; r < kChunk; r++) {
            int l, k;
            if (ROWS) { l = r; k = lane; } else { l = lane; k = r; }
            if (l < nl && k < nk) {
                const size_t e = eidx(l0 + l, k0 + k);
                sU0[l * kTilePitch + k] = u0[e];
                if (u1) sU1[l * kTilePitch + k] = u1[e];
                sT[l * kTilePitch + k] = t[e];
            }
        }
        __syncthreads();
        if (active) {
            float* r0 = sU0 + lane * kTilePitch;
            float* r1 = sU1 + lane * kTilePitch;
            const float* rt = sT + lane * kTilePitch;
            int k = nk - 1;
            if (k0 + k == n - 1) {  // the last sample keeps its forward value
                q0 = r0[k];
                if (u1) q1 = r1[k];
                k--;
            }
            for (; k >= 0; k--) {
                q0 = r0[k] - rt[k] * q0;
                r0[k] = q0;
                if (u1) { q1 = r1[k] - rt[k] * q1; r1[k] = q1; }
            }
        }
        __syncthreads();
        for (int r = 0; r < kChunk; r++) {
            int l, k;
            if (ROWS) { l = r; k = lane; } else { l = lane; k = r; }
            if (l < nl && k < nk) {
                const size_t e = eidx(l0 + l, k0 + k);
                u0[e] = sU0[l * kTilePitch + k];
                if (u1) u1[e] = sU1[l * kTilePitch + k];
            }
        }
        __syncthreads();
    }
}

// saturate_cast<short>(float): round half to even, saturate; 0 where FGS(conf) == 0 (cv::divide
// of floats returns 0 for a zero divisor)
__global__ __launch_bounds__(256) void k_wls_final(const float* __restrict__ A,
                                                   const float* __restrict__ B, WlsGeom g,
                                                   int16_t* __restrict__ out) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const size_t o = (size_t)blockIdx.z * g.W * g.H + (size_t)y * g.W + x;
    const int j = x - g.rx, i = y - g.ry;
    int16_t r = (int16_t)g.fill;
    if (j >= 0 && j < g.rw && i >= 0 && i < g.rh) {
        const size_t co = (size_t)blockIdx.z * g.rw * g.rh + (size_t)i * g.rw + j;
        const float c = B[co];
        const float v = c != 0.0f ? A[co] / c : 0.0f;
        // cvRound (cvtss2si): NaN / |v| >= 2^31 give INT_MIN, which saturates to -32768
        float q = rintf(v);
        q = fminf(fmaxf(q, -32768.0f), 32767.0f);
        r = fabsf(v) < 2147483648.0f ? (int16_t)(int)q : (int16_t)-32768;
    }
    out[o] = r;
}

static void launch_fgs(const uint8_t* guide, size_t gstride, size_t gfstride, const float* lut,
                       float* U0, float* U1, float* T, int nimg, int w, int h, int F,
                       double lambda, double att, int iters, hipStream_t st) {
    float lam = (float)lambda;
    const float fa = (float)att;
    for (int it = 0; it < iters; it++) {
        hipLaunchKernelGGL(k_fgs_lines<true>, dim3((h + kChunk - 1) / kChunk, F), dim3(64), 0, st,
                           guide, gstride, gfstride, lut, U0, U1, T, nimg, w, h, lam);
        hipLaunchKernelGGL(k_fgs_lines<false>, dim3((w + kChunk - 1) / kChunk, F), dim3(64), 0, st,
                           guide, gstride, gfstride, lut, U0, U1, T, nimg, w, h, lam);
        lam = lam * fa;  // FastGlobalSmootherFilterImpl::filter: lambda *= lambda_attenuation
    }
}

// ComputeLUT_ParBody: LUT[i] = -exp(-sqrt((float)i) / sigmaColor), float math on the host
static void fgs_lut_host(double sigma, std::vector<float>* lut) {
    lut->resize(kFgsLevels);
    const float s = (float)sigma;
    for (int i = 0; i < kFgsLevels; i++) (*lut)[i] = -expf(-sqrtf((float)i) / s);
}

}  // namespace sdr

// ===========================================================================================
// C ABI (include/sdr/sdr.h)
// ===========================================================================================
struct sdr_wls {
    sdr_wls_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    sdr::Buf rdisc, conf, A, B, T, lut, out, hbuf;
    double lut_sigma = -1.0;
};

namespace {

#define WLS_HIP(call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return sdr::set_error(SDR_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

int check_wls_params(const sdr_wls_params& p) {
    if (!(p.lambda >= 0.0) || !(p.sigma_color >= 0.0) || p.num_iter < 1)
        return sdr::set_error(SDR_ERR_ARG, "FGS needs lambda >= 0, sigma_color >= 0, num_iter >= 1");
    if (p.depth_discontinuity_radius < 0 || p.left_offset < 0 || p.right_offset < 0 ||
        p.top_offset < 0 || p.bottom_offset < 0)
        return sdr::set_error(SDR_ERR_ARG, "negative WLS radius or offset");
    return SDR_OK;
}

int upload_lut(sdr_wls* h, double sigma, const float** out) {
    int rc;
    if ((rc = sdr::ensure(h->lut, sizeof(float) * sdr::kFgsLevels))) return rc;
    if (h->lut_sigma != sigma) {
        std::vector<float> lut;
        sdr::fgs_lut_host(sigma, &lut);
        WLS_HIP(hipMemcpy(h->lut.p, lut.data(), sizeof(float) * lut.size(), hipMemcpyHostToDevice));
        h->lut_sigma = sigma;
    }
    *out = (const float*)h->lut.p;
    return SDR_OK;
}

}  // namespace

extern "C" {

void sdr_wls_params_for_sgbm(sdr_sgbm_params* m, sdr_wls_params* p) {
    if (!m || !p) return;
    // createDisparityWLSFilter(Ptr<StereoMatcher>) [ximgproc disparity_filters.cpp]:
    // setDisp12MaxDiff(1000000), setSpeckleWindowSize(0), and for SGBM setUniquenessRatio(0);
    // offsets (max(0, minD+numD), max(0, -minD), 0, 0); radius ceil(0.5 * blockSize)
    m->disp12MaxDiff = 1000000;
    m->speckleWindowSize = 0;
    m->uniquenessRatio = 0;
    const int l = m->minDisparity + m->numDisparities;
    p->lambda = 8000.0;
    p->sigma_color = 1.5;
    p->lrc_thresh = 24;
    p->depth_discontinuity_radius = (int)std::ceil(0.5 * m->blockSize);
    p->roll_off = 0.001f;
    p->lambda_attenuation = 0.25;
    p->num_iter = 3;
    p->left_offset = l > 0 ? l : 0;
    p->right_offset = m->minDisparity < 0 ? -m->minDisparity : 0;
    p->top_offset = 0;
    p->bottom_offset = 0;
    p->min_disp = m->minDisparity;
}

int sdr_wls_create(const sdr_wls_params* p, int device, sdr_wls** out) {
    if (!p || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    int rc = check_wls_params(*p);
    if (rc) return rc;
    WLS_HIP(hipSetDevice(device));
    sdr_wls* h = new sdr_wls();
    h->p = *p;
    h->device = device;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return sdr::set_error(SDR_ERR_DEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    *out = h;
    return SDR_OK;
}

int sdr_wls_destroy(sdr_wls* h) {
    if (!h) return SDR_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (sdr::Buf* b : {&h->rdisc, &h->conf, &h->A, &h->B, &h->T, &h->lut, &h->out, &h->hbuf})
        if (b->p) (void)hipFree(b->p);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return SDR_OK;
}

int sdr_wls_set_params(sdr_wls* h, const sdr_wls_params* p) {
    if (!h || !p) return sdr::set_error(SDR_ERR_ARG, "null argument");
    int rc = check_wls_params(*p);
    if (rc) return rc;
    h->p = *p;
    return SDR_OK;
}

int sdr_wls_get_params(const sdr_wls* h, sdr_wls_params* p) {
    if (!h || !p) return sdr::set_error(SDR_ERR_ARG, "null argument");
    *p = h->p;
    return SDR_OK;
}

int sdr_wls_set_stream(sdr_wls* h, void* stream) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = (hipStream_t)stream;  // NULL = the HIP null (legacy default) stream
    return SDR_OK;
}

int sdr_wls_reset_stream(sdr_wls* h) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = h->own_stream;
    return SDR_OK;
}

void* sdr_wls_get_stream(const sdr_wls* h) { return h ? (void*)h->stream : nullptr; }

int sdr_wls_get_roi(const sdr_wls* h, int W, int H, int roi[4]) {
    if (!h || !roi) return sdr::set_error(SDR_ERR_ARG, "null argument");
    roi[0] = h->p.left_offset;
    roi[1] = h->p.top_offset;
    roi[2] = W - h->p.left_offset - h->p.right_offset;
    roi[3] = H - h->p.top_offset - h->p.bottom_offset;
    return SDR_OK;
}

int sdr_wls_filter_device(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide,
                          int W, int H, size_t gstride, size_t gfstride, int F, int16_t* out,
                          float* conf) {
    if (!h || !dl || !dr || !guide || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0 || gstride < (size_t)W || (F > 1 && gfstride < gstride * H))
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    WLS_HIP(hipSetDevice(h->device));
    hipStream_t st = h->stream;
    const sdr_wls_params& p = h->p;
    sdr::WlsGeom g{};
    g.W = W;
    g.H = H;
    g.rx = p.left_offset;
    g.ry = p.top_offset;
    g.rw = W - p.left_offset - p.right_offset;
    g.rh = H - p.top_offset - p.bottom_offset;
    g.rrx = W - (g.rx + g.rw);
    g.radius = p.depth_discontinuity_radius;
    const int k = 2 * g.radius + 1;
    g.scale = 1.0 / (double)(k * k);
    g.roll_off = p.roll_off;
    g.lrc_thresh = p.lrc_thresh;
    g.fill = 16 * (p.min_disp - 1);
    const size_t px = (size_t)W * H;
    const bool roi = g.rw > 0 && g.rh > 0;
    const size_t cpx = roi ? (size_t)g.rw * g.rh : 0;
    int rc;
    const float* lut = nullptr;
    if ((rc = sdr::ensure(h->rdisc, F * px * 4))) return rc;
    if ((rc = sdr::ensure(h->A, F * cpx * 4 + 4))) return rc;
    if ((rc = sdr::ensure(h->B, F * cpx * 4 + 4))) return rc;
    if ((rc = sdr::ensure(h->T, F * cpx * 4 + 4))) return rc;
    if ((rc = upload_lut(h, p.sigma_color, &lut))) return rc;
    float* A = (float*)h->A.p;
    float* B = (float*)h->B.p;
    const dim3 blk(256);
    if (roi) {
        hipLaunchKernelGGL(sdr::k_wls_disc, dim3((g.rw + 63) / 64, (g.rh + 3) / 4, F), blk, 0, st,
                           dr, g, (float*)h->rdisc.p);
    }
    const dim3 grid((W + 63) / 64, (H + 3) / 4, F);
    hipLaunchKernelGGL(sdr::k_wls_conf, grid, blk, 0, st, dl, dr, (const float*)h->rdisc.p, g,
                       conf, A, B);
    if (roi) {
        const uint8_t* g0 = guide + (size_t)g.ry * gstride + g.rx;
        sdr::launch_fgs(g0, gstride, gfstride, lut, A, B, (float*)h->T.p, 2, g.rw, g.rh, F,
                        p.lambda, p.lambda_attenuation, p.num_iter, st);
    }
    hipLaunchKernelGGL(sdr::k_wls_final, grid, blk, 0, st, A, B, g, out);
    WLS_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_wls_filter(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide, int W,
                   int H, size_t gstride, int16_t* out, float* conf) {
    if (!h || !dl || !dr || !guide || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || gstride < (size_t)W) return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    WLS_HIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    // device staging: dl, dr, guide, out (int16), conf (float)
    int rc;
    if ((rc = sdr::ensure(h->hbuf, px * (2 + 2 + 1 + 2 + 4) + 64))) return rc;
    uint8_t* base = (uint8_t*)h->hbuf.p;
    float* dconf = (float*)base;
    int16_t* ddl = (int16_t*)(base + px * 4);
    int16_t* ddr = ddl + px;
    int16_t* dout = ddr + px;
    uint8_t* dg = (uint8_t*)(dout + px);
    hipStream_t st = h->stream;
    WLS_HIP(hipMemcpyAsync(ddl, dl, px * 2, hipMemcpyHostToDevice, st));
    WLS_HIP(hipMemcpyAsync(ddr, dr, px * 2, hipMemcpyHostToDevice, st));
    WLS_HIP(hipMemcpy2DAsync(dg, W, guide, gstride, W, H, hipMemcpyHostToDevice, st));
    if ((rc = sdr_wls_filter_device(h, ddl, ddr, dg, W, H, W, px, 1, dout, conf ? dconf : nullptr)))
        return rc;
    WLS_HIP(hipMemcpyAsync(out, dout, px * 2, hipMemcpyDeviceToHost, st));
    if (conf) WLS_HIP(hipMemcpyAsync(conf, dconf, px * 4, hipMemcpyDeviceToHost, st));
    WLS_HIP(hipStreamSynchronize(st));
    return SDR_OK;
}

int sdr_fgs_filter_device(const uint8_t* d_guide, size_t gstride, int w, int h, double lambda,
                          double sigma, double att, int iters, float* d_img, int nimg,
                          void* stream) {
    if (!d_guide || !d_img) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (w <= 0 || h <= 0 || nimg <= 0 || gstride < (size_t)w)
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    if (!(lambda >= 0.0) || !(sigma >= 0.0) || iters < 1)
        return sdr::set_error(SDR_ERR_ARG, "FGS needs lambda >= 0, sigma_color >= 0, num_iter >= 1");
    hipStream_t st = (hipStream_t)stream;
    std::vector<float> lut;
    sdr::fgs_lut_host(sigma, &lut);
    // stream-ordered scratch: LUT + elimination coefficients
    float* dlut = nullptr;
    float* T = nullptr;
    const size_t px = (size_t)w * h;
    WLS_HIP(hipMallocAsync((void**)&dlut, sizeof(float) * lut.size(), st));
    WLS_HIP(hipMallocAsync((void**)&T, sizeof(float) * px * 2, st));
    WLS_HIP(hipMemcpyAsync(dlut, lut.data(), sizeof(float) * lut.size(), hipMemcpyHostToDevice, st));
    // images are filtered in pairs (two right-hand sides of one system per line)
    for (int i = 0; i < nimg; i += 2) {
        const int m = nimg - i >= 2 ? 2 : 1;
        sdr::launch_fgs(d_guide, gstride, 0, dlut, d_img + i * px, m == 2 ? d_img + (i + 1) * px : nullptr,
                        T, m, w, h, 1, lambda, att, iters, st);
    }
    WLS_HIP(hipGetLastError());
    WLS_HIP(hipFreeAsync(dlut, st));
    WLS_HIP(hipFreeAsync(T, st));
    // the host LUT vector dies here: wait for its upload before returning
    WLS_HIP(hipStreamSynchronize(st));
    return SDR_OK;
}

}  // extern "C"
