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
//   k_fgs_pcr      one FGS pass (rows or columns), the default solver (SDR_FGS_PCR): every line's
//                  tridiagonal system solved by parallel cyclic reduction in LDS, a 256-thread
//                  workgroup per line (or per G short lines), both right-hand sides at once, the
//                  diagonal carried as the row sum (oracle/wls_oracle.c fgs_line_pcr: every term
//                  non-negative, ~200x closer to the exact solution than the sequential sweep);
//                  rows and columns are both read in place from the row-major images
//   k_fgs_sweep    one FGS pass with the sequential solver (SDR_FGS_THOMAS, ximgproc's own
//                  elimination order, bit-exact with oracle/wls_oracle.c fgs_line): lane = line
//                  over k-major data, PF samples loaded ahead in registers; one lane per line
//                  leaves the chip nearly idle (6-9 waves at 640x360: ~112 us per pass)
//   k_transpose2   LDS-tiled transposes between the sweep's column-major copies and the row-major
//                  images; k_fgs_weights builds the weights once per frame
//   k_wls_final    FGS(conf*d) / FGS(conf) -> saturate_cast<short>, 16*(min_disp-1) outside ROI
#include "../../include/sdr/sdr.h"
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
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

// The filter's outputs (the class path's epilogue: fout = out / 16, xyz = reprojectImageTo3D(fout,
// Q), both nullable), written by whichever kernel holds a pixel's final value: k_wls_final, or,
// with SDR_FGS_PCR, k_wls_prep (pixels outside the ROI) and the last FGS column pass (the ROI).
struct WlsOut {
    int16_t* out;
    float* fout;
    float* xyz;
    Q16 Q;
};

// saturate_cast<short>(FGS(conf*d) / FGS(conf)) (cv::divide of floats: 0 for a zero divisor;
// cvRound = cvtss2si: NaN / |v| >= 2^31 give INT_MIN, which saturates to -32768)
__device__ __forceinline__ int16_t wls_value(float a, float c) {
    const float v = c != 0.0f ? a / c : 0.0f;
    float q = rintf(v);
    q = fminf(fmaxf(q, -32768.0f), 32767.0f);
    return fabsf(v) < 2147483648.0f ? (int16_t)(int)q : (int16_t)-32768;
}

// pixel (x, y) of frame f: the int16 value and the epilogue
__device__ __forceinline__ void wls_emit(const WlsOut& o, const WlsGeom& g, int f, int x, int y, int16_t r) {
    const size_t p = (size_t)f * g.W * g.H + (size_t)y * g.W + x;
    o.out[p] = r;
    if (o.fout) {
        const float df = (float)r * 0.0625f;
        o.fout[p] = df;
        if (o.xyz) reproject_px(o.Q, x, y, (double)df, 0.0, 0, o.xyz + 3 * p);
    }
}

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
//
// Layout: a sweep runs over "k-major" arrays, element (line l, sample k) at k*nlines + l, so that
// the 64 lanes of a wave (64 consecutive lines) touch 256 contiguous bytes per sample.  The row
// pass therefore works on column-major copies and the column pass on row-major ones; k_transpose2
// moves both right-hand sides between the two (LDS tiles).  Each lane walks its line with the
// loads of the next PF samples in flight (register ring), so a step costs the dependent-division
// latency of the t recurrence, not a memory round trip.
constexpr int kFgsPF = 8;  // samples each lane loads ahead in the line solves

// The line solve has no per-sample branches: the second right-hand side is a template parameter,
// the first sample uses the general step (with cprev = tprev = p = 0 it computes
// den = (1 - c) - 0, t = c / den, p = (r - 0) / den: the k = 0 formulas, bit for bit), and only
// the last, partial batch of PF samples checks the line's end.  The step's divisions are plain
// IEEE divisions (a shared refined reciprocal was bit-exact too, and no faster: the sweep is not
// bound by the division chain).
template <bool U1>
__global__ __launch_bounds__(64) void k_fgs_sweep(float* U0, float* U1p, const float* __restrict__ Cw,
                                                   float* __restrict__ T, int nlines, int n,
                                                   size_t fstride, float lam) {
    constexpr int PF = kFgsPF;
    const int l = blockIdx.x * 64 + threadIdx.x;
    if (l >= nlines) return;
    const size_t base = (size_t)blockIdx.y * fstride + l;
    float* u0 = U0 + base;
    float* u1 = U1 ? U1p + base : nullptr;
    const float* cw = Cw + base;
    float* t = T + base;
    const size_t st = (size_t)nlines;
    const int last = n - 1;
    // ---- forward elimination ----
    float r0[PF], r1[PF], rc[PF];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const size_t o = (size_t)min(j, last) * st;
        r0[j] = u0[o];
        if constexpr (U1) r1[j] = u1[o];
        rc[j] = cw[o];
    }
    float cprev = 0.0f, tprev = 0.0f, p0 = 0.0f, p1 = 0.0f;
    auto fwd = [&](int k, int j) __attribute__((always_inline)) {
        const size_t o = (size_t)k * st;
        const float aa = lam * cprev;
        const float c = lam * rc[j];
        const float den = (1.0f - c) - aa * (1.0f + tprev);
        tprev = c / den;
        p0 = (r0[j] - aa * p0) / den;
        if constexpr (U1) p1 = (r1[j] - aa * p1) / den;
        cprev = rc[j];
        t[o] = tprev;
        u0[o] = p0;
        if constexpr (U1) u1[o] = p1;
    };
    int k0 = 0;
    for (;; k0 += PF) {
        float n0[PF], n1[PF], nc[PF];
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const size_t o = (size_t)min(k0 + PF + j, last) * st;
            n0[j] = u0[o];
            if constexpr (U1) n1[j] = u1[o];
            nc[j] = cw[o];
        }
        if (k0 + PF - 1 <= last) {
#pragma unroll
            for (int j = 0; j < PF; j++) fwd(k0 + j, j);
        } else {
#pragma unroll
            for (int j = 0; j < PF; j++)
                if (k0 + j <= last) fwd(k0 + j, j);
        }
        if (k0 + PF > last) break;
        // whole-array copies (register renames after SROA; an element loop here was rewritten
        // into a copy idiom before the unroller ran, which then warned)
        __builtin_memcpy(r0, n0, sizeof r0);
        if constexpr (U1) __builtin_memcpy(r1, n1, sizeof r1);
        __builtin_memcpy(rc, nc, sizeof rc);
    }
    // ---- back substitution: u_k -= t[k] * u_{k+1}, k = n-2 .. 0 (the last sample keeps p) ----
    if (last < 1) return;
    float q0 = p0, q1 = p1;
    float b0[PF], b1[PF], bt[PF];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const size_t o = (size_t)max(last - 1 - j, 0) * st;
        b0[j] = u0[o];
        if constexpr (U1) b1[j] = u1[o];
        bt[j] = t[o];
    }
    auto bwd = [&](int k, int j) __attribute__((always_inline)) {
        const size_t o = (size_t)k * st;
        q0 = b0[j] - bt[j] * q0;
        u0[o] = q0;
        if constexpr (U1) {
            q1 = b1[j] - bt[j] * q1;
            u1[o] = q1;
        }
    };
    for (int k1 = last - 1;; k1 -= PF) {
        float n0[PF], n1[PF], nt[PF];
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const size_t o = (size_t)max(k1 - PF - j, 0) * st;
            n0[j] = u0[o];
            if constexpr (U1) n1[j] = u1[o];
            nt[j] = t[o];
        }
        if (k1 - PF + 1 >= 0) {
#pragma unroll
            for (int j = 0; j < PF; j++) bwd(k1 - j, j);
        } else {
#pragma unroll
            for (int j = 0; j < PF; j++)
                if (k1 - j >= 0) bwd(k1 - j, j);
        }
        if (k1 - PF < 0) break;
#pragma unroll
        for (int j = 0; j < PF; j++) {
            b0[j] = n0[j];
            if constexpr (U1) b1[j] = n1[j];
            bt[j] = nt[j];
        }
    }
}

// FGS line solves by parallel cyclic reduction (the default solver), in the operation order of
// oracle/wls_oracle.c fgs_line_pcr.  A workgroup of T threads (blockDim.x, a multiple of 64, up
// to 1024) owns G lines of n samples of one frame (G = 1 for long lines); equation e = g*n + k of
// the block lives in registers of thread e mod T (slot e / T), so a thread keeps its equations'
// (a, c, e, b, d0, d1) across the log2(n) stages and only publishes what its neighbours read:
//   X[e] = {row sum, 1/b, d0, d1} (one 16-byte LDS word), A[e] = a, Cc[e] = c
// Stage s reads X and A of e - s, X and Cc of e + s (zeros past the line's ends), then every
// equation is rewritten at once.  The published values are double-buffered by stage parity, so
// a stage costs one barrier: a thread can only overwrite a buffer two stages later, after the
// barrier every reader of it has passed.  The chip holds few lines (360 rows or 280 column pairs
// at 640x360), so the block takes as many threads as equations (EPT = 1 up to 1024 samples):
// several waves per SIMD hide the LDS and division latencies of the stage chain.  The images are
// read and written in place in their row-major layout: for rows (lines = rows) a block's loads
// are whole rows, for columns (lines = columns) G adjacent columns per row; loads and stores go
// through LDS with consecutive threads on consecutive addresses.  Weights Cw: same layout as the
// images (Ch for rows, Cv for columns, 0 on each line's last sample).
constexpr int kPcrMaxN = 4096;  // samples per block (G * n): 4 equations per thread of 1024

// DB: the stage buffers double-buffered (48 B of LDS per sample, one barrier per stage), or single
// (24 B per sample, two barriers per stage) for blocks whose 48 B per sample exceed the
// workgroup's LDS (160 KiB on gfx950: past 3413 samples)
// FIN (the last column pass, both right-hand sides): instead of storing the solved A, B back, the
// block writes the filter's outputs for its ROI pixels (wls_value / wls_emit; gw = the geometry)
template <int EPT, bool TWO, bool DB = true, bool FIN = false>
__global__ __launch_bounds__(1024) void k_fgs_pcr(float* U0, float* U1, const float* __restrict__ Cw,
                                                  int w, int h, size_t fstride, int rows, int G,
                                                  float lam, WlsGeom gw = {}, WlsOut wo = {}) {
    extern __shared__ float4 pcr_smem[];
    constexpr int NB = DB ? 2 : 1;
    const int T = blockDim.x;
    const int n = rows ? w : h;
    const int nlines = rows ? h : w;
    const int N = G * n;
    // NB stage buffers: X [NB][N] {row sum, 1/b, d0, d1}, then A [NB][N] (a; the weights during
    // the load), Cc [NB][N] (c)
    float4* X = pcr_smem;
    float* A = (float*)(X + NB * N);
    float* Cc = A + NB * N;
    const int tid = threadIdx.x;
    // consecutive line groups share an XCD: the column pass's G-column blocks of one row band
    // read and write parts of the same cache lines, which then meet in one L2
    const int gx = gridDim.x;
    const int lb = xcd_block(blockIdx.x + gx * blockIdx.y, gx * gridDim.y);
    const int l0 = (lb % gx) * G;
    const size_t fo = (size_t)(lb / gx) * fstride;
    auto addr = [&](int idx, int& g, int& k) -> size_t {
        if (rows) {
            g = idx / n;
            k = idx - g * n;
            return (size_t)(l0 + g) * w + k;
        }
        k = idx / G;
        g = idx - k * G;
        return (size_t)k * w + l0 + g;
    };
    // ---- coalesced load into LDS: weight -> A[e], rhs -> X[e].z/.w ----
    for (int idx = tid; idx < N; idx += T) {
        int g, k;
        const size_t off = addr(idx, g, k);
        const int e = g * n + k;
        float cw = 0.0f, r0 = 0.0f, r1 = 0.0f;
        if (l0 + g < nlines) {
            cw = Cw[fo + off];
            r0 = U0[fo + off];
            if constexpr (TWO) r1 = U1[fo + off];
        }
        A[e] = cw;
        X[e] = make_float4(0.0f, 0.0f, r0, r1);
    }
    __syncthreads();
    float a[EPT], c[EPT], rs[EPT], b[EPT], d0[EPT], d1[EPT];
    int kk[EPT];
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int e = tid + j * T;
        kk[j] = 0;
        a[j] = c[j] = 0.0f;
        rs[j] = b[j] = 1.0f;
        d0[j] = d1[j] = 0.0f;
        if (e < N) {
            const int k = e - (e / n) * n;
            kk[j] = k;
            c[j] = lam * A[e];
            a[j] = k > 0 ? lam * A[e - 1] : 0.0f;
            rs[j] = 1.0f;
            b[j] = (1.0f - a[j]) - c[j];
            d0[j] = X[e].z;
            d1[j] = X[e].w;
        }
    }
    __syncthreads();
    int buf = 0;
    for (int s = 1; s < n; s <<= 1, buf ^= DB ? N : 0) {
        float4* Xb = X + buf;
        float* Ab = A + buf;
        float* Cb = Cc + buf;
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int e = tid + j * T;
            if (e < N) {
                Xb[e] = make_float4(rs[j], 1.0f / b[j], d0[j], d1[j]);
                Ab[e] = a[j];
                Cb[e] = c[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            // branch-free: all four reads in flight at once, missing neighbours selected to zero
            // (threads past N compute on a clamped equation and never publish)
            const int e = min(tid + j * T, N - 1);
            {
                const bool hm = kk[j] >= s, hp = kk[j] + s < n;
                const int em = hm ? e - s : e, ep = hp ? e + s : e;
                float4 xm = Xb[em], xp = Xb[ep];
                float am = Ab[em], cp = Cb[ep];
                const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (!hm) {
                    xm = z4;
                    am = 0.0f;
                }
                if (!hp) {
                    xp = z4;
                    cp = 0.0f;
                }
                const float k1 = a[j] * xm.y;
                const float k2 = c[j] * xp.y;
                const float na = -(am * k1);
                const float nc = -(cp * k2);
                const float ne = (rs[j] - xm.x * k1) - xp.x * k2;
                b[j] = (ne - na) - nc;
                a[j] = na;
                c[j] = nc;
                rs[j] = ne;
                d0[j] = (d0[j] - xm.z * k1) - xp.z * k2;
                if constexpr (TWO) d1[j] = (d1[j] - xm.w * k1) - xp.w * k2;
            }
        }
        if constexpr (!DB) __syncthreads();  // every read of the one buffer done before the next writes
    }
    // ---- decoupled: u = d / b, staged in LDS (buffer `buf`, untouched since two stages back) for
    // the coalesced store ----
    float4* Xo = X + buf;
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int e = tid + j * T;
        if (e < N) Xo[e] = make_float4(0.0f, 0.0f, d0[j] / b[j], TWO ? d1[j] / b[j] : 0.0f);
    }
    __syncthreads();
    for (int idx = tid; idx < N; idx += T) {
        int g, k;
        const size_t off = addr(idx, g, k);
        if (l0 + g >= nlines) continue;
        const float4 x = Xo[g * n + k];
        if constexpr (FIN) {
            // columns pass: line l0 + g is ROI column j, sample k its ROI row i
            wls_emit(wo, gw, lb / gx, gw.rx + l0 + g, gw.ry + k, wls_value(x.z, x.w));
        } else {
            U0[fo + off] = x.z;
            if constexpr (TWO) U1[fo + off] = x.w;
        }
    }
}

// FGS weights of one guide (per frame): Ch (weight between (i, j) and (i, j+1): column-major at
// j*h + i for the sequential sweep, row-major at i*w + j for k_fgs_pcr) and Cv (row-major:
// (i, j)-(i+1, j) at i*w + j)
__global__ __launch_bounds__(256) void k_fgs_weights(const uint8_t* __restrict__ guide, size_t gstride,
                                                     size_t gfstride, const float* __restrict__ lut,
                                                     int w, int h, int ch_rowmajor, float* __restrict__ ChT,
                                                     float* __restrict__ Cv) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (j >= w || i >= h) return;
    const uint8_t* g = guide + (size_t)blockIdx.z * gfstride + (size_t)i * gstride + j;
    const size_t fo = (size_t)blockIdx.z * w * h;
    const int v = g[0];
    float ch = 0.0f, cv = 0.0f;
    if (j + 1 < w) {
        const int d = v - g[1];
        ch = lut[d * d];
    }
    if (i + 1 < h) {
        const int d = v - g[gstride];
        cv = lut[d * d];
    }
    ChT[fo + (ch_rowmajor ? (size_t)i * w + j : (size_t)j * h + i)] = ch;
    Cv[fo + (size_t)i * w + j] = cv;
}

// dst[f][c][r] = src[f][r][c] for two arrays (rows x cols per frame), 64x64 LDS tiles
__global__ __launch_bounds__(256) void k_transpose2(const float* __restrict__ s0,
                                                    const float* __restrict__ s1, float* __restrict__ d0,
                                                    float* __restrict__ d1, int rows, int cols) {
    __shared__ float tile[2][64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
    const size_t fo = (size_t)blockIdx.z * rows * cols;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int rr = r0 + r, cc = c0 + tx;
        if (rr < rows && cc < cols) {
            tile[0][r][tx] = s0[fo + (size_t)rr * cols + cc];
            if (s1) tile[1][r][tx] = s1[fo + (size_t)rr * cols + cc];
        }
    }
    __syncthreads();
    for (int c = ty; c < 64; c += 4) {
        const int cc = c0 + c, rr = r0 + tx;
        if (rr < rows && cc < cols) {
            d0[fo + (size_t)cc * rows + rr] = tile[0][tx][c];
            if (s1) d1[fo + (size_t)cc * rows + rr] = tile[1][tx][c];
        }
    }
}

// The whole filter front end of one ROI row in one workgroup (grid: rows x frames), replacing
// k_wls_disc + k_wls_conf + k_fgs_weights:
//   1. vertical (2r+1)-row sums of d and d^2 of both maps over the row's window (BORDER_REFLECT_101
//      inside the ROI), one column per thread, into LDS (int32 / int64: exact integers)
//   2. horizontal sums of those -> the depth-discontinuity value of every ROI column of both maps
//      (the same integers as disc_at's 2-D loop, so the same floats) into LDS
//   3. the discontinuity-aware LR check of the row (its partner column x - (d >> 4) is in the same
//      row, so the row's right map is all it needs): full-size confidence x255, A = conf * d,
//      B = conf (ROI-compact)
//   4. the row's FGS weights from the guide (Ch row-major for k_fgs_pcr or column-major for the
//      sequential sweep, Cv row-major)
// Rows outside the ROI only get the confidence map's 255.  Dynamic LDS: 32 B per ROI column
// (int64 + int32 column sums and a float discontinuity value, per map).
template <int RMAX>
__global__ __launch_bounds__(256) void k_wls_prep(const int16_t* __restrict__ dl, const int16_t* __restrict__ dr,
                                                  WlsGeom g, const uint8_t* __restrict__ guide,
                                                  size_t gstride, size_t gfstride,
                                                  const float* __restrict__ lut, int ch_rowmajor,
                                                  float* __restrict__ conf_full, float* __restrict__ A,
                                                  float* __restrict__ B, float* __restrict__ ChW,
                                                  float* __restrict__ Cv, int border, WlsOut wo) {
    extern __shared__ int64_t wls_smem[];
    const int y = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, T = blockDim.x;
    const size_t fo = (size_t)f * g.W * g.H;
    const int i = y - g.ry;
    // border: this row's outputs outside the ROI (16 * (min_disp - 1)) are final now (the last FGS
    // pass writes the ROI's)
    if (border)
        for (int x = tid; x < g.W; x += T)
            if (i < 0 || i >= g.rh || x < g.rx || x >= g.rx + g.rw) wls_emit(wo, g, f, x, y, (int16_t)g.fill);
    if (i < 0 || i >= g.rh) {
        if (conf_full)
            for (int x = tid; x < g.W; x += T) conf_full[fo + (size_t)y * g.W + x] = 255.0f;
        return;
    }
    const int rw = g.rw, r = g.radius;
    int64_t* V2 = wls_smem;                // [2][rw] column sums of d^2 (left, right)
    int* V = (int*)(V2 + 2 * rw);          // [2][rw] column sums of d
    float* disc = (float*)(V + 2 * rw);    // [2][rw] discontinuity values
    const int16_t* L = dl + fo;
    const int16_t* R = dr + fo;
    // the window's rows (wave-uniform: one image row per workgroup), then all 2(2r+1) loads of a
    // column at once: RMAX taps unrolled, those past the radius loading a duplicate row and masked
    // (a runtime-length tap loop issued its loads one iteration at a time)
    size_t rowo[2 * RMAX + 1];
#pragma unroll
    for (int t = 0; t <= 2 * RMAX; t++)
        rowo[t] = (size_t)(g.ry + reflect101(i + min(max(t - RMAX, -r), r), g.rh)) * g.W;
    for (int j = tid; j < rw; j += T) {
        int vl[2 * RMAX + 1], vr[2 * RMAX + 1];
#pragma unroll
        for (int t = 0; t <= 2 * RMAX; t++) {
            vl[t] = L[rowo[t] + g.rx + j];
            vr[t] = R[rowo[t] + g.rrx + j];
        }
        int s0 = 0, s1 = 0;
        int64_t q0 = 0, q1 = 0;
#pragma unroll
        for (int t = 0; t <= 2 * RMAX; t++) {
            const int a = t - RMAX;
            const int ml = a >= -r && a <= r ? vl[t] : 0, mr = a >= -r && a <= r ? vr[t] : 0;
            s0 += ml;
            q0 += (int64_t)ml * ml;
            s1 += mr;
            q1 += (int64_t)mr * mr;
        }
        V[j] = s0;
        V[rw + j] = s1;
        V2[j] = q0;
        V2[rw + j] = q1;
    }
    __syncthreads();
    // BORDER_REFLECT_101 of a column index one reflection deep (rw > RMAX; narrower ROIs loop)
    const bool shallow = rw > RMAX;
    auto refl = [&](int p) { return shallow ? (p < 0 ? -p : p >= rw ? 2 * rw - 2 - p : p) : reflect101(p, rw); };
    for (int j = tid; j < rw; j += T) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            long long s = 0, s2 = 0;
#pragma unroll
            for (int t = 0; t <= 2 * RMAX; t++) {
                const int b = t - RMAX;
                if (b < -r || b > r) continue;  // uniform
                const int jj = refl(j + b);
                s += V[m * rw + jj];
                s2 += V2[m * rw + jj];
            }
            const float mean = (float)((double)s * g.scale);
            const float msq = (float)((double)s2 * g.scale);
            const float var = msq - mean * mean;
            const float c = 1.0f - g.roll_off * var;
            disc[m * rw + j] = c > 0.0f ? c : 0.0f;
        }
    }
    __syncthreads();
    const size_t cf = (size_t)f * rw * g.rh + (size_t)i * rw;
    for (int x = tid; x < g.W; x += T) {
        const size_t o = (size_t)y * g.W + x;
        const int j = x - g.rx;
        const bool in_roi = j >= 0 && j < rw;
        float c = 1.0f;
        int v = 0;
        if (in_roi) {
            c = disc[j];
            v = L[o];
            const int ridx = x - (v >> 4);
            if (ridx >= g.rrx && ridx < g.rrx + rw) {
                if (abs(v + (int)R[(size_t)y * g.W + ridx]) < g.lrc_thresh) {
                    const float rc = disc[rw + ridx - g.rrx];
                    c = c < rc ? c : rc;
                } else {
                    c = 0.0f;
                }
            }
        }
        const float conf = 255.0f * c;
        if (conf_full) conf_full[fo + o] = conf;
        if (in_roi) {
            A[cf + j] = conf * (float)v;
            B[cf + j] = conf;
        }
    }
    // FGS weights of the guide's ROI row i (k_fgs_weights' formulas)
    const uint8_t* gr = guide + (size_t)f * gfstride + (size_t)(g.ry + i) * gstride + g.rx;
    const size_t wfo = (size_t)f * rw * g.rh;
    for (int j = tid; j < rw; j += T) {
        const int v = gr[j];
        float ch = 0.0f, cv = 0.0f;
        if (j + 1 < rw) {
            const int d = v - gr[j + 1];
            ch = lut[d * d];
        }
        if (i + 1 < g.rh) {
            const int d = v - gr[gstride + j];
            cv = lut[d * d];
        }
        ChW[wfo + (ch_rowmajor ? (size_t)i * rw + j : (size_t)j * g.rh + i)] = ch;
        Cv[wfo + (size_t)i * rw + j] = cv;
    }
}

// saturate_cast<short>(float): round half to even, saturate; 0 where FGS(conf) == 0 (cv::divide
// of floats returns 0 for a zero divisor)
// Optional epilogue of the class path (stereo_disparity.cpp:34, :76-80), fused: fout = out / 16
// (convertTo(CV_32F, 1/16)) and xyz = reprojectImageTo3D(fout, Q) (computeDepth,
// handleMissing = false).
__global__ __launch_bounds__(256) void k_wls_final(const float* __restrict__ A,
                                                   const float* __restrict__ B, WlsGeom g, WlsOut wo) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const int j = x - g.rx, i = y - g.ry;
    int16_t r = (int16_t)g.fill;
    if (j >= 0 && j < g.rw && i >= 0 && i < g.rh) {
        const size_t co = (size_t)blockIdx.z * g.rw * g.rh + (size_t)i * g.rw + j;
        r = wls_value(A[co], B[co]);
    }
    wls_emit(wo, g, blockIdx.z, x, y, r);
}

// FastGlobalSmootherFilter::filter on nimg (1 or 2) row-major w x h images per frame (R0, R1, in
// place), F frames sharing per-frame guides.  Scratch (each F*w*h floats): A, B (column-major
// copies), T (elimination coefficients), ChT, Cv (weights).
struct FgsScratch {
    float *A, *B, *T, *ChT, *Cv;
};

static void fgs_sweep(dim3 grid, hipStream_t st, float* U0, float* U1, const float* Cw, float* T,
                      int nlines, int n, size_t fs, float lam) {
    if (U1) hipLaunchKernelGGL((k_fgs_sweep<true>), grid, dim3(64), 0, st, U0, U1, Cw, T, nlines, n, fs, lam);
    else hipLaunchKernelGGL((k_fgs_sweep<false>), grid, dim3(64), 0, st, U0, U1, Cw, T, nlines, n, fs, lam);
}

// k_fgs_pcr instance for G*n samples per block: one equation per thread up to 1024 samples
// (T = the samples rounded up to whole waves), 2 or 4 per thread of 1024 beyond
template <bool TWO, bool FIN = false>
static int launch_pcr(float* U0, float* U1, const float* Cw, int w, int h, int F, int rows,
                      float lam, hipStream_t st, const WlsGeom& gw = {}, const WlsOut& wo = {}) {
    const int n = rows ? w : h, nlines = rows ? h : w;
    if (n > kPcrMaxN) return -1;
    // short lines: G per block so that a block holds up to 1024 samples
    const int G = std::max(1, std::min(nlines, 1024 / n));
    const int N = G * n;
    // (one equation per thread: 2 or 4 per thread at 640x360 measured 12.8 -> 15.0 / 16.8 us a pass)
    const int ept = N <= 1024 ? 1 : N <= 2048 ? 2 : 4;
    const int T = std::min(1024, ((N + ept - 1) / ept + 63) / 64 * 64);
    const dim3 grid((nlines + G - 1) / G, F), blk(T);
    const size_t fs = (size_t)w * h;
    // the workgroup's LDS (160 KiB on gfx950) holds double-buffered stages up to 3413 samples
    static thread_local int max_lds = 0;
    if (!max_lds) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
            max_lds <= 0)
            max_lds = 64 * 1024;
    }
    const bool db = (size_t)N * 48 <= (size_t)max_lds;
    if (!db && (size_t)N * 24 > (size_t)max_lds) return -1;
    if (!db) {
        hipLaunchKernelGGL((k_fgs_pcr<4, TWO, false, FIN>), grid, blk, (size_t)N * 24, st, U0, U1, Cw, w, h, fs,
                           rows, G, lam, gw, wo);
        return 0;
    }
    const size_t lds = (size_t)N * 48;
    if (ept == 1)
        hipLaunchKernelGGL((k_fgs_pcr<1, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    else if (ept == 2)
        hipLaunchKernelGGL((k_fgs_pcr<2, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    else
        hipLaunchKernelGGL((k_fgs_pcr<4, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    return 0;
}

// FastGlobalSmootherFilter::filter on R0 (and R1 when non-null: a second right-hand side of the
// same systems), row-major w x h per frame, F frames with per-frame guides, in place.
//   SDR_FGS_PCR:    weights (Ch, Cv row-major), then per iteration k_fgs_pcr over the rows and
//                   over the columns of the images themselves (2 launches per iteration)
//   SDR_FGS_THOMAS: weights (ChT column-major, Cv), then per iteration transpose -> row sweep ->
//                   transpose back -> column sweep (4 launches per iteration)
// Scratch (each F*w*h floats): A, B (column-major copies, THOMAS), T (THOMAS), ChT, Cv (weights).
static int launch_fgs(const uint8_t* guide, size_t gstride, size_t gfstride, const float* lut,
                      float* R0, float* R1, int w, int h, int F, double lambda, double att,
                      int iters, int solver, const FgsScratch& s, hipStream_t st,
                      bool weights_ready = false, sdr_sgbm* timer = nullptr,
                      const WlsGeom* fin_g = nullptr, const WlsOut* fin_o = nullptr) {
    const size_t fs = (size_t)w * h;
    const bool pcr = solver == SDR_FGS_PCR;
    if (!weights_ready)
        hipLaunchKernelGGL(k_fgs_weights, dim3((w + 63) / 64, (h + 3) / 4, F), dim3(256), 0, st, guide,
                           gstride, gfstride, lut, w, h, pcr ? 1 : 0, s.ChT, s.Cv);
    const dim3 t_rm((w + 63) / 64, (h + 63) / 64, F), t_cm((h + 63) / 64, (w + 63) / 64, F);
    float lam = (float)lambda;
    const float fa = (float)att;
    for (int it = 0; it < iters; it++) {
        if (pcr) {
            int e1, e2;
            {
                KScope kt(timer, SDR_KERNEL_FGS);
                e1 = R1 ? launch_pcr<true>(R0, R1, s.ChT, w, h, F, 1, lam, st)
                        : launch_pcr<false>(R0, R1, s.ChT, w, h, F, 1, lam, st);
            }
            {
                KScope kt(timer, SDR_KERNEL_FGS);
                // the last column pass writes the filter's outputs itself (fin_g / fin_o)
                if (fin_g && R1 && it == iters - 1)
                    e2 = launch_pcr<true, true>(R0, R1, s.Cv, w, h, F, 0, lam, st, *fin_g, *fin_o);
                else
                    e2 = R1 ? launch_pcr<true>(R0, R1, s.Cv, w, h, F, 0, lam, st)
                            : launch_pcr<false>(R0, R1, s.Cv, w, h, F, 0, lam, st);
            }
            if (e1 || e2) return -1;
        } else {
            {
                // row pass on column-major copies (lines = rows, k = column)
                KScope kt(timer, SDR_KERNEL_FGS);
                hipLaunchKernelGGL(k_transpose2, t_rm, dim3(256), 0, st, R0, R1, s.A, R1 ? s.B : nullptr, h, w);
                fgs_sweep(dim3((h + 63) / 64, F), st, s.A, R1 ? s.B : nullptr, s.ChT, s.T, h, w, fs, lam);
                hipLaunchKernelGGL(k_transpose2, t_cm, dim3(256), 0, st, s.A, R1 ? s.B : nullptr, R0, R1, w, h);
            }
            // column pass in place on the row-major images (lines = columns, k = row)
            KScope kt(timer, SDR_KERNEL_FGS);
            fgs_sweep(dim3((w + 63) / 64, F), st, R0, R1, s.Cv, s.T, w, h, fs, lam);
        }
        lam = lam * fa;  // FastGlobalSmootherFilterImpl::filter: lambda *= lambda_attenuation
    }
    return 0;
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
    sdr::Buf rdisc, conf, A, B, Ac, Bc, T, ChT, Cv, lut, out, hbuf;
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
    if (p.fgs_solver != SDR_FGS_PCR && p.fgs_solver != SDR_FGS_THOMAS)
        return sdr::set_error(SDR_ERR_ARG, "fgs_solver must be SDR_FGS_PCR or SDR_FGS_THOMAS");
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
    p->fgs_solver = SDR_FGS_PCR;
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
    for (sdr::Buf* b : {&h->rdisc, &h->conf, &h->A, &h->B, &h->Ac, &h->Bc, &h->T, &h->ChT, &h->Cv,
                        &h->lut, &h->out, &h->hbuf})
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

}  // extern "C"

// DisparityWLSFilter::filter on device with the class path's optional fused epilogue (fout =
// out / 16, xyz = reprojectImageTo3D(fout, Q)); sdr_wls_filter_device is this with neither.
// ROIs up to kPcrMaxN columns take the fused front end (k_wls_prep: discontinuity maps, LR check,
// confidence, FGS weights in one launch); wider ones the per-pixel k_wls_disc / k_wls_conf /
// k_fgs_weights kernels.
int sdr::wls_filter_enqueue(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide,
                            int W, int H, size_t gstride, size_t gfstride, int F, int16_t* out,
                            float* conf, float* fout, const double* Q, float* xyz, sdr_sgbm* timer) {
    if (!h || !dl || !dr || !guide || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0 || gstride < (size_t)W || (F > 1 && gfstride < gstride * H))
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    if (xyz && (!fout || !Q)) return sdr::set_error(SDR_ERR_ARG, "the fused reprojection needs fout and Q");
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
    if (roi && p.fgs_solver == SDR_FGS_PCR && (g.rw > sdr::kPcrMaxN || g.rh > sdr::kPcrMaxN))
        return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                            "(use SDR_FGS_THOMAS for larger ROIs)");
    const bool fused = roi && g.rw <= sdr::kPcrMaxN && g.radius <= 9;
    const size_t cpx = roi ? (size_t)g.rw * g.rh : 0;
    int rc;
    const float* lut = nullptr;
    if (!fused && (rc = sdr::ensure(h->rdisc, F * px * 4))) return rc;
    for (sdr::Buf* b : {&h->A, &h->B, &h->ChT, &h->Cv})
        if ((rc = sdr::ensure(*b, F * cpx * 4 + 4))) return rc;
    if (p.fgs_solver == SDR_FGS_THOMAS)
        for (sdr::Buf* b : {&h->Ac, &h->Bc, &h->T})
            if ((rc = sdr::ensure(*b, F * cpx * 4 + 4))) return rc;
    if ((rc = upload_lut(h, p.sigma_color, &lut))) return rc;
    float* A = (float*)h->A.p;
    float* B = (float*)h->B.p;
    const dim3 blk(256);
    const bool rowmajor = p.fgs_solver == SDR_FGS_PCR;
    const dim3 grid((W + 63) / 64, (H + 3) / 4, F);
    sdr::WlsOut wo{out, fout, xyz, {}};
    if (Q)
        for (int t = 0; t < 16; t++) wo.Q.q[t] = Q[t];
    // with the default solver the outputs need no pass of their own: k_wls_prep writes the pixels
    // outside the ROI and the last FGS column pass the ROI's (k_wls_final otherwise)
    const bool fin_fused = fused && roi && p.fgs_solver == SDR_FGS_PCR;
    if (fused) {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_PREP);
        // the window radius is ceil(blockSize / 2) <= 9 for every valid SGBM block; wider ones
        // (setDepthDiscontinuityRadius) take the per-pixel kernels below
        if (g.radius <= 4)
            hipLaunchKernelGGL(sdr::k_wls_prep<4>, dim3(H, F), blk, (size_t)g.rw * 32, st, dl, dr, g, guide,
                               gstride, gfstride, lut, rowmajor ? 1 : 0, conf, A, B, (float*)h->ChT.p,
                               (float*)h->Cv.p, fin_fused ? 1 : 0, wo);
        else
            hipLaunchKernelGGL(sdr::k_wls_prep<9>, dim3(H, F), blk, (size_t)g.rw * 32, st, dl, dr, g, guide,
                               gstride, gfstride, lut, rowmajor ? 1 : 0, conf, A, B, (float*)h->ChT.p,
                               (float*)h->Cv.p, fin_fused ? 1 : 0, wo);
    } else {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_PREP);
        if (roi)
            hipLaunchKernelGGL(sdr::k_wls_disc, dim3((g.rw + 63) / 64, (g.rh + 3) / 4, F), blk, 0, st,
                               dr, g, (float*)h->rdisc.p);
        hipLaunchKernelGGL(sdr::k_wls_conf, grid, blk, 0, st, dl, dr, (const float*)h->rdisc.p, g,
                           conf, A, B);
    }
    if (roi) {
        const uint8_t* g0 = guide + (size_t)g.ry * gstride + g.rx;
        const sdr::FgsScratch fs{(float*)h->Ac.p, (float*)h->Bc.p, (float*)h->T.p, (float*)h->ChT.p,
                                 (float*)h->Cv.p};
        if (sdr::launch_fgs(g0, gstride, gfstride, lut, A, B, g.rw, g.rh, F, p.lambda,
                            p.lambda_attenuation, p.num_iter, p.fgs_solver, fs, st, fused, timer,
                            fin_fused ? &g : nullptr, fin_fused ? &wo : nullptr))
            return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                                "(use SDR_FGS_THOMAS for larger ROIs)");
        if (fin_fused) {
            WLS_HIP(hipGetLastError());
            return SDR_OK;
        }
    }
    {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_FINAL);
        hipLaunchKernelGGL(sdr::k_wls_final, grid, blk, 0, st, A, B, g, wo);
    }
    WLS_HIP(hipGetLastError());
    return SDR_OK;
}

extern "C" {

int sdr_wls_filter_device(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide,
                          int W, int H, size_t gstride, size_t gfstride, int F, int16_t* out,
                          float* conf) {
    return sdr::wls_filter_enqueue(h, dl, dr, guide, W, H, gstride, gfstride, F, out, conf, nullptr,
                                   nullptr, nullptr);
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
                          int solver, void* stream) {
    if (!d_guide || !d_img) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (w <= 0 || h <= 0 || nimg <= 0 || gstride < (size_t)w)
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    if (!(lambda >= 0.0) || !(sigma >= 0.0) || iters < 1)
        return sdr::set_error(SDR_ERR_ARG, "FGS needs lambda >= 0, sigma_color >= 0, num_iter >= 1");
    if (solver != SDR_FGS_PCR && solver != SDR_FGS_THOMAS)
        return sdr::set_error(SDR_ERR_ARG, "solver must be SDR_FGS_PCR or SDR_FGS_THOMAS");
    if (solver == SDR_FGS_PCR && (w > sdr::kPcrMaxN || h > sdr::kPcrMaxN))
        return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                            "(use SDR_FGS_THOMAS for larger images)");
    hipStream_t st = (hipStream_t)stream;
    std::vector<float> lut;
    sdr::fgs_lut_host(sigma, &lut);
    // stream-ordered scratch: LUT, column-major copies, coefficients, weights
    float* dlut = nullptr;
    float* scr = nullptr;
    const size_t px = (size_t)w * h;
    WLS_HIP(hipMallocAsync((void**)&dlut, sizeof(float) * lut.size(), st));
    WLS_HIP(hipMallocAsync((void**)&scr, sizeof(float) * px * 5, st));
    WLS_HIP(hipMemcpyAsync(dlut, lut.data(), sizeof(float) * lut.size(), hipMemcpyHostToDevice, st));
    const sdr::FgsScratch fs{scr, scr + px, scr + 2 * px, scr + 3 * px, scr + 4 * px};
    // images are filtered in pairs (two right-hand sides of one system per line)
    for (int i = 0; i < nimg; i += 2) {
        const int m = nimg - i >= 2 ? 2 : 1;
        (void)sdr::launch_fgs(d_guide, gstride, 0, dlut, d_img + i * px, m == 2 ? d_img + (i + 1) * px : nullptr,
                              w, h, 1, lambda, att, iters, solver, fs, st);
    }
    WLS_HIP(hipGetLastError());
    WLS_HIP(hipFreeAsync(dlut, st));
    WLS_HIP(hipFreeAsync(scr, st));
    // the host LUT vector dies here: wait for its upload before returning
    WLS_HIP(hipStreamSynchronize(st));
    return SDR_OK;
}

}  // extern "C"
