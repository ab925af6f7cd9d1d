// sdr_post.hip -- post-WTA stages: A.10 median 3x3, A.11 speckle filter (connected components),
// per-frame minimum, A.12 reprojectImageTo3D, convertTo(1/16), A.13 class-path pre-steps
// (BGR2GRAY, INTER_AREA 0.5x) and a device self-test of the cross-lane primitives.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <float.h>

namespace sdr {

// ------------------------------------------------------------------------------------------
// A.10 medianBlur 3x3, replicate border (Devillard's 19-exchange median-of-9 network)
// ------------------------------------------------------------------------------------------
// 3x3 median at (x, y) of a frame, BORDER_REPLICATE (medianBlur ksize 3: 19-exchange network).
// MASK: columns outside [c0, c1) read as `fill` (the WTA map outside the matched columns, which
// the LR check would have written as INVALID; used when that check cannot fire)
template <bool MASK = false>
__device__ __forceinline__ int median3_at(const int16_t* __restrict__ src, int W, int H, int x, int y,
                                          int c0 = 0, int c1 = 0, int fill = 0) {
    int p[9];
    const int xs[3] = {max(x - 1, 0), x, min(x + 1, W - 1)};
    const int ys[3] = {max(y - 1, 0), y, min(y + 1, H - 1)};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            if (MASK && (xs[j] < c0 || xs[j] >= c1)) p[i * 3 + j] = fill;
            else p[i * 3 + j] = src[(size_t)ys[i] * W + xs[j]];
        }
#define SDR_S(a, b) { int t_ = min(p[a], p[b]); p[b] = max(p[a], p[b]); p[a] = t_; }
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 1) SDR_S(3, 4) SDR_S(6, 7)
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 3) SDR_S(5, 8) SDR_S(4, 7)
    SDR_S(3, 6) SDR_S(1, 4) SDR_S(2, 5) SDR_S(4, 7) SDR_S(4, 2) SDR_S(6, 4)
    SDR_S(4, 2)
#undef SDR_S
    return p[4];
}

__global__ __launch_bounds__(256) void k_median3(const int16_t* __restrict__ src,
                                                 int16_t* __restrict__ dst, int W, int H) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const size_t fo = (size_t)blockIdx.z * W * H;
    if (x >= W || y >= H) return;
    dst[fo + (size_t)y * W + x] = (int16_t)median3_at(src + fo, W, H, x, y);
}

void launch_median3(const int16_t* src, int16_t* dst, int W, int H, int F, hipStream_t st) {
    dim3 grid((W + 63) / 64, (H + 3) / 4, F);
    hipLaunchKernelGGL(k_median3, grid, dim3(256), 0, st, src, dst, W, H);
}

// the (TW + 2) x (TH + 2) neighbourhood of a TW x TH tile of the LR-checked map (A.9 from the WTA
// map and the right-view keys), rows and columns clamped (medianBlur's BORDER_REPLICATE), in LDS
// (lr_at unrolled over a thread's NPT pixels: all WTA loads, then all key loads, so the block
// pays two dependent memory round trips, not two per pixel)
template <int TW, int TH, int NT>
__device__ __forceinline__ void stage_lr_halo(const LrSrc& lr, int tx0, int ty0, int f, int16_t* hal) {
    const Geometry g = frame_geom(lr.g, f);
    const size_t fo = (size_t)f * lr.fstride;
    const int16_t* raw = lr.raw + fo;
    const uint32_t* d2 = lr.d2 + fo;
    constexpr int HW = TW + 2, N = HW * (TH + 2), NPT = (N + NT - 1) / NT;
    const int invalid = (g.minD - 1) * 16, c0 = g.minX1, c1 = g.minX1 + g.W1;
    int d1[NPT], xa[NPT], xb[NPT];
    size_t ro[NPT];
    bool m[NPT];
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = min((int)threadIdx.x + k * NT, N - 1);
        const int hy = i / HW, hx = i - hy * HW;
        const int y = min(max(ty0 - 1 + hy, 0), g.H - 1), x = min(max(tx0 - 1 + hx, 0), g.W - 1);
        ro[k] = (size_t)y * g.W;
        m[k] = x >= c0 && x < c1;
        d1[k] = raw[ro[k] + min(max(x, c0), c1 - 1)];  // matched columns only hold values
        xa[k] = x;
    }
    uint32_t ka[NPT], kb[NPT];
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        if (!m[k]) d1[k] = invalid;
        const int x = xa[k];
        xa[k] = x - (d1[k] >> 4);
        xb[k] = x - ((d1[k] + 15) >> 4);
        ka[k] = d2[ro[k] + min(max(xa[k], 0), g.W - 1)];
        kb[k] = d2[ro[k] + min(max(xb[k], 0), g.W - 1)];
    }
#pragma unroll
    for (int k = 0; k < NPT; k++) {
        const int i = threadIdx.x + k * NT;
        if (i >= N) break;
        int v = d1[k];
        const int _d = v >> 4, d_ = (v + 15) >> 4;
        if (v != invalid && xa[k] >= 0 && xa[k] < g.W && xb[k] >= 0 && xb[k] < g.W) {
            const int a2 = ka[k] == kD2None ? invalid : (0xffff - (int)(ka[k] & 0xffff)) + g.minX1 - xa[k];
            const int b2 = kb[k] == kD2None ? invalid : (0xffff - (int)(kb[k] & 0xffff)) + g.minX1 - xb[k];
            if (a2 >= g.minD && abs(a2 - _d) > lr.d12 && b2 >= g.minD && abs(b2 - d_) > lr.d12) v = invalid;
        }
        hal[i] = (int16_t)v;
    }
}

// 3x3 median at (lx, ly) of a tile from its staged neighbourhood (row pitch HW)
template <int HW>
__device__ __forceinline__ int median3_lds(const int16_t* hal, int lx, int ly) {
    int p[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) p[i * 3 + j] = hal[(ly + i) * HW + lx + j];
#define SDR_S(a, b) { int t_ = min(p[a], p[b]); p[b] = max(p[a], p[b]); p[a] = t_; }
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 1) SDR_S(3, 4) SDR_S(6, 7)
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 3) SDR_S(5, 8) SDR_S(4, 7)
    SDR_S(3, 6) SDR_S(1, 4) SDR_S(2, 5) SDR_S(4, 7) SDR_S(4, 2) SDR_S(6, 4)
    SDR_S(4, 2)
#undef SDR_S
    return p[4];
}

// A.9 + A.10 without the speckle filter: 64 x 4 tiles, the LR check computed once per staged pixel
__global__ __launch_bounds__(256) void k_median3_lr(LrSrc lr, int16_t* __restrict__ dst) {
    __shared__ int16_t hal[66 * 6];
    const int tx0 = blockIdx.x * 64, ty0 = blockIdx.y * 4, f = blockIdx.z;
    stage_lr_halo<64, 4, 256>(lr, tx0, ty0, f, hal);
    __syncthreads();
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
    const int x = tx0 + lx, y = ty0 + ly;
    if (x >= lr.g.W || y >= lr.g.H) return;
    dst[(size_t)f * lr.g.W * lr.g.H + (size_t)y * lr.g.W + x] = (int16_t)median3_lds<66>(hal, lx, ly);
}

void launch_median3_lr(const LrSrc& lr, int16_t* dst, int F, hipStream_t st) {
    dim3 grid((lr.g.W + 63) / 64, (lr.g.H + 3) / 4, F);
    hipLaunchKernelGGL(k_median3_lr, grid, dim3(256), 0, st, lr, dst);
}

// the column mask of frame f: the matched columns [minX1, minX1 + W1) and INVALID of its matcher
__global__ __launch_bounds__(256) void k_median3_cols(const int16_t* __restrict__ src,
                                                      int16_t* __restrict__ dst, Geometry g) {
    const int W = g.W, H = g.H;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const size_t fo = (size_t)blockIdx.z * W * H;
    if (x >= W || y >= H) return;
    const Geometry gf = frame_geom(g, blockIdx.z);
    dst[fo + (size_t)y * W + x] =
        (int16_t)median3_at<true>(src + fo, W, H, x, y, gf.minX1, gf.minX1 + gf.W1, (gf.minD - 1) * 16);
}

void launch_median3_cols(const int16_t* src, int16_t* dst, const Geometry& g, int F, hipStream_t st) {
    dim3 grid((g.W + 63) / 64, (g.H + 3) / 4, F);
    hipLaunchKernelGGL(k_median3_cols, grid, dim3(256), 0, st, src, dst, g);
}

// src outside each frame's matched columns -> its INVALID (the LR-check stage's map when the check
// cannot fire)
__global__ void k_mask_cols(const int16_t* __restrict__ src, int16_t* __restrict__ dst, Geometry g, int F) {
    const size_t px = (size_t)g.W * g.H, n = px * F;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const Geometry gf = frame_geom(g, (int)(i / px));
        const int x = (int)(i % g.W);
        dst[i] = (x < gf.minX1 || x >= gf.minX1 + gf.W1) ? (int16_t)((gf.minD - 1) * 16) : src[i];
    }
}

void launch_mask_cols(const int16_t* src, int16_t* dst, const Geometry& g, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_mask_cols, dim3(256), dim3(256), 0, st, src, dst, g, F);
}

// ------------------------------------------------------------------------------------------
// A.11 filterSpeckles as connected-component labelling: 4-neighbours p,q are joined iff
// neither equals newVal and |v(p)-v(q)| <= maxDiff; components of <= maxSize pixels are set to
// newVal.  The flood fill of OpenCV and CCL give identical components (the join relation is
// symmetric and evaluated on the unmodified image).
//
//   k_ccl_local    32x32 tile in LDS: horizontal runs from one ballot per row (no atomics), run
//                  unions across rows (lock-free union-find, Playne & Hawick 2018), local sizes
//                  with one LDS atomic per (wave, root).  P[pixel] = tile-root pixel index,
//                  S[tile root] = its pixel count, S = 0 elsewhere.
//   k_ccl_merge    tile-border pixel pairs unite the tile roots (global union-find); a pair whose
//                  previous pair along the border is joined through in-tile edges is skipped.
//   k_ccl_finalize each tile root finds its global root, adds its count there, points at it.
//   k_ccl_apply    P[P[pixel]] is the global root -> size test -> output (+ fused frame minimum
//                  for reprojectImageTo3D's handleMissingValues).
// Pixel-level work is streaming; global finds and atomics scale with the number of tile
// components, not with the pixels of a large component.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int uf_load(const int* P, int i) {
    return __hip_atomic_load(&P[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// find with path halving; parents only ever decrease (union links the larger root under the
// smaller), so a no-return atomicMin keeps concurrent unions intact
__device__ __forceinline__ int uf_find(int* P, int x) {
    int p = uf_load(P, x);
    while (p != x) {
        const int gp = uf_load(P, p);
        if (gp != p) atomicMin(&P[x], gp);
        x = p;
        p = gp;
    }
    return x;
}
__device__ __forceinline__ void uf_unite(int* P, int a, int b) {
    for (;;) {
        a = uf_find(P, a);
        b = uf_find(P, b);
        if (a == b) return;
        if (a < b) {
            int old = atomicMin(&P[b], a);
            if (old == b) return;
            b = old;
        } else {
            int old = atomicMin(&P[a], b);
            if (old == a) return;
            a = old;
        }
    }
}

constexpr int kCT = 32;

__device__ __forceinline__ int lds_find(int* lab, int x) {
    int p = __hip_atomic_load(&lab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(&lab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return x;
}
__device__ __forceinline__ void lds_unite(int* lab, int a, int b) {
    for (;;) {
        a = lds_find(lab, a);
        b = lds_find(lab, b);
        if (a == b) return;
        if (a < b) {
            int old = atomicMin(&lab[b], a);
            if (old == b) return;
            b = old;
        } else {
            int old = atomicMin(&lab[a], b);
            if (old == a) return;
            a = old;
        }
    }
}

__device__ __forceinline__ bool joined(int a, int b, int newVal, int maxDiff) {
    return a != newVal && b != newVal && abs(a - b) <= maxDiff;
}

// 256 threads = 4 waves; pixel i = t + 256k (k < 4): a wave covers two tile rows per k.
// LRMED: the image is the 3x3 median of the LR-checked map; the tile's neighbourhood of that map
// is computed into LDS (A.9 from the WTA map and the right-view keys), its medians are computed
// here and written to med (the image merge and apply read): the LR check and the median pass
// run inside the labelling's first pass.
template <bool LRMED>
__global__ __launch_bounds__(256) void k_ccl_local(const int16_t* __restrict__ img, int16_t* __restrict__ med,
                                                   int* __restrict__ P, int* __restrict__ S, int W, int H,
                                                   int newVal, int maxDiff, int* out_min, LrSrc lr) {
    __shared__ int v[kCT * kCT];
    __shared__ int lab[kCT * kCT];
    __shared__ int cnt[kCT * kCT];
    __shared__ int16_t hal[LRMED ? (kCT + 2) * (kCT + 2) : 1];
    const int tx0 = blockIdx.x * kCT, ty0 = blockIdx.y * kCT;
    const size_t fo = (size_t)blockIdx.z * W * H;
    const int t = threadIdx.x, lane = t & 63, lx = t & (kCT - 1);
    if (out_min && blockIdx.x == 0 && blockIdx.y == 0)
        for (int j = t; j < kMinSlots; j += 256) out_min[blockIdx.z * kMinSlots + j] = 32767;
    const int gx = tx0 + lx;
    if (LRMED) {
        stage_lr_halo<kCT, kCT, 256>(lr, tx0, ty0, blockIdx.z, hal);
        __syncthreads();
    }
    int val[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = t + 256 * k, gy = ty0 + (i >> 5);
        if (LRMED) {
            val[k] = newVal;
            if (gx < W && gy < H) {
                val[k] = median3_lds<kCT + 2>(hal, lx, i >> 5);
                med[fo + (size_t)gy * W + gx] = (int16_t)val[k];
            }
        } else {
            val[k] = (gx < W && gy < H) ? (int)img[fo + (size_t)gy * W + gx] : newVal;
        }
        v[i] = val[k];
        cnt[i] = 0;
    }
    __syncthreads();
    // horizontal runs: a run starts at every valid pixel not joined to its left neighbour
    int run[4];
    bool hc[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = t + 256 * k;
        const bool valid = val[k] != newVal;
        hc[k] = valid && lx > 0 && joined(val[k], v[i - 1], newVal, maxDiff);
        const unsigned long long starts = __ballot(valid && !hc[k]);
        const unsigned long long below = starts & (~0ull >> (63 - lane));
        const int s = 63 - __clzll(below);  // the row's first valid pixel is a start: below != 0
        run[k] = valid ? i - (lane - s) : -1;
        lab[i] = run[k];
    }
    __syncthreads();
    // vertical joins between runs; skip the join when the left pixel (same run) is joined to the
    // up-left pixel (same run as up): those two runs are already being united
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = t + 256 * k;
        if (run[k] < 0 || i < kCT) continue;
        const int up = i - kCT, vu = v[up];
        if (!joined(val[k], vu, newVal, maxDiff)) continue;
        if (hc[k]) {
            const int vl = v[i - 1], vul = v[up - 1];
            if (joined(vl, vul, newVal, maxDiff) && joined(vu, vul, newVal, maxDiff)) continue;
        }
        lds_unite(lab, run[k], up);
    }
    __syncthreads();
    // roots and local sizes (one LDS atomic per distinct root of a wave)
    int root[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        root[k] = run[k] >= 0 ? lds_find(lab, run[k]) : -1;
        unsigned long long pend = __ballot(root[k] >= 0);
        while (pend) {
            const int src = __ffsll((long long)pend) - 1;
            const int r = __shfl(root[k], src);
            const unsigned long long m = __ballot(root[k] == r) & pend;
            if (lane == src) atomicAdd(&cnt[r], __popcll(m));
            pend &= ~m;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = t + 256 * k, gy = ty0 + (i >> 5);
        if (gx >= W || gy >= H) continue;
        const size_t g = fo + (size_t)gy * W + gx;
        const int r = root[k];
        P[g] = r >= 0 ? (ty0 + (r >> 5)) * W + tx0 + (r & (kCT - 1)) : -1;
        S[g] = (r >= 0 && r == i) ? cnt[i] : 0;
    }
}

// tile-border pairs: vertical borders (x = 32k-1 | 32k) and horizontal ones (y = 32k-1 | 32k)
__global__ __launch_bounds__(256) void k_ccl_merge(const int16_t* __restrict__ img, int* P, int W,
                                                   int H, int newVal, int maxDiff) {
    const size_t fo = (size_t)blockIdx.y * W * H;
    const int16_t* I = img + fo;
    int* Pf = P + fo;
    const int nvx = (W - 1) / kCT, nhy = (H - 1) / kCT;
    const int nv = nvx * H, nh = nhy * W;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nv + nh; t += gridDim.x * blockDim.x) {
        int a, b, step;
        bool inner;  // the previous pair along the border is tied to this one by in-tile edges
        if (t < nv) {
            const int xb = t % nvx, y = t / nvx, x = (xb + 1) * kCT - 1;
            a = y * W + x;
            b = a + 1;
            step = W;
            inner = (y % kCT) != 0;
        } else {
            const int u = t - nv;
            const int yb = u / W, x = u - yb * W, y = (yb + 1) * kCT - 1;
            a = y * W + x;
            b = a + W;
            step = 1;
            inner = (x % kCT) != 0;
        }
        // every load this pair may need is issued up front (the previous pair's values, and the
        // labels of a and b with one more hop): three dependent round trips instead of up to six
        const int sa = inner ? a - step : a, sb = inner ? b - step : b;
        const int va = I[a], vb = I[b], pa = I[sa], pb = I[sb];
        const int ra = uf_load(Pf, a), rb = uf_load(Pf, b);
        if (!joined(va, vb, newVal, maxDiff)) continue;
        if (inner && joined(pa, pb, newVal, maxDiff) && joined(va, pa, newVal, maxDiff) &&
            joined(vb, pb, newVal, maxDiff))
            continue;
        int x = uf_load(Pf, ra), y = uf_load(Pf, rb);
        if (x == ra && y == rb) {
            // both were roots: link the larger under the smaller (uf_unite's step without its finds)
            if (x == y) continue;
            const int lo = min(x, y), hi = max(x, y);
            const int old = atomicMin(&Pf[hi], lo);
            if (old == hi) continue;
            x = lo;
            y = old;
        }
        uf_unite(Pf, x, y);
    }
}

// tile roots (S > 0): global root, size accumulated there, one-hop pointer for apply.  Only
// "size <= maxSize" is ever asked, so a tile part larger than maxSize marks its component with a
// plain store of kBigComponent instead of adding (every atomic add to a large component's root
// serialises at that one address; the store may land before or after the adds of other parts,
// and either way the size reads as more than maxSize).
constexpr int kBigComponent = 0x40000000;
__global__ __launch_bounds__(256) void k_ccl_finalize(int* P, int* S, int n, int maxSize) {
    const size_t fo = (size_t)blockIdx.y * n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int c = S[fo + i];
        if (c <= 0) continue;
        const int g = uf_find(P + fo, i);
        if (g != i) {
            if (c > maxSize) S[fo + g] = kBigComponent;
            else atomicAdd(&S[fo + g], c);
            P[fo + i] = g;
        }
    }
}

// A thread owns kApplyU pixels (a grid stride apart) and walks them in phases -- all pixel and
// label loads, then all tile-root -> global-root gathers, then all size gathers -- so its three
// dependent memory round trips are paid once, not once per pixel.  (src and dst may be one
// buffer: every pixel is read and then written by its own thread only.)
constexpr int kApplyU = 2;
__global__ __launch_bounds__(256) void k_ccl_apply(const int16_t* src, int16_t* dst,
                                                   const int* __restrict__ P, const int* __restrict__ S,
                                                   int n, int newVal, int maxSize, int* out_min) {
    __shared__ int wm[4];
    const size_t fo = (size_t)blockIdx.y * n;
    const int* Pf = P + fo;
    const int* Sf = S + fo;
    const int stride = gridDim.x * blockDim.x;
    int m = 32767;
    for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += kApplyU * stride) {
        int v[kApplyU], l[kApplyU], s[kApplyU];
#pragma unroll
        for (int u = 0; u < kApplyU; u++) {
            const int i = min(i0 + u * stride, n - 1);  // surplus pixels repeat the last one
            v[u] = src[fo + i];
            l[u] = Pf[i];
        }
#pragma unroll
        for (int u = 0; u < kApplyU; u++) l[u] = l[u] >= 0 ? Pf[l[u]] : -1;
#pragma unroll
        for (int u = 0; u < kApplyU; u++) s[u] = l[u] >= 0 ? Sf[l[u]] : 0x7fffffff;
#pragma unroll
        for (int u = 0; u < kApplyU; u++) {
            const int i = i0 + u * stride;
            if (i >= n) break;
            const int o = s[u] <= maxSize ? newVal : v[u];
            dst[fo + i] = (int16_t)o;
            m = min(m, o);
        }
    }
    if (!out_min) return;
    m = (int)wave_min_u32((uint32_t)(m + 32768)) - 32768;
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMin(&out_min[blockIdx.y * kMinSlots + blockIdx.x % kMinSlots], min(min(wm[0], wm[1]), min(wm[2], wm[3])));
}

void launch_speckle(const int16_t* src, int16_t* dst, int W, int H, int F, int newVal, int maxSize,
                    int maxDiff, int* labels, int* sizes, int* out_min, hipStream_t st,
                    const LrSrc* lr, int16_t* median_out) {
    const int n = W * H;
    const dim3 tiles((W + kCT - 1) / kCT, (H + kCT - 1) / kCT, F);
    if (lr)
        hipLaunchKernelGGL((k_ccl_local<true>), tiles, dim3(256), 0, st, (const int16_t*)nullptr, median_out,
                           labels, sizes, W, H, newVal, maxDiff, out_min, *lr);
    else
        hipLaunchKernelGGL((k_ccl_local<false>), tiles, dim3(256), 0, st, src, (int16_t*)nullptr, labels, sizes,
                           W, H, newVal, maxDiff, out_min, LrSrc{});
    const int nb = ((W - 1) / kCT) * H + ((H - 1) / kCT) * W;
    if (nb > 0)
        hipLaunchKernelGGL(k_ccl_merge, dim3((unsigned)min((nb + 255) / 256, 1024), F), dim3(256), 0,
                           st, src, labels, W, H, newVal, maxDiff);
    // finalize / apply: about 2048 blocks over the batch (2 pixels per thread at one 1280x720
    // frame: 44 -> 34 us for the four speckle kernels; 256 blocks per frame left one wave per SIMD
    // for the label gathers), never fewer than 256 per frame
    const unsigned gb = (unsigned)min((n + 511) / 512, max(256, 2048 / F));
    hipLaunchKernelGGL(k_ccl_finalize, dim3(gb, F), dim3(256), 0, st, labels, sizes, n, maxSize);
    const unsigned ga = (unsigned)min((n + 256 * kApplyU - 1) / (256 * kApplyU), max(256, 2048 / F));
    hipLaunchKernelGGL(k_ccl_apply, dim3(ga, F), dim3(256), 0, st, src, dst, labels, sizes, n, newVal,
                       maxSize, out_min);
}

// ------------------------------------------------------------------------------------------
// per-frame minimum (reprojectImageTo3D handleMissingValues needs min(disp)), kept as kMinSlots
// partial minima per frame: block b folds into slot b % kMinSlots and the reprojection takes the
// minimum of the slots.  (One slot per frame serialised ~1800 same-address device-scope atomics
// at the end of k_ccl_apply.)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_min_s16(const int16_t* img, size_t n, size_t fstride, int* out) {
    __shared__ int wm[4];
    const int16_t* I = img + (size_t)blockIdx.y * fstride;
    int m = 32767;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        m = min(m, (int)I[i]);
    m = (int)wave_min_u32((uint32_t)(m + 32768)) - 32768;
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMin(&out[blockIdx.y * kMinSlots + blockIdx.x % kMinSlots], min(min(wm[0], wm[1]), min(wm[2], wm[3])));
}

__global__ void k_init_i32(int* p, int v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

void launch_min_s16(const int16_t* img, size_t n_per_frame, size_t fstride, int F, int* out_min,
                    hipStream_t st) {
    hipLaunchKernelGGL(k_init_i32, dim3((F * kMinSlots + 255) / 256), dim3(256), 0, st, out_min, 32767,
                       F * kMinSlots);
    dim3 grid((unsigned)min((n_per_frame + 1023) / 1024, (size_t)128), F);
    hipLaunchKernelGGL(k_min_s16, grid, dim3(256), 0, st, img, n_per_frame, fstride, out_min);
}

// ------------------------------------------------------------------------------------------
// A.12 reprojectImageTo3D: double math, sequential sums from 0, no contraction, Vec3f then
// *(1.0/h3) rounded to float; handleMissing: Z = 10000 where |d - min(disp)| <= FLT_EPSILON.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_reproject_s16(const int16_t* disp, int W, int H,
                                                       size_t dstride, size_t dfstride, Q16 Q,
                                                       int hm, const int* mins, float* xyz,
                                                       size_t xstride, size_t xfstride) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    double mind = (double)FLT_MAX;
    if (hm) {
        // the frame minimum from its slots: kMinSlots / 64 coalesced loads per lane + a wave minimum
        // (before any lane leaves)
        static_assert(kMinSlots % 64 == 0, "slots per lane");
        const int lane = threadIdx.x & 63;
        int m = 32767;
#pragma unroll
        for (int k = 0; k < kMinSlots / 64; k++) m = min(m, mins[f * kMinSlots + k * 64 + lane]);
        m = (int)wave_min_u32_uniform((uint32_t)(m + 32768)) - 32768;
        mind = (double)((float)m * 0.0625f);
    }
    if (x >= W) return;
    const int v = disp[(size_t)f * dfstride + (size_t)y * dstride + x];
    const double d = (double)((float)v * 0.0625f);
    reproject_px(Q, x, y, d, mind, hm, xyz + (size_t)f * xfstride + (size_t)y * xstride + 3 * (size_t)x);
}

__device__ __forceinline__ int f2ord(float f) {
    int i = __float_as_int(f);
    return i < 0 ? i ^ 0x7fffffff : i;
}
__device__ __forceinline__ float ord2f(int i) {
    return __int_as_float(i < 0 ? i ^ 0x7fffffff : i);
}

__global__ void k_min_f32(const float* disp, int W, int H, size_t dstride, size_t dfstride, int* out) {
    const float* I = disp + (size_t)blockIdx.y * dfstride;
    int m = 0x7fffffff;
    const size_t n = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        float v = I[(i / W) * dstride + (i % W)];
        if (v == v) m = min(m, f2ord(v));
    }
    for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMin(&out[blockIdx.y], m);
}

__global__ __launch_bounds__(256) void k_reproject_f32(const float* disp, int W, int H,
                                                       size_t dstride, size_t dfstride, Q16 Q,
                                                       int hm, const int* minbits, float* xyz,
                                                       size_t xstride, size_t xfstride) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= W) return;
    const double d = (double)disp[(size_t)f * dfstride + (size_t)y * dstride + x];
    const double mind = hm ? (double)ord2f(minbits[f]) : (double)FLT_MAX;
    reproject_px(Q, x, y, d, mind, hm, xyz + (size_t)f * xfstride + (size_t)y * xstride + 3 * (size_t)x);
}

void launch_reproject_s16(const int16_t* disp, int W, int H, size_t dstride, size_t dfstride,
                          const double* Q, int hm, const int* mins, float* xyz, size_t xstride,
                          size_t xfstride, int F, hipStream_t st) {
    Q16 q;
    for (int i = 0; i < 16; i++) q.q[i] = Q[i];
    hipLaunchKernelGGL(k_reproject_s16, dim3((W + 255) / 256, H, F), dim3(256), 0, st, disp, W, H,
                       dstride, dfstride, q, hm, mins, xyz, xstride, xfstride);
}

void launch_reproject_f32(const float* disp, int W, int H, size_t dstride, size_t dfstride,
                          const double* Q, int hm, int* minbits, float* xyz, size_t xstride,
                          size_t xfstride, int F, hipStream_t st) {
    Q16 q;
    for (int i = 0; i < 16; i++) q.q[i] = Q[i];
    if (hm) {
        hipLaunchKernelGGL(k_init_i32, dim3((F + 255) / 256), dim3(256), 0, st, minbits, 0x7fffffff, F);
        hipLaunchKernelGGL(k_min_f32, dim3(256, F), dim3(256), 0, st, disp, W, H, dstride, dfstride, minbits);
    }
    hipLaunchKernelGGL(k_reproject_f32, dim3((W + 255) / 256, H, F), dim3(256), 0, st, disp, W, H,
                       dstride, dfstride, q, hm, minbits, xyz, xstride, xfstride);
}

__global__ void k_disp16_to_f32(const int16_t* d, float* o, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        o[i] = (float)d[i] * 0.0625f;
}

void launch_disp16_to_f32(const int16_t* d, float* o, size_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_disp16_to_f32, dim3((unsigned)min((n + 255) / 256, (size_t)4096)),
                       dim3(256), 0, st, d, o, n);
}

// ------------------------------------------------------------------------------------------
// A.13 class-path pre-steps
// ------------------------------------------------------------------------------------------
__global__ void k_bgr2gray(const uint8_t* bgr, int W, int H, size_t bstride, uint8_t* gray,
                           size_t gstride) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= W) return;
    const uint8_t* s = bgr + (size_t)f * bstride * H + (size_t)y * bstride + 3 * (size_t)x;
    int v = (s[0] * 1868 + s[1] * 9617 + s[2] * 4899 + (1 << 13)) >> 14;
    gray[(size_t)f * gstride * H + (size_t)y * gstride + x] = (uint8_t)v;
}

__global__ void k_area_half(const uint8_t* src, int W, int H, size_t stride, uint8_t* dst,
                            size_t dstride) {
    const int dw = W / 2, dh = H / 2;
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= dw || y >= dh) return;
    const uint8_t* a = src + (size_t)f * stride * H + (size_t)(2 * y) * stride + 2 * x;
    const uint8_t* b = a + stride;
    dst[(size_t)f * dstride * dh + (size_t)y * dstride + x] = (uint8_t)((a[0] + a[1] + b[0] + b[1] + 2) >> 2);
}

void launch_bgr2gray(const uint8_t* bgr, int W, int H, size_t bstride, uint8_t* gray,
                     size_t gstride, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_bgr2gray, dim3((W + 255) / 256, H, F), dim3(256), 0, st, bgr, W, H,
                       bstride, gray, gstride);
}

void launch_area_half(const uint8_t* src, int W, int H, size_t stride, uint8_t* dst,
                      size_t dstride, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_area_half, dim3((W / 2 + 255) / 256, H / 2, F), dim3(256), 0, st, src, W,
                       H, stride, dst, dstride);
}

// ------------------------------------------------------------------------------------------
// self-test of the cross-lane primitives (DPP wave shifts, permlane swaps) on the device
// ------------------------------------------------------------------------------------------
__global__ void k_selftest(int* fails, uint32_t seed) {
    const int lane = threadIdx.x & 63;
    uint32_t v = (lane * 2654435761u + seed) ^ (seed >> 3);
    v &= 0x7fff7fffu;
    uint32_t prev = lane_from_prev(v, kMaxPair);
    uint32_t next = lane_from_next(v, kMaxPair);
    // shuffles run on all lanes first (a shuffle inside a divergent branch reads inactive lanes)
    const uint32_t sp = (uint32_t)__shfl((int)v, (lane + 63) & 63);
    const uint32_t sn = (uint32_t)__shfl((int)v, (lane + 1) & 63);
    uint32_t exp_prev = lane == 0 ? kMaxPair : sp;
    uint32_t exp_next = lane == 63 ? kMaxPair : sn;
    if (prev != exp_prev) atomicAdd(&fails[0], 1);
    if (next != exp_next) atomicAdd(&fails[1], 1);
    uint32_t m = wave_min_pk(v);
    uint32_t lo = v & 0xffff, hi = v >> 16;
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = min(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    if (m != (lo | (hi << 16))) atomicAdd(&fails[2], 1);
    uint32_t mu = wave_min_u32(v);
    uint32_t e = v;
    for (int o = 32; o > 0; o >>= 1) e = min(e, (uint32_t)__shfl_xor((int)e, o));
    if (mu != e) atomicAdd(&fails[3], 1);
}

// The streaming probe (sdr_stream_probe): the box's copy rate over buffers far larger than the
// caches (2 GiB each way against the 256 MiB Infinity Cache), so a bench line can put the box's
// streaming rate beside its kernels'.  Each thread moves U 16-byte vectors per trip, all U loads
// issued before the first store (a one-load grid-stride loop keeps one load in flight per wave
// and read 4.75-5.0 TB/s in round 5); a workgroup owns a contiguous span per trip, so its waves
// sweep whole DRAM pages.  Variants: U = 4 / 8, plain or non-temporal stores, 4 / 8 / 16
// workgroups a CU; the probe reports the fastest (the yardstick must reach the
// guide's ~6.3 TB/s float4 copy for frac_of_probe to mean anything).
typedef unsigned int probe_u32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stream_probe(const probe_u32x4* __restrict__ src,
                                                      probe_u32x4* __restrict__ dst, size_t n) {
    const size_t span = (size_t)256 * U;  // vectors a workgroup moves per trip
    for (size_t base = (size_t)blockIdx.x * span; base < n; base += (size_t)gridDim.x * span) {
        probe_u32x4 v[U];
        if (base + span <= n) {
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(&src[base + u * 256 + threadIdx.x]);
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (NT) __builtin_nontemporal_store(v[u], &dst[base + u * 256 + threadIdx.x]);
                else dst[base + u * 256 + threadIdx.x] = v[u];
            }
        } else {
            for (int u = 0; u < U; u++) {
                const size_t i = base + u * 256 + threadIdx.x;
                if (i < n) dst[i] = src[i];
            }
        }
    }
}

// read-only (an XOR of every vector, stored only if it matches an unlikely value) and write-only
// forms of the same access shape: the box's HBM rates for the two directions
template <int U>
__global__ __launch_bounds__(256) void k_stream_read(const probe_u32x4* __restrict__ src, probe_u32x4* __restrict__ dst,
                                                     size_t n) {
    const size_t span = (size_t)256 * U;
    probe_u32x4 acc = {0u, 0u, 0u, 0u};
    for (size_t base = (size_t)blockIdx.x * span; base + span <= n; base += (size_t)gridDim.x * span) {
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= __builtin_nontemporal_load(&src[base + u * 256 + threadIdx.x]);
    }
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) dst[threadIdx.x] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void k_stream_write(const probe_u32x4* __restrict__ src, probe_u32x4* __restrict__ dst,
                                                      size_t n) {
    const size_t span = (size_t)256 * U;
    const probe_u32x4 v = {1u, 2u, 3u, (unsigned)blockIdx.x};
    for (size_t base = (size_t)blockIdx.x * span; base + span <= n; base += (size_t)gridDim.x * span) {
#pragma unroll
        for (int u = 0; u < U; u++) dst[base + u * 256 + threadIdx.x] = v;
    }
}

int stream_probe_ex(size_t bytes, int iters, double* out3);
int stream_probe(size_t bytes, int iters, double* gbs) {
    double r[3];
    const int rc = stream_probe_ex(bytes, iters, r);
    if (rc == 0) *gbs = r[0];
    return rc;
}

// out3: the fastest copy (read + write bytes), read-only and write-only rates, GB/s
int stream_probe_ex(size_t bytes, int iters, double* out3) {
    probe_u32x4 *a = nullptr, *b = nullptr;
    const size_t n = bytes / 16;
    if (hipMalloc((void**)&a, n * 16) != hipSuccess) return -1;
    if (hipMalloc((void**)&b, n * 16) != hipSuccess) {
        (void)hipFree(a);
        return -1;
    }
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = -1;
    double best[3] = {0.0, 0.0, 0.0};
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
        hipEventCreate(&e1) == hipSuccess && hipMemsetAsync(a, 1, n * 16, st) == hipSuccess) {
        typedef void (*probe_fn)(const probe_u32x4*, probe_u32x4*, size_t);
        // (kind 0: copy, 1: read, 2: write) -- the copy variants of profiles/r6_copy_rate.txt's best
        const struct { probe_fn f; int kind; } fns[] = {
            {k_stream_probe<4, false>, 0}, {k_stream_probe<4, true>, 0}, {k_stream_probe<8, false>, 0},
            {k_stream_probe<8, true>, 0},  {k_stream_read<4>, 1},        {k_stream_read<8>, 1},
            {k_stream_write<8>, 2}};
        for (int wpc : {2, 4, 8, 16})
            for (const auto& v : fns) {
                const dim3 grid(device_cus() * wpc), blk(256);
                hipLaunchKernelGGL(v.f, grid, blk, 0, st, a, b, n);  // warm
                (void)hipEventRecord(e0, st);
                for (int i = 0; i < iters; i++) hipLaunchKernelGGL(v.f, grid, blk, 0, st, a, b, n);
                (void)hipEventRecord(e1, st);
                float ms = 0.0f;
                if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess &&
                    ms > 0.0f) {
                    const double by = (v.kind == 0 ? 2.0 : 1.0) * (double)(n * 16) * iters;
                    best[v.kind] = std::max(best[v.kind], by / (ms * 1e-3) / 1e9);
                    rc = 0;
                }
            }
    }
    if (rc == 0)
        for (int i = 0; i < 3; i++) out3[i] = best[i];
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(a);
    (void)hipFree(b);
    return rc;
}

int selftest_wave_ops(int* failures) {
    int* d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(int)) != hipSuccess) return -1;
    (void)hipMemset(d, 0, 4 * sizeof(int));
    for (uint32_t s = 1; s < 64; s++) hipLaunchKernelGGL(k_selftest, dim3(4), dim3(256), 0, 0, d, s * 7919u);
    hipError_t e = hipMemcpy(failures, d, 4 * sizeof(int), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? 0 : -1;
}

}  // namespace sdr
