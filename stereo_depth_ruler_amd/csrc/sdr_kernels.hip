// sdr_kernels.hip -- HIP/CDNA4 kernels of the stereo disparity hot path.
//
// Data layout in HBM (per frame):
//   planes  u64 [2][H][W]       Birchfield-Tomasi planes per image pixel, bytes
//                               {sobel, sobel_lo, sobel_hi, raw, raw_lo, raw_hi, 0, 0}
//   C       s16 [H][W1][D]      cost volume P2 + box(BT)                 
//   S       s16 [H][W1][D]      sum of path costs L_r                    (A.4-A.7)
//   wta     u32 [H][W1]         (minS << 16 | bestDisp) or ~0 (uniqueness reject)
//   disp    s16 [H][W]          1/16-px disparity, raw -> LR -> median -> speckle
//
// Every kernel is integer min/add work bound by HBM traffic, not MFMA.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <float.h>

#include <type_traits>

namespace sdr {

// ------------------------------------------------------------------------------------------
// fill
// ------------------------------------------------------------------------------------------
__global__ void k_fill_s16(int16_t* p, int16_t v, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t step = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += step) p[i] = v;
}

void launch_fill_s16(int16_t* p, int16_t v, size_t n, hipStream_t st) {
    if (!n) return;
    int blocks = (int)min((n + 255) / 256, (size_t)4096);
    hipLaunchKernelGGL(k_fill_s16, dim3(blocks), dim3(256), 0, st, p, v, n);
}

// ------------------------------------------------------------------------------------------
// A.1 prefilter + BT half-sample envelopes (calcPixelCostBT's per-row preprocessing).
// cols 0 and W-1 of both channels hold tab[0] = ftzero; rows replicate at top/bottom.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prefilter(const uint8_t* __restrict__ L,
                                                   const uint8_t* __restrict__ R, size_t stride,
                                                   size_t fstride, int W, int H, int ftzero,
                                                   uint64_t* __restrict__ planes) {
    const int y = blockIdx.x, img = blockIdx.y, f = blockIdx.z;
    const uint8_t* base = (img ? R : L) + (size_t)f * fstride;
    const uint8_t* r = base + (size_t)y * stride;
    const uint8_t* n = y > 0 ? r - stride : r;
    const uint8_t* s = y < H - 1 ? r + stride : r;
    uint64_t* out = planes + ((size_t)f * 2 + img) * (size_t)H * W + (size_t)y * W;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int sv[3], rv[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            int xx = x + k - 1;
            if (xx <= 0 || xx >= W - 1) {
                sv[k] = ftzero;
                rv[k] = ftzero;
            } else {
                int g = 2 * (r[xx + 1] - r[xx - 1]) + n[xx + 1] - n[xx - 1] + s[xx + 1] - s[xx - 1];
                g = g < -ftzero ? -ftzero : (g > ftzero ? ftzero : g);
                sv[k] = g + ftzero;
                rv[k] = r[xx];
            }
        }
        uint64_t q = 0;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int* val = c == 0 ? sv : rv;
            int v = val[1];
            int a = x < W - 1 ? (v + val[2]) >> 1 : v;
            int b = x > 0 ? (v + val[0]) >> 1 : v;
            int lo = min(min(a, b), v), hi = max(max(a, b), v);
            q |= (uint64_t)v << (24 * c);
            q |= (uint64_t)lo << (24 * c + 8);
            q |= (uint64_t)hi << (24 * c + 16);
        }
        out[x] = q;
    }
}

void launch_prefilter(const uint8_t* L, const uint8_t* R, size_t stride, size_t fstride, int W,
                      int H, int F, int ftzero, uint64_t* planes, hipStream_t st) {
    hipLaunchKernelGGL(k_prefilter, dim3(H, 2, F), dim3(256), 0, st, L, R, stride, fstride, W, H,
                       ftzero, planes);
}

// ------------------------------------------------------------------------------------------
// A.2 + A.3 cost volume: C(y, x, d) = P2 + sum_{|j|<=SH2} hsum(clamp(t(y)+j, s0, H-1), x, d),
//   hsum(r, x, d) = sum_{|k|<=SW2} BT(r, clamp(x+k, 0, W1-1), d),   t(y) = min(y, ylim).
// This closed form equals OpenCV's running sums (int16 wrap arithmetic is associative), incl.
// the bottom rows where the running sum stops updating (t clamps at ylim = H-1-SH2).
// One block = TX matched columns x TY output rows x all D.  Per input row r the block stages
// the BT planes in LDS, computes one row of pixel costs (TX+2*SW2 columns), the horizontal box
// sums into an LDS ring of 2*SH2+1 rows, and emits every output row whose window is complete.
// ------------------------------------------------------------------------------------------
int cost_lds_bytes(const Geometry& g, int TX) {
    const int NXP = TX + 2 * g.SW2, Dh = g.D / 2, NR = 2 * g.SH2 + 1;
    return 4 * (6 * NXP + 6 * (NXP + g.D) + NXP * (Dh + 1) + NR * TX * Dh);
}

__global__ __launch_bounds__(256) void k_cost(Geometry g, CostArgs a) {
    extern __shared__ __align__(16) uint32_t smem[];
    const int TX = a.TX, D = g.D, Dh = D / 2, SW2 = g.SW2, SH2 = g.SH2, W1 = g.W1, H = g.H;
    const int W = g.W;
    const int NXP = TX + 2 * SW2, NRP = NXP + D, PS = Dh + 1, NR = 2 * SH2 + 1;
    uint32_t* Lsp = smem;
    uint32_t* Rpr = Lsp + 6 * NXP;
    uint32_t* pix = Rpr + 6 * NRP;
    uint32_t* ring = pix + NXP * PS;
    const int tid = threadIdx.x;
    const int f = blockIdx.z;
    const int mx0 = blockIdx.x * TX;
    const int ty0 = a.row_begin + blockIdx.y * a.TY;
    const int ty1 = min(ty0 + a.TY, a.row_end);
    if (ty0 >= ty1) return;

    const uint64_t* PL = a.planes + (size_t)f * a.planes_fstride;
    const uint64_t* PR = PL + (size_t)H * W;
    int16_t* out = a.out + (size_t)f * a.out_fstride;
    const uint32_t P2x2 = splat16(g.P2);
    const int nout = TX * Dh;

    // rows [yl, ty1) of MODE_HH keep the initial P2
    int yl = ty1;
    if (a.hh_bottom) {
        int first_p2 = max(1, H - SH2);
        yl = max(ty0, min(ty1, first_p2));
    }

    if (yl > ty0) {
        const int ylim = a.ylim, s0 = a.s0;
        const int rmin = max(min(ty0, ylim) - SH2, s0);
        const int rmax = min(min(yl - 1, ylim) + SH2, H - 1);
        const int mlo = min(max(mx0 - SW2, 0), W1 - 1);
        const int mhi = min(max(mx0 + TX + SW2 - 1, 0), W1 - 1);
        const int xr_lo = mlo + g.minX1 - g.minD - D + 1;
        const int nrp = (mhi + g.minX1 - g.minD) - xr_lo + 1;
        // per-thread item walks without runtime div/mod: item idx = tid + 256*it
        const int npix = NXP * Dh;
        const int pj0 = tid % NXP, pp0 = tid / NXP, pdj = 256 % NXP, pdp = 256 / NXP;
        const int ox0 = tid / Dh, op0 = tid % Dh, odx = 256 / Dh, odp = 256 % Dh;
        int ynext = ty0;
        int slot = 0;  // ring slot of row r
        // staging of row r+1's BT planes is issued while row r computes (registers -> LDS)
        uint64_t ql = 0, qa[2] = {0, 0}, qb[2] = {0, 0};
        auto fetch = [&](int r) {
            const uint64_t* pl = PL + (size_t)r * W;
            const uint64_t* pr = PR + (size_t)r * W;
            if (tid < NXP) ql = pl[min(max(mx0 - SW2 + tid, 0), W1 - 1) + g.minX1];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const int i = tid + 256 * t;
                if (i < nrp) {
                    const int xr = xr_lo + i;
                    qa[t] = pr[xr];
                    qb[t] = pr[max(xr - 1, 0)];
                }
            }
        };
        fetch(rmin);
        for (int r = rmin; r <= rmax; r++, slot = (slot + 1 == NR) ? 0 : slot + 1) {
            if (tid < NXP) {
#pragma unroll
                for (int c = 0; c < 6; c++) Lsp[c * NXP + tid] = (uint32_t)((ql >> (8 * c)) & 0xff) * 0x10001u;
            }
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const int i = tid + 256 * t;
                if (i < nrp) {
#pragma unroll
                    for (int c = 0; c < 6; c++)
                        Rpr[c * NRP + i] = (uint32_t)((qa[t] >> (8 * c)) & 0xff) |
                                           ((uint32_t)((qb[t] >> (8 * c)) & 0xff) << 16);
                }
            }
            if (r < rmax) fetch(r + 1);
            __syncthreads();
            {
                int j = pj0, p = pp0;
                for (int idx = tid; idx < npix; idx += 256) {
                    const int m = min(max(mx0 - SW2 + j, 0), W1 - 1);
                    const int xi = (m + g.minX1 - g.minD - 2 * p) - xr_lo;
                    uint32_t tot = 0;
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        uint32_t u = Lsp[(3 * c) * NXP + j], u0 = Lsp[(3 * c + 1) * NXP + j],
                                 u1 = Lsp[(3 * c + 2) * NXP + j];
                        uint32_t v = Rpr[(3 * c) * NRP + xi], v0 = Rpr[(3 * c + 1) * NRP + xi],
                                 v1 = Rpr[(3 * c + 2) * NRP + xi];
                        uint32_t c0 = pk_max(pk_max(pk_sub(u, v1), pk_sub(v0, u)), 0u);
                        uint32_t c1 = pk_max(pk_max(pk_sub(v, u1), pk_sub(u0, v)), 0u);
                        uint32_t bt = pk_min(c0, c1);
                        if (c == 1) bt = as_u32(as_s16x2(bt) >> (short)2);
                        tot = pk_add(tot, bt);
                    }
                    pix[j * PS + p] = tot;
                    j += pdj;
                    p += pdp;
                    if (j >= NXP) { j -= NXP; p++; }
                }
            }
            __syncthreads();
            {
                uint32_t* rrow = ring + slot * nout;
                int x = ox0, p = op0;
                for (int idx = tid; idx < nout; idx += 256) {
                    uint32_t sum = 0;
                    const uint32_t* pc = pix + x * PS + p;
                    for (int k = 0; k <= 2 * SW2; k++) sum = pk_add(sum, pc[k * PS]);
                    rrow[idx] = sum;
                    x += odx;
                    p += odp;
                    if (p >= Dh) { p -= Dh; x++; }
                }
            }
            // emit output rows whose box window [t-SH2, t+SH2] is complete (same thread mapping
            // as the ring writes above, so no barrier is needed)
            while (ynext < yl && min(min(ynext, ylim) + SH2, H - 1) <= r) {
                const int t = min(ynext, ylim);
                int16_t* orow = out + ((size_t)(ynext - a.out_row0) * W1) * D;
                int x = ox0, p = op0;
                for (int idx = tid; idx < nout; idx += 256) {
                    if (mx0 + x < W1) {
                        uint32_t sum = P2x2;
                        for (int jj = -SH2; jj <= SH2; jj++) {
                            const int rr = min(max(t + jj, s0), H - 1);
                            int sl = slot - (r - rr);
                            sl += sl < 0 ? NR : 0;
                            sum = pk_add(sum, ring[sl * nout + idx]);
                        }
                        *(uint32_t*)(orow + (size_t)(mx0 + x) * D + 2 * p) = sum;
                    }
                    x += odx;
                    p += odp;
                    if (p >= Dh) { p -= Dh; x++; }
                }
                ynext++;
            }
        }
    }
    for (int y = max(yl, ty0); y < ty1; y++) {
        int16_t* orow = out + ((size_t)(y - a.out_row0) * W1) * D;
        for (int idx = tid; idx < nout; idx += 256) {
            const int x = idx / Dh, p = idx - x * Dh;
            if (mx0 + x < W1) *(uint32_t*)(orow + (size_t)(mx0 + x) * D + 2 * p) = P2x2;
        }
    }
}

void launch_cost(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    int rows = a.row_end - a.row_begin;
    if (rows <= 0) return;
    dim3 grid((g.W1 + a.TX - 1) / a.TX, (rows + a.TY - 1) / a.TY, F);
    hipLaunchKernelGGL(k_cost, grid, dim3(256), cost_lds_bytes(g, a.TX), st, g, a);
}

// ------------------------------------------------------------------------------------------
// A.4-A.8 path aggregation.  One wave64 = one scanline chain; lane l holds disparities
// [l*DPL, l*DPL+DPL) as DPL/2 packed int16 pairs.  Per step:
//   L = C + min(Lp, min(Lp[d-1], Lp[d+1]) + P1, minLp + P2) - (minLp + P2)
// S is written (first path), accumulated with int16 saturation (middle paths), or, for the
// last path, completed in registers and reduced to the WTA disparity right away (S never
// written back).  C/S loads are software-pipelined PF steps ahead.
// ------------------------------------------------------------------------------------------
template <int K>
struct Regs {
    uint32_t r[K];
};

// Unconditional loads: the caller clamps addresses into the buffer, so no exec-masked branch
// splits the software pipeline (a masked load makes hipcc fall back to s_waitcnt vmcnt(0)).
template <int K>
__device__ __forceinline__ Regs<K> load_regs(const int16_t* p) {
    Regs<K> v;
    if constexpr (K == 1) {
        v.r[0] = *(const uint32_t*)p;
    } else if constexpr (K == 2) {
        uint2 t = *(const uint2*)p;
        v.r[0] = t.x;
        v.r[1] = t.y;
    } else {
        uint4 t = *(const uint4*)p;
        v.r[0] = t.x; v.r[1] = t.y; v.r[2] = t.z; v.r[3] = t.w;
    }
    return v;
}

template <int K>
__device__ __forceinline__ void store_regs(int16_t* p, const Regs<K>& v) {
    if constexpr (K == 1) {
        *(uint32_t*)p = v.r[0];
    } else if constexpr (K == 2) {
        *(uint2*)p = make_uint2(v.r[0], v.r[1]);
    } else {
        *(uint4*)p = make_uint4(v.r[0], v.r[1], v.r[2], v.r[3]);
    }
}

template <typename F, int... J>
__device__ __forceinline__ void unroll_steps(F& f, int k0, std::integer_sequence<int, J...>) {
    (f(k0 + J, std::integral_constant<int, J>{}), ...);
}
template <typename F, int... J>
__device__ __forceinline__ void unroll_tail(F& f, int k0, int len, std::integer_sequence<int, J...>) {
    ((k0 + J < len ? f(k0 + J, std::integral_constant<int, J>{}) : void()), ...);
}

// trunc(n / d) for d >= 1 and |n / d| < 2^20 without a divide loop: float estimate, then one
// exact integer correction step (the quotients here are in [-9, 9]).
__device__ __forceinline__ int div_trunc_small(int n, int d) {
    const int an = abs(n);
    int q = (int)((float)an * __builtin_amdgcn_rcpf((float)d));
    const int r = an - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return n < 0 ? -q : q;
}

struct Chain {
    int x0, y0, dx, dy, len, kwrite;
};

__device__ __forceinline__ Chain make_chain(const Geometry& g, const PathArgs& a, int c) {
    Chain ch;
    const int W1 = g.W1, H = g.H;
    ch.kwrite = 0;
    switch (a.dir) {
    case DIR_E: ch.x0 = 0; ch.y0 = c; ch.dx = 1; ch.dy = 0; ch.len = W1; break;
    case DIR_W: ch.x0 = W1 - 1; ch.y0 = c; ch.dx = -1; ch.dy = 0; ch.len = W1; break;
    case DIR_S:
        ch.x0 = c; ch.y0 = a.ybeg; ch.dx = 0; ch.dy = 1; ch.len = a.yend - a.ybeg;
        ch.kwrite = a.write_from - a.ybeg;
        break;
    case DIR_N: ch.x0 = c; ch.y0 = H - 1; ch.dx = 0; ch.dy = -1; ch.len = H; break;
    case DIR_SE:
        if (c < W1) { ch.x0 = c; ch.y0 = 0; } else { ch.x0 = 0; ch.y0 = c - W1 + 1; }
        ch.dx = 1; ch.dy = 1; ch.len = min(W1 - ch.x0, H - ch.y0);
        break;
    case DIR_SW:
        if (c < W1) { ch.x0 = c; ch.y0 = 0; } else { ch.x0 = W1 - 1; ch.y0 = c - W1 + 1; }
        ch.dx = -1; ch.dy = 1; ch.len = min(ch.x0 + 1, H - ch.y0);
        break;
    case DIR_NE:
        if (c < W1) { ch.x0 = c; ch.y0 = H - 1; } else { ch.x0 = 0; ch.y0 = H - 2 - (c - W1); }
        ch.dx = 1; ch.dy = -1; ch.len = min(W1 - ch.x0, ch.y0 + 1);
        break;
    default: /* DIR_NW */
        if (c < W1) { ch.x0 = c; ch.y0 = H - 1; } else { ch.x0 = W1 - 1; ch.y0 = H - 2 - (c - W1); }
        ch.dx = -1; ch.dy = -1; ch.len = min(ch.x0 + 1, ch.y0 + 1);
        break;
    }
    return ch;
}

template <int DPL, int SMODE, bool PAD>
__global__ __launch_bounds__(256) void k_path(Geometry g, PathArgs a, int nchains) {
    constexpr int K = DPL / 2;
    constexpr int PF = 16;
    const int lane = threadIdx.x & 63;
    // wave-uniform chain index in an SGPR: all chain control flow stays scalar
    const int chain = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int f = blockIdx.y;
    if (chain >= nchains) return;
    const Chain ch = make_chain(g, a, chain);
    if (ch.len <= 0) return;

    const int D = g.D, W1 = g.W1;
    const bool active = !PAD || lane * DPL < D;
    // inactive (padding) lanes read the pixel's last word and discard it
    const int loff = (PAD ? min(lane, D / DPL - 1) : lane) * DPL;
    const ptrdiff_t pstep = (ptrdiff_t)(ch.dy * W1 + ch.dx) * D;
    const size_t p0 = ((size_t)ch.y0 * W1 + ch.x0) * D;
    // chain base pointers (C, S and, for 3WAY stripe starts, the stripe-local C rows which a
    // DIR_S chain starting at aux_row0 reads for its first aux_rows steps)
    const int16_t* cb = a.C + (size_t)f * a.cs_fstride + p0 + loff;
    int16_t* sb = a.S + (size_t)f * a.cs_fstride + p0 + loff;
    const int naux = a.Caux ? a.aux_rows : 0;
    const int16_t* ab = a.Caux ? a.Caux + (size_t)f * a.aux_fstride + (size_t)ch.x0 * D + loff : cb;
    const int last = ch.len - 1;

    auto cptr = [&](int k) -> const int16_t* {
        return (k < naux ? ab : cb) + (ptrdiff_t)k * pstep;
    };
    auto sptr = [&](int k) -> int16_t* { return sb + (ptrdiff_t)k * pstep; };

    Regs<K> cring[PF], sring[PF];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        cring[j] = load_regs<K>(cptr(min(j, last)));
        if constexpr (SMODE != S_WRITE) sring[j] = load_regs<K>(sptr(min(j, last)));
    }

    Regs<K> Lp;
#pragma unroll
    for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    uint32_t delta2 = P2x2;

    int16_t* drow = nullptr;
    uint32_t* wrow = nullptr;
    int res_d = 0;
    uint32_t res_w = 0;
    const bool check_uniq = a.uniq > 0 || !a.uniq_simd;
    const int uniq_simd = a.uniq_simd ? 1 : 0;
    // 1/(100-u) rounded so that trunc((double)n * inv100u) == n / (100-u) for 0 <= n < 2^22
    const double inv100u = 1.0 / (double)(100 - a.uniq) * (1.0 + 0x1p-40);
    const int invalid16 = (g.minD - 1) * 16;
    if constexpr (SMODE == S_ADD_WTA) {
        drow = a.disp_raw + (size_t)f * a.disp_fstride;
        wrow = a.wta + (size_t)f * a.wta_fstride;
    }

    // one recurrence step for pixel k of the chain, ring slot j (compile-time)
    auto step = [&](const int k, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        Regs<K> c = cring[j];
        Regs<K> s;
        if constexpr (SMODE != S_WRITE) s = sring[j];
        if constexpr (PAD) {
#pragma unroll
            for (int i = 0; i < K; i++) c.r[i] = active ? c.r[i] : kMaxPair;
        }
        {
            const int kn = min(k + PF, last);
            cring[j] = load_regs<K>(cptr(kn));
            if constexpr (SMODE != S_WRITE) sring[j] = load_regs<K>(sptr(kn));
        }
        const uint32_t up = lane_from_prev(Lp.r[K - 1], kMaxPair);
        const uint32_t dn = lane_from_next(Lp.r[0], kMaxPair);
        Regs<K> L;
        uint32_t m = kMaxPair;
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint32_t dm1 = funnel16(Lp.r[i], i == 0 ? up : Lp.r[i == 0 ? 0 : i - 1]);
            const uint32_t dp1 = funnel16(i == K - 1 ? dn : Lp.r[i == K - 1 ? 0 : i + 1], Lp.r[i]);
            uint32_t t = pk_add_sat(pk_min(dm1, dp1), P1x2);
            t = pk_min(pk_min(t, Lp.r[i]), delta2);
            uint32_t l = pk_sub(pk_add(c.r[i], t), delta2);
            if constexpr (PAD) l = active ? l : kMaxPair;
            L.r[i] = l;
            m = pk_min(m, l);
        }
        m = pk_min(m, funnel16(m, m));
        m = wave_min_pk(m);
        delta2 = pk_add(m, P2x2);
        Lp = L;

        if constexpr (SMODE != S_ADD_WTA) {
            if (k < ch.kwrite) return;  // 3WAY stripe warm-up rows: recurrence only
        }
        if constexpr (SMODE == S_WRITE) {
            if (active) store_regs<K>(sptr(k), L);
        } else if constexpr (SMODE == S_ADD) {
            Regs<K> o;
#pragma unroll
            for (int i = 0; i < K; i++) o.r[i] = pk_add_sat(s.r[i], L.r[i]);
            if (active) store_regs<K>(sptr(k), o);
        } else {
            // ---- A.8 winner-take-all on the completed S of this pixel (branch-free; lane j of
            // the wave keeps step j's result, stored once per PF-block by flush()) ----
            Regs<K> St;
            uint32_t key = 0xffffffffu;
#pragma unroll
            for (int i = 0; i < K; i++) {
                St.r[i] = pk_add_sat(s.r[i], L.r[i]);
                const uint32_t d = (uint32_t)(lane * DPL + 2 * i);
                const uint32_t lo = (uint32_t)((int)(short)(St.r[i] & 0xffff) + 32768);
                const uint32_t hi = (uint32_t)((int)(short)(St.r[i] >> 16) + 32768);
                const uint32_t kk = min((lo << 16) | d, (hi << 16) | (d + 1));
                key = min(key, active ? kk : 0xffffffffu);
            }
            key = __builtin_amdgcn_readfirstlane(wave_min_u32(key));
            const int minS = (int)(key >> 16) - 32768;
            const int best = (int)(key & 0xffff);
            // uniqueness (bitwise, no short-circuit branches): reject if some d with |d-best| > 1
            // has S[d]*(100-u) < minS*100 (scalar rule) / S[d] < (short)(thresh+1) (SIMD rule)
            const int thr16 = (int)(short)((int)((double)(100 * minS) * inv100u) + 1);
            const int lhs_scale = 100 - a.uniq, rhs = minS * 100;
            int bad = 0;
#pragma unroll
            for (int i = 0; i < K; i++) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int d = lane * DPL + 2 * i + h;
                    const int v = (int)(short)(h ? (St.r[i] >> 16) : (St.r[i] & 0xffff));
                    const int cs = (v < thr16) & uniq_simd;
                    const int cc = (v * lhs_scale < rhs) & (uniq_simd ^ 1);
                    bad |= (cs | cc) & (abs(d - best) > 1);
                }
            }
            bad &= (int)active & (int)check_uniq;
            const bool reject = __ballot(bad != 0) != 0;
            // subpixel: d*16 + ((S[d-1]-S[d+1])*16 + den) / (2*den), C truncating division
            const int dm = max(best - 1, 0), dp = min(best + 1, D - 1);
            uint32_t wm = St.r[0], wp = St.r[0];
#pragma unroll
            for (int i = 1; i < K; i++) {
                if (((dm % DPL) >> 1) == i) wm = St.r[i];
                if (((dp % DPL) >> 1) == i) wp = St.r[i];
            }
            const uint32_t am = __builtin_amdgcn_readlane(wm, dm / DPL);
            const uint32_t ap = __builtin_amdgcn_readlane(wp, dp / DPL);
            const int Sm = (int)(short)((dm & 1) ? (am >> 16) : (am & 0xffff));
            const int Sp = (int)(short)((dp & 1) ? (ap >> 16) : (ap & 0xffff));
            const int den = max(Sm + Sp - 2 * minS, 1);
            const int q = div_trunc_small((Sm - Sp) * 16 + den, 2 * den);
            const int d16 = best * 16 + (((0 < best) & (best < D - 1)) ? q : 0);
            const int dval = reject ? invalid16 : d16 + g.minD * 16;
            const uint32_t wval = reject ? 0xffffffffu : (((uint32_t)minS << 16) | (uint32_t)best);
            res_d = lane == j ? dval : res_d;
            res_w = lane == j ? wval : res_w;
        }
    };
    // WTA results of steps [kbase, kbase + n) live in lanes [0, n): one store per block
    auto flush = [&](int kbase, int n) __attribute__((always_inline)) {
        if constexpr (SMODE == S_ADD_WTA) {
            const int k = kbase + lane;
            if (lane < n && k >= ch.kwrite) {
                const int x = ch.x0 + k * ch.dx, y = ch.y0 + k * ch.dy;
                drow[(size_t)y * g.W + x + g.minX1] = (int16_t)res_d;
                wrow[(size_t)y * W1 + x] = res_w;
            }
        }
    };
    int k0 = 0;
    for (; k0 + PF <= ch.len; k0 += PF) {
        unroll_steps(step, k0, std::make_integer_sequence<int, PF>{});
        flush(k0, PF);
    }
    unroll_tail(step, k0, ch.len, std::make_integer_sequence<int, PF - 1>{});
    flush(k0, ch.len - k0);
}

template <int DPL>
static void launch_path_dpl(const Geometry& g, const PathArgs& a, int smode, int nchains, int F,
                            hipStream_t st) {
    dim3 grid((nchains + 3) / 4, F);
    const bool pad = g.D < 64 * DPL;
#define SDR_LAUNCH(SM, PADV) \
    hipLaunchKernelGGL((k_path<DPL, SM, PADV>), grid, dim3(256), 0, st, g, a, nchains)
    if (pad) {
        if (smode == S_WRITE) SDR_LAUNCH(S_WRITE, true);
        else if (smode == S_ADD) SDR_LAUNCH(S_ADD, true);
        else SDR_LAUNCH(S_ADD_WTA, true);
    } else {
        if (smode == S_WRITE) SDR_LAUNCH(S_WRITE, false);
        else if (smode == S_ADD) SDR_LAUNCH(S_ADD, false);
        else SDR_LAUNCH(S_ADD_WTA, false);
    }
#undef SDR_LAUNCH
}

void launch_path(const Geometry& g, const PathArgs& a, int smode, int nchains, int F,
                 hipStream_t st) {
    if (nchains <= 0) return;
    if (g.D <= 128) launch_path_dpl<2>(g, a, smode, nchains, F, st);
    else launch_path_dpl<4>(g, a, smode, nchains, F, st);
}

// ------------------------------------------------------------------------------------------
// A.8 disp2 + A.9 left-right check, one block per (row, frame).  disp2[x2] is the candidate
// with the smallest minS (ties: the largest x, i.e. the first one OpenCV's descending-x loop
// visits); keys (minS << 16 | 0xffff - x) are reduced with LDS atomicMin.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lr(Geometry g, LrArgs a) {
    extern __shared__ int lsm[];
    uint32_t* keys = (uint32_t*)lsm;
    int* disp2 = lsm + g.W;
    const int y = blockIdx.x, f = blockIdx.y, W = g.W, W1 = g.W1;
    const uint32_t kInit = 32767u << 16;
    const int invalid = (g.minD - 1) * 16;
    for (int x = threadIdx.x; x < W; x += blockDim.x) keys[x] = kInit;
    __syncthreads();
    const uint32_t* wrow = a.wta + (size_t)f * a.wta_fstride + (size_t)y * W1;
    for (int x = threadIdx.x; x < W1; x += blockDim.x) {
        uint32_t w = wrow[x];
        if (w == 0xffffffffu) continue;
        int best = (int)(w & 0xffff);
        int x2 = x + g.minX1 - best - g.minD;
        if (x2 >= 0 && x2 < W) atomicMin(&keys[x2], (w & 0xffff0000u) | (uint32_t)(0xffff - x));
    }
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        uint32_t k = keys[x];
        disp2[x] = k == kInit ? invalid : ((0xffff - (int)(k & 0xffff)) + g.minX1 - x);
    }
    __syncthreads();
    const int16_t* drow = a.disp_raw + (size_t)f * a.disp_fstride + (size_t)y * W;
    int16_t* orow = a.out + (size_t)f * a.disp_fstride + (size_t)y * W;
    const int maxX1 = g.minX1 + W1;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int d1 = drow[x];
        if (x >= g.minX1 && x < maxX1 && d1 != invalid) {
            int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < W && disp2[_x] >= g.minD && abs(disp2[_x] - _d) > a.disp12MaxDiff &&
                0 <= x_ && x_ < W && disp2[x_] >= g.minD && abs(disp2[x_] - d_) > a.disp12MaxDiff)
                d1 = invalid;
        }
        orow[x] = (int16_t)d1;
    }
}

void launch_lr(const Geometry& g, const LrArgs& a, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_lr, dim3(g.H, F), dim3(256), 8 * g.W, st, g, a);
}

// ------------------------------------------------------------------------------------------
// A.10 medianBlur 3x3, replicate border (Devillard's 19-exchange median-of-9 network)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_median3(const int16_t* __restrict__ src,
                                                 int16_t* __restrict__ dst, int W, int H) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const size_t fo = (size_t)blockIdx.z * W * H;
    if (x >= W || y >= H) return;
    int p[9];
    const int xs[3] = {max(x - 1, 0), x, min(x + 1, W - 1)};
    const int ys[3] = {max(y - 1, 0), y, min(y + 1, H - 1)};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) p[i * 3 + j] = src[fo + (size_t)ys[i] * W + xs[j]];
#define SDR_S(a, b) { int t_ = min(p[a], p[b]); p[b] = max(p[a], p[b]); p[a] = t_; }
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 1) SDR_S(3, 4) SDR_S(6, 7)
    SDR_S(1, 2) SDR_S(4, 5) SDR_S(7, 8) SDR_S(0, 3) SDR_S(5, 8) SDR_S(4, 7)
    SDR_S(3, 6) SDR_S(1, 4) SDR_S(2, 5) SDR_S(4, 7) SDR_S(4, 2) SDR_S(6, 4)
    SDR_S(4, 2)
#undef SDR_S
    dst[fo + (size_t)y * W + x] = (int16_t)p[4];
}

void launch_median3(const int16_t* src, int16_t* dst, int W, int H, int F, hipStream_t st) {
    dim3 grid((W + 63) / 64, (H + 3) / 4, F);
    hipLaunchKernelGGL(k_median3, grid, dim3(256), 0, st, src, dst, W, H);
}

// ------------------------------------------------------------------------------------------
// A.11 filterSpeckles as connected-component labelling: 4-neighbours p,q are joined iff
// neither equals newVal and |v(p)-v(q)| <= maxDiff; components of <= maxSize pixels are set to
// newVal.  Lock-free union-find with atomicMin (Playne & Hawick 2018), then flatten, count,
// apply.  The flood fill of OpenCV and CCL give identical components (the join relation is
// symmetric and evaluated on the unmodified image).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int uf_load(int* P, int i) {
    return __hip_atomic_load(&P[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_find(int* P, int x) {
    int p = uf_load(P, x);
    while (p != x) {
        x = p;
        p = uf_load(P, x);
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

// Tile-local pass: 32x32 tile in LDS, union-find with LDS atomics, roots written as global
// pixel indices.  Then only tile borders are merged with global atomics.
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

__global__ __launch_bounds__(256) void k_ccl_local(const int16_t* img, int* P, int* sizes, int W,
                                                   int H, int newVal, int maxDiff) {
    __shared__ int16_t v[kCT * kCT];
    __shared__ int lab[kCT * kCT];
    const int tx0 = blockIdx.x * kCT, ty0 = blockIdx.y * kCT;
    const size_t fo = (size_t)blockIdx.z * W * H;
    const int16_t* I = img + fo;
    for (int i = threadIdx.x; i < kCT * kCT; i += 256) {
        const int gx = tx0 + (i & (kCT - 1)), gy = ty0 + (i >> 5);
        int val = newVal;
        if (gx < W && gy < H) val = I[(size_t)gy * W + gx];
        v[i] = (int16_t)val;
        lab[i] = val != newVal ? i : -1;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCT * kCT; i += 256) {
        if (lab[i] < 0) continue;
        const int lx = i & (kCT - 1), ly = i >> 5;
        const int val = v[i];
        if (lx + 1 < kCT && lab[i + 1] >= 0 && abs(val - v[i + 1]) <= maxDiff) lds_unite(lab, i, i + 1);
        if (ly + 1 < kCT && lab[i + kCT] >= 0 && abs(val - v[i + kCT]) <= maxDiff) lds_unite(lab, i, i + kCT);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCT * kCT; i += 256) {
        const int gx = tx0 + (i & (kCT - 1)), gy = ty0 + (i >> 5);
        if (gx >= W || gy >= H) continue;
        const size_t g = (size_t)gy * W + gx;
        int r = -1;
        if (lab[i] >= 0) {
            const int lr = lds_find(lab, i);
            r = (ty0 + (lr >> 5)) * W + tx0 + (lr & (kCT - 1));
        }
        P[fo + g] = r;
        sizes[fo + g] = 0;
    }
}

// merge across tile borders: vertical borders (x = 32k-1 | 32k) and horizontal ones
__global__ void k_ccl_merge(const int16_t* img, int* P, int W, int H, int newVal, int maxDiff) {
    const size_t fo = (size_t)blockIdx.y * W * H;
    const int16_t* I = img + fo;
    int* Pf = P + fo;
    const int nvx = (W - 1) / kCT, nhy = (H - 1) / kCT;
    const int nv = nvx * H, nh = nhy * W;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nv + nh; t += gridDim.x * blockDim.x) {
        int a, b;
        if (t < nv) {
            const int y = t / nvx, x = (t - y * nvx + 1) * kCT - 1;
            a = y * W + x;
            b = a + 1;
        } else {
            const int u = t - nv;
            const int yb = u / W, x = u - yb * W;
            const int y = (yb + 1) * kCT - 1;
            a = y * W + x;
            b = a + W;
        }
        const int va = I[a], vb = I[b];
        if (va != newVal && vb != newVal && abs(va - vb) <= maxDiff) uf_unite(Pf, a, b);
    }
}

// flatten to roots and count component sizes with one atomic per (wave, root)
__global__ void k_ccl_count(int* P, int* sizes, int n) {
    const size_t fo = (size_t)blockIdx.y * n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int r = -1;
    if (i < n) {
        r = P[fo + i];
        if (r >= 0) {
            r = uf_find(P + fo, r);
            P[fo + i] = r;
        }
    }
    unsigned long long pend = __ballot(r >= 0);
    const int lane = threadIdx.x & 63;
    while (pend) {
        const int src = __ffsll((long long)pend) - 1;
        const int lr = __shfl(r, src);
        const unsigned long long m = __ballot(r == lr) & pend;
        if (lane == src) atomicAdd(&sizes[fo + lr], __popcll(m));
        pend &= ~m;
    }
}

__global__ void k_ccl_apply(int16_t* img, const int* P, const int* sizes, int n, int newVal,
                            int maxSize) {
    const size_t fo = (size_t)blockIdx.y * n;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = P[fo + i];
    if (r >= 0 && sizes[fo + r] <= maxSize) img[fo + i] = (int16_t)newVal;
}

void launch_speckle(int16_t* img, int W, int H, int F, int newVal, int maxSize, int maxDiff,
                    int* labels, int* sizes, hipStream_t st) {
    const int n = W * H;
    hipLaunchKernelGGL(k_ccl_local, dim3((W + kCT - 1) / kCT, (H + kCT - 1) / kCT, F), dim3(256), 0,
                       st, img, labels, sizes, W, H, newVal, maxDiff);
    const int nb = ((W - 1) / kCT) * H + ((H - 1) / kCT) * W;
    if (nb > 0)
        hipLaunchKernelGGL(k_ccl_merge, dim3((unsigned)min((nb + 255) / 256, 1024), F), dim3(256), 0,
                           st, img, labels, W, H, newVal, maxDiff);
    hipLaunchKernelGGL(k_ccl_count, dim3((n + 255) / 256, F), dim3(256), 0, st, labels, sizes, n);
    hipLaunchKernelGGL(k_ccl_apply, dim3((n + 255) / 256, F), dim3(256), 0, st, img, labels, sizes, n,
                       newVal, maxSize);
}

// ------------------------------------------------------------------------------------------
// per-frame minimum (reprojectImageTo3D handleMissingValues needs min(disp))
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
    if (threadIdx.x == 0) atomicMin(&out[blockIdx.y], min(min(wm[0], wm[1]), min(wm[2], wm[3])));
}

__global__ void k_init_i32(int* p, int v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

void launch_min_s16(const int16_t* img, size_t n_per_frame, size_t fstride, int F, int* out_min,
                    hipStream_t st) {
    hipLaunchKernelGGL(k_init_i32, dim3((F + 255) / 256), dim3(256), 0, st, out_min, 32767, F);
    dim3 grid((unsigned)min((n_per_frame + 1023) / 1024, (size_t)128), F);
    hipLaunchKernelGGL(k_min_s16, grid, dim3(256), 0, st, img, n_per_frame, fstride, out_min);
}

// ------------------------------------------------------------------------------------------
// A.12 reprojectImageTo3D: double math, sequential sums from 0, no contraction, Vec3f then
// *(1.0/h3) rounded to float; handleMissing: Z = 10000 where |d - min(disp)| <= FLT_EPSILON.
// ------------------------------------------------------------------------------------------
struct Q16 {
    double q[16];
};

__device__ __forceinline__ void reproject_px(const Q16& Q, int x, int y, double d, double mind,
                                             int hm, float* o) {
#pragma clang fp contract(off)
    const double v0 = (double)x, v1 = (double)y;
    double h[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double s = 0.0;
        s += Q.q[i * 4 + 0] * v0;
        s += Q.q[i * 4 + 1] * v1;
        s += Q.q[i * 4 + 2] * d;
        s += Q.q[i * 4 + 3] * 1.0;
        h[i] = s;
    }
    const double ia = 1.0 / h[3];
    const float X = (float)((double)(float)h[0] * ia);
    const float Y = (float)((double)(float)h[1] * ia);
    float Z = (float)((double)(float)h[2] * ia);
    if (hm && fabs(d - mind) <= (double)FLT_EPSILON) Z = 10000.f;
    o[0] = X;
    o[1] = Y;
    o[2] = Z;
}

__global__ __launch_bounds__(256) void k_reproject_s16(const int16_t* disp, int W, int H,
                                                       size_t dstride, size_t dfstride, Q16 Q,
                                                       int hm, const int* mins, float* xyz,
                                                       size_t xstride, size_t xfstride) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= W) return;
    const int v = disp[(size_t)f * dfstride + (size_t)y * dstride + x];
    const double d = (double)((float)v * 0.0625f);
    const double mind = hm ? (double)((float)mins[f] * 0.0625f) : (double)FLT_MAX;
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
