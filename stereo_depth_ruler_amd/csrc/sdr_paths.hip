// sdr_paths.hip -- A.4-A.9: path aggregation and winner-take-all/LR kernels (CDNA4).
//
// k_paths: every scanline chain of every direction of the mode in ONE launch (a direction table
// in the kernel arguments).  One wave64 = one chain; lane l holds disparities [l*DPL, l*DPL+DPL)
// as DPL/2 packed int16 pairs.  Per step
//     L = C + min(Lp, min(Lp[d-1], Lp[d+1]) + P1, minLp + P2) - (minLp + P2)
// and L is written to the direction's own buffer.  The latency-bound chains (E/W: H chains of
// W1 steps at batch 1) overlap with the bandwidth-bound ones instead of running alone.
// C loads are software-pipelined PF steps ahead with unconditional (clamped) addresses.
//
// k_wta_lr: one workgroup per image row: S = sat(sum_r L_r) per pixel, first-minimum WTA,
// uniqueness test, subpixel fit, disp2 (right-view WTA by LDS atomicMin, ties -> largest x as in
// OpenCV's descending loop) and the left-right check; fully parallel over pixels.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

namespace sdr {

template <int K>
struct Regs {
    uint32_t r[K];
};

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
        static_assert(K % 4 == 0, "K = 1, 2 or a multiple of 4");
#pragma unroll
        for (int j = 0; j < K / 4; j++) {
            uint4 t = ((const uint4*)p)[j];
            v.r[4 * j] = t.x; v.r[4 * j + 1] = t.y; v.r[4 * j + 2] = t.z; v.r[4 * j + 3] = t.w;
        }
    }
    return v;
}

template <int K>
__device__ __forceinline__ void store_regs_nt(int16_t* p, const Regs<K>& v) {
    if constexpr (K == 1) {
        __builtin_nontemporal_store(v.r[0], (uint32_t*)p);
    } else if constexpr (K == 2) {
        __builtin_nontemporal_store(v.r[0], (uint32_t*)p);
        __builtin_nontemporal_store(v.r[1], (uint32_t*)p + 1);
    } else {
#pragma unroll
        for (int j = 0; j < K; j++) __builtin_nontemporal_store(v.r[j], (uint32_t*)p + j);
    }
}

template <int K>
__device__ __forceinline__ void store_regs(int16_t* p, const Regs<K>& v) {
    if constexpr (K == 1) {
        *(uint32_t*)p = v.r[0];
    } else if constexpr (K == 2) {
        *(uint2*)p = make_uint2(v.r[0], v.r[1]);
    } else {
#pragma unroll
        for (int j = 0; j < K / 4; j++)
            ((uint4*)p)[j] = make_uint4(v.r[4 * j], v.r[4 * j + 1], v.r[4 * j + 2], v.r[4 * j + 3]);
    }
}

struct Chain {
    int x0, y0, dx, dy, len, kwrite;
};

__device__ __forceinline__ Chain make_chain(const Geometry& g, const PathDir& d, int c) {
    Chain ch;
    const int W1 = g.W1, H = g.H;
    ch.kwrite = 0;
    switch (d.dir) {
    case DIR_E: ch.x0 = 0; ch.y0 = c; ch.dx = 1; ch.dy = 0; ch.len = W1; break;
    case DIR_W: ch.x0 = W1 - 1; ch.y0 = c; ch.dx = -1; ch.dy = 0; ch.len = W1; break;
    case DIR_S:
        ch.x0 = c; ch.y0 = d.ybeg; ch.dx = 0; ch.dy = 1; ch.len = d.yend - d.ybeg;
        ch.kwrite = d.write_from - d.ybeg;
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

template <int DPL, bool PAD, bool NT = false>
__global__ __launch_bounds__(256) void k_paths(Geometry g, PathLaunch pl) {
    constexpr int K = DPL / 2;
    constexpr int PF = 16;
    const int lane = threadIdx.x & 63;
    // wave-uniform chain index in an SGPR: all chain control flow stays scalar
    const int cg = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int f = blockIdx.y;
    if (cg >= pl.prefix[pl.ndirs]) return;
    int di = 0;
    while (cg >= pl.prefix[di + 1]) di++;
    const PathDir pd = pl.d[di];
    const Chain ch = make_chain(g, pd, cg - pl.prefix[di]);
    if (ch.len <= 0) return;

    const int D = g.D, W1 = g.W1;
    const bool active = !PAD || lane * DPL < D;
    // inactive (padding) lanes read the pixel's last word and discard it
    const int loff = (PAD ? min(lane, D / DPL - 1) : lane) * DPL;
    const ptrdiff_t pstep = (ptrdiff_t)(ch.dy * W1 + ch.dx) * D;
    const size_t p0 = ((size_t)ch.y0 * W1 + ch.x0) * D;
    const int16_t* cb = pl.C + (size_t)f * pl.cs_fstride + p0 + loff;
    int16_t* ob = pd.out + (size_t)f * pl.cs_fstride + p0 + loff;
    // 3WAY stripes: a DIR_S chain starting at aux_row0 reads stripe-local cost rows first
    const int naux = pd.Caux ? pd.aux_rows : 0;
    const int16_t* ab = pd.Caux ? pd.Caux + (size_t)f * pl.aux_fstride + (size_t)ch.x0 * D + loff : cb;
    const int last = ch.len - 1;
    auto cptr = [&](int k) -> const int16_t* { return (k < naux ? ab : cb) + (ptrdiff_t)k * pstep; };

    Regs<K> cring[PF];
#pragma unroll
    for (int j = 0; j < PF; j++) cring[j] = load_regs<K>(cptr(min(j, last)));

    Regs<K> Lp;
#pragma unroll
    for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    uint32_t delta2 = P2x2;  // minLp + P2 with minLp = 0 before the first pixel

    auto step = [&](const int k, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        Regs<K> c = cring[j];
        if constexpr (PAD) {
#pragma unroll
            for (int i = 0; i < K; i++) c.r[i] = active ? c.r[i] : kMaxPair;
        }
        cring[j] = load_regs<K>(cptr(min(k + PF, last)));
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
        if (k >= ch.kwrite && active) {
            if constexpr (NT) store_regs_nt<K>(ob + (ptrdiff_t)k * pstep, L);
            else store_regs<K>(ob + (ptrdiff_t)k * pstep, L);
        }
    };
    int k0 = 0;
    for (; k0 + PF <= ch.len; k0 += PF) unroll_rows(step, k0, std::make_integer_sequence<int, PF>{});
    unroll_rows_tail(step, k0, last, std::make_integer_sequence<int, PF - 1>{});
}

// Path-cost stores are non-temporal (nt): measured on MI355X (C2, 2 frames in flight) +4 % fps
// over default-policy stores, the WTA's re-reads of the L buffers getting faster.
void launch_paths(const Geometry& g, const PathLaunch& pl, int F, hipStream_t st) {
    const int total = pl.prefix[pl.ndirs];
    if (total <= 0) return;
    dim3 grid((total + 3) / 4, F);
    if (g.D <= 128) {
        if (g.D < 128) hipLaunchKernelGGL((k_paths<2, true, true>), grid, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths<2, false, true>), grid, dim3(256), 0, st, g, pl);
    } else {
        if (g.D < 256) hipLaunchKernelGGL((k_paths<4, true, true>), grid, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths<4, false, true>), grid, dim3(256), 0, st, g, pl);
    }
}

// ------------------------------------------------------------------------------------------
// A.8 + A.9 fused: WTA / uniqueness / subpixel / disp2 / LR check, one workgroup per row.
// A pixel's D path-cost sums live on a 16-lane DPP row (DPL disparities per lane), so one wave
// instruction covers 4 pixels: each lane loads DPL*2 contiguous bytes per direction (16 B at
// D = 128: a wave reads 1 KiB of consecutive pixels), and the argmin is a 4-step row reduction.
// ------------------------------------------------------------------------------------------
constexpr int kWtaWaves = 4;   // 4 workgroups/CU at <= 128 VGPRs: 720 rows resident in one pass
constexpr int kWtaGL = 16;     // lanes per pixel
constexpr int kWtaPPW = 4;     // pixels per wave instruction

template <int DPL, bool PAD, int NP>
__global__ __launch_bounds__(64 * kWtaWaves) void k_wta_lr(Geometry g, WtaArgs a) {
    constexpr int K = DPL / 2;
    // directions x pairs x in-flight iterations held in registers: keep the ring near 64 VGPRs
    constexpr int PF = (NP * K <= 16) ? 4 : (NP * K <= 24 ? 3 : 2);
    extern __shared__ int wsm[];
    const int W = g.W, W1 = g.W1, D = g.D;
    uint32_t* keys = (uint32_t*)wsm;   // [W]
    int* disp2 = wsm + W;              // [W]
    int* drow = wsm + 2 * W;           // [W]
    const int y = blockIdx.x, f = blockIdx.y;
    const int lane = threadIdx.x & 63, gl = lane & (kWtaGL - 1), grp = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t kInit = 32767u << 16;
    const int invalid = (g.minD - 1) * 16;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        keys[x] = kInit;
        drow[x] = invalid;
    }
    __syncthreads();

    const bool active = !PAD || gl * DPL < D;
    const int d0 = (PAD ? min(gl, D / DPL - 1) : gl) * DPL;  // padding lanes re-read the last word
    const size_t rowoff = (size_t)f * a.cs_fstride + (size_t)y * W1 * D + d0;
    const bool check_uniq = a.uniq > 0 || !a.uniq_simd;
    const int uniq_simd = a.uniq_simd ? 1 : 0;
    const int lhs_scale = 100 - a.uniq;
    // trunc((double)n * inv100u) == n / (100-u) for 0 <= n < 2^22
    const double inv100u = 1.0 / (double)(100 - a.uniq) * (1.0 + 0x1p-40);
    const int16_t* Lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) Lp[p] = a.L[p] + rowoff;

    // iteration t of this wave covers pixels xw(t) .. xw(t)+3, pixel xw(t)+grp on this lane
    const int nit = (W1 + kWtaPPW * kWtaWaves - 1) / (kWtaPPW * kWtaWaves);
    auto xw = [&](int t) { return (t * kWtaWaves + wave) * kWtaPPW; };
    auto load_px = [&](int t, Regs<K>* dst) __attribute__((always_inline)) {
        const size_t o = (size_t)min(xw(t) + grp, W1 - 1) * D;
#pragma unroll
        for (int p = 0; p < NP; p++) dst[p] = load_regs<K>(Lp[p] + o);
    };

    Regs<K> ring[PF][NP];
#pragma unroll
    for (int s = 0; s < PF; s++) load_px(s, ring[s]);

    auto iter = [&](const int t, auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        Regs<K> St = ring[s][0];
#pragma unroll
        for (int p = 1; p < NP; p++)
#pragma unroll
            for (int i = 0; i < K; i++) St.r[i] = pk_add_sat(St.r[i], ring[s][p].r[i]);
        load_px(t + PF, ring[s]);
        const int x = xw(t) + grp;
        uint32_t key = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint32_t d = (uint32_t)(gl * DPL + 2 * i);
            const uint32_t lo = (uint32_t)((int)(short)(St.r[i] & 0xffff) + 32768);
            const uint32_t hi = (uint32_t)((int)(short)(St.r[i] >> 16) + 32768);
            key = min(key, min((lo << 16) | d, (hi << 16) | (d + 1)));
        }
        key = row16_min_u32(active ? key : 0xffffffffu);
        const int minS = (int)(key >> 16) - 32768;
        const int best = (int)(key & 0xffff);
        // uniqueness: reject if some d with |d-best| > 1 has S[d]*(100-u) < minS*100 (scalar
        // rule) or S[d] < (short)(thresh+1), thresh = (100*minS)/(100-u) (SIMD rule)
        const int thr16 = (int)(short)((int)((double)(100 * minS) * inv100u) + 1);
        const int rhs = minS * 100;
        int bad = 0;
#pragma unroll
        for (int i = 0; i < K; i++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int d = gl * DPL + 2 * i + h;
                const int v = (int)(short)(h ? (St.r[i] >> 16) : (St.r[i] & 0xffff));
                const int cs = (v < thr16) & uniq_simd;
                const int cc = (v * lhs_scale < rhs) & (uniq_simd ^ 1);
                bad |= (cs | cc) & (abs(d - best) > 1);
            }
        }
        bad &= (int)active & (int)check_uniq;
        const bool reject = ((__ballot(bad != 0) >> (16 * grp)) & 0xffffull) != 0;
        // subpixel: d*16 + ((S[d-1]-S[d+1])*16 + den) / (2*den), C truncating division
        const int dm = max(best - 1, 0), dp = min(best + 1, D - 1);
        uint32_t wm = St.r[0], wp = St.r[0];
#pragma unroll
        for (int i = 1; i < K; i++) {
            if (((dm % DPL) >> 1) == i) wm = St.r[i];
            if (((dp % DPL) >> 1) == i) wp = St.r[i];
        }
        const uint32_t am = (uint32_t)__shfl((int)wm, grp * kWtaGL + dm / DPL);
        const uint32_t ap = (uint32_t)__shfl((int)wp, grp * kWtaGL + dp / DPL);
        const int Sm = (int)(short)((dm & 1) ? (am >> 16) : (am & 0xffff));
        const int Sp = (int)(short)((dp & 1) ? (ap >> 16) : (ap & 0xffff));
        const int den = max(Sm + Sp - 2 * minS, 1);
        const int q = div_trunc_small((Sm - Sp) * 16 + den, 2 * den);
        const int d16 = best * 16 + (((0 < best) & (best < D - 1)) ? q : 0);
        if (gl == 0 && !reject && x < W1) {
            drow[x + g.minX1] = d16 + g.minD * 16;
            const int x2 = x + g.minX1 - best - g.minD;
            if (x2 >= 0 && x2 < W) atomicMin(&keys[x2], ((uint32_t)minS << 16) | (uint32_t)(0xffff - x));
        }
    };
    int t = 0;
    for (; t + PF <= nit; t += PF) unroll_rows(iter, t, std::make_integer_sequence<int, PF>{});
    unroll_rows_tail(iter, t, nit - 1, std::make_integer_sequence<int, PF - 1>{});
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        const uint32_t k = keys[x];
        disp2[x] = k == kInit ? invalid : ((0xffff - (int)(k & 0xffff)) + g.minX1 - x);
    }
    __syncthreads();
    int16_t* raw = a.disp_raw + (size_t)f * a.disp_fstride + (size_t)y * W;
    int16_t* out = a.disp_lr + (size_t)f * a.disp_fstride + (size_t)y * W;
    const int maxX1 = g.minX1 + W1;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int d1 = drow[x];
        raw[x] = (int16_t)d1;
        if (x >= g.minX1 && x < maxX1 && d1 != invalid) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = x - _d, x_ = x - d_;
            if (0 <= _x && _x < W && disp2[_x] >= g.minD && abs(disp2[_x] - _d) > a.disp12MaxDiff &&
                0 <= x_ && x_ < W && disp2[x_] >= g.minD && abs(disp2[x_] - d_) > a.disp12MaxDiff)
                d1 = invalid;
        }
        out[x] = (int16_t)d1;
    }
}

template <int DPL, bool PAD>
static void launch_wta_np(const Geometry& g, const WtaArgs& a, int F, hipStream_t st) {
    dim3 grid(g.H, F);
    const size_t lds = (size_t)3 * g.W * 4;
    const dim3 block(64 * kWtaWaves);
    switch (a.npaths) {
    case 3: hipLaunchKernelGGL((k_wta_lr<DPL, PAD, 3>), grid, block, lds, st, g, a); break;
    case 5: hipLaunchKernelGGL((k_wta_lr<DPL, PAD, 5>), grid, block, lds, st, g, a); break;
    default: hipLaunchKernelGGL((k_wta_lr<DPL, PAD, 8>), grid, block, lds, st, g, a); break;
    }
}

void launch_wta_lr(const Geometry& g, const WtaArgs& a, int F, hipStream_t st) {
    // DPL = disparities per lane so that a pixel fits one 16-lane row
    if (g.D <= 64) {
        if (g.D < 64) launch_wta_np<4, true>(g, a, F, st);
        else launch_wta_np<4, false>(g, a, F, st);
    } else if (g.D <= 128) {
        if (g.D < 128) launch_wta_np<8, true>(g, a, F, st);
        else launch_wta_np<8, false>(g, a, F, st);
    } else {
        if (g.D < 256) launch_wta_np<16, true>(g, a, F, st);
        else launch_wta_np<16, false>(g, a, F, st);
    }
}

}  // namespace sdr
