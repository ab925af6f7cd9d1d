// sdr_cost.hip -- A.1 prefilter + BT planes and A.2/A.3 cost volume kernels (CDNA4).
//
//   planes L  u64 [F][3][H][W]  int16 splats of the left image's BT operands at x:
//                               {sob,sob_lo} {sob_hi,raw} {raw_lo,raw_hi}  (each 32-bit half = q|q<<16)
//   planes R  u64 [F][3][H][W]  int16 PAIRS of the right image's operands: q(x) | q(x-1) << 16, so a
//                               lane holding disparities (d, d+1) reads one word for xr = x-d, x-d-1
//   C         s16 [F][H][W1][D] P2 + blockSize^2 box sum of the BT pixel cost
//
// Cost kernel: lanes = disparity pairs (as in the path kernels), each wave walks CW output
// columns; the horizontal window and the vertical running sum live in registers (static ring
// slots by unrolling the row loop by the window height), the right image's pair planes for the
// block's column span are staged in LDS (double-buffered, one barrier per row). The staged R
// pair planes are split into even/odd-x halves: lane p reads entry x - 2p, so with the split
// adjacent lanes read adjacent 8-byte words and ds_read_b64 is bank-conflict free (interleaved,
// the -16 B lane stride hits each bank pair twice per 32-lane group).
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <type_traits>
#include <utility>

namespace sdr {

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
// A.1 prefilter (x-Sobel clipped to [0, 2*ftzero], raw intensity; cols 0 and W-1 of both
// channels = tab[0] = ftzero; rows replicate) + half-sample envelopes (calcPixelCostBT).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prefilter(const uint8_t* __restrict__ Limg,
                                                   const uint8_t* __restrict__ Rimg, size_t stride,
                                                   size_t fstride, int W, int H, int ftzero,
                                                   Planes pl) {
    extern __shared__ uint64_t q6[];  // [W] 6 bytes per pixel
    const int y = blockIdx.x, img = blockIdx.y, f = blockIdx.z;
    const uint8_t* base = (img ? Rimg : Limg) + (size_t)f * fstride;
    const uint8_t* r = base + (size_t)y * stride;
    const uint8_t* n = y > 0 ? r - stride : r;
    const uint8_t* s = y < H - 1 ? r + stride : r;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int sv[3], rv[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            int xx = x + k - 1;
            if (xx <= 0 || xx >= W - 1) {
                sv[k] = ftzero;
                rv[k] = ftzero;
            } else {
                int gr = 2 * (r[xx + 1] - r[xx - 1]) + n[xx + 1] - n[xx - 1] + s[xx + 1] - s[xx - 1];
                gr = gr < -ftzero ? -ftzero : (gr > ftzero ? ftzero : gr);
                sv[k] = gr + ftzero;
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
        q6[x] = q;
    }
    __syncthreads();
    const size_t plane = (size_t)H * W;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        const uint64_t a = q6[x];
        const uint64_t b = q6[x > 0 ? x - 1 : 0];
        uint32_t w[6];
#pragma unroll
        for (int c = 0; c < 6; c++) {
            const uint32_t va = (uint32_t)(a >> (8 * c)) & 0xff, vb = (uint32_t)(b >> (8 * c)) & 0xff;
            w[c] = img ? (va | (vb << 16)) : va * 0x10001u;
        }
        uint64_t* dst = (img ? pl.R + (size_t)f * pl.fstrideR : pl.L + (size_t)f * pl.fstrideL) + (size_t)y * W + x;
        dst[0] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        dst[plane] = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
        dst[2 * plane] = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
    }
}

void launch_prefilter(const uint8_t* L, const uint8_t* R, size_t stride, size_t fstride, int W,
                      int H, int F, int ftzero, const Planes& pl, hipStream_t st) {
    hipLaunchKernelGGL(k_prefilter, dim3(H, 2, F), dim3(256), (size_t)W * 8, st, L, R, stride, fstride,
                       W, H, ftzero, pl);
}

// ------------------------------------------------------------------------------------------
// A.2 + A.3 cost volume
//   C(y, x, d) = P2 + sum_{|j|<=SH2} hsum(clamp(t(y)+j, s0, H-1), x, d),   t(y) = min(y, ylim)
//   hsum(r, x, d) = sum_{|k|<=SW2} BT(r, clamp(x+k, 0, W1-1), d)
// equals OpenCV's running sums in int16 wrap arithmetic, incl. the bottom rows where the running
// sum stops updating (t clamps at ylim = H-1-SH2) and MODE_HH's untouched P2 rows.
// The window is walked over "virtual" rows q = t-SH2 .. t+SH2 (physical row clamp(q, s0, H-1)),
// so the ring of the last NR rows is a plain sliding window with compile-time slots.
// ------------------------------------------------------------------------------------------
// parity half of a staged R plane: >= ceil(STR/2), == 16 (mod 32) so the even/odd halves of a
// 32-lane staging store land on disjoint banks
__host__ __device__ inline int cost_half_r(int STR) { return ((STR + 1) / 2 + 15) / 32 * 32 + 16; }

template <int K>
struct CostCfg {
    static constexpr int CW = K == 1 ? 8 : 4;  // output columns per wave
    // waves per SIMD the register budget is capped for (the ring holds NR x K x CW pairs)
    static constexpr int waves(int NR) { return NR * K <= 5 ? 3 : (NR * K <= 14 ? 2 : 1); }
};

// Birchfield-Tomasi dissimilarity of packed pairs: min(max(0, u-v1, v0-u), max(0, v-u1, u0-v)).
// Operands are in [0, 255], so max(x, 0) of a difference is an unsigned saturating subtract and
// one of each pair is zero: 4 v_pk_sub_u16 (clamp) + 2 v_pk_max_u16 + 1 v_pk_min_u16.
__device__ __forceinline__ uint32_t bt_cost(uint32_t u, uint32_t u0, uint32_t u1, uint32_t v,
                                            uint32_t v0, uint32_t v1) {
    const uint32_t c0 = pk_max_u(pk_sub_usat(u, v1), pk_sub_usat(v0, u));
    const uint32_t c1 = pk_max_u(pk_sub_usat(v, u1), pk_sub_usat(u0, v));
    return pk_min_u(c0, c1);
}

// pix[j] = pix[src] for the columns a block-edge wave sees beyond the image (x clamped to
// [0, W1-1]): J0 = first in-image column (left edge), J1 = last in-image column (right edge)
template <int K, int NC, int J0>
__device__ __forceinline__ void clamp_left(uint32_t (&pix)[K][NC]) {
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int j = 0; j < J0; j++) pix[i][j] = pix[i][J0];
}
template <int K, int NC, int J1>
__device__ __forceinline__ void clamp_right(uint32_t (&pix)[K][NC]) {
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int j = J1 + 1; j < NC; j++) pix[i][j] = pix[i][J1];
}
template <int K, int NC, int... J>
__device__ __forceinline__ void clamp_edges(uint32_t (&pix)[K][NC], int j0, int j1,
                                            std::integer_sequence<int, J...>) {
    ((j0 == J ? clamp_left<K, NC, J>(pix) : void()), ...);
    ((j1 == J ? clamp_right<K, NC, J>(pix) : void()), ...);
}

template <int NR, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CostCfg<K>::waves(NR)))) void k_cost(Geometry g, CostArgs a) {
    constexpr int SW2 = (NR - 1) / 2, SH2 = SW2;
    constexpr int CW = CostCfg<K>::CW;
    constexpr int NC = CW + 2 * SW2;
    constexpr int BCOLS = 4 * CW;
    constexpr int NLV = BCOLS + 2 * SW2;  // staged (virtual) columns of a block
    extern __shared__ uint64_t lds[];
    const int W = g.W, H = g.H, W1 = g.W1, D = g.D;
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int f = blockIdx.z;
    const int bx0 = blockIdx.x * BCOLS;
    const int wx0 = bx0 + wave * CW;
    const int ty0 = a.row_begin + blockIdx.y * a.TY;
    const int ty1 = min(ty0 + a.TY, a.row_end);
    if (ty0 >= ty1) return;
    const uint32_t P2x2 = splat16(g.P2);
    int16_t* out = a.out + (size_t)f * a.out_fstride;

    // output addressing: uniform row base + per-lane byte offset; the wave's column count and
    // the active-lane predicate are hoisted so each row is one exec region of plain stores
    const int ncols = min(CW, W1 - wx0);
    const size_t colstride = (size_t)D * 2;
    auto row_base = [&](int y) {
        return (char*)(out + ((size_t)(y - a.out_row0) * W1 + wx0) * D) + 4 * lane;
    };
    auto emit = [&](int y, auto&& val) __attribute__((always_inline)) {
        char* rb = row_base(y);
#pragma unroll
        for (int i = 0; i < K; i++) {
            if (2 * (lane + 64 * i) < D) {
#pragma unroll
                for (int c = 0; c < CW; c++)
                    if (c < ncols) *(uint32_t*)(rb + c * colstride + 256 * i) = val(i, c);
            }
        }
    };

    // rows [yl, ty1) of MODE_HH keep the initial P2
    int yl = ty1;
    if (a.hh_bottom) yl = max(ty0, min(ty1, max(1, H - SH2)));
    auto emit_p2 = [&](int y) { emit(y, [&](int, int) { return P2x2; }); };
    for (int y = yl; y < ty1; y++) emit_p2(y);
    if (yl <= ty0) return;

    // Staged spans in VIRTUAL columns v = bx0 - SW2 + e (e = 0 .. NLV-1): L at image column
    // minX1 + clamp(v); R pairs for xr = minX1 + v - minD - (D-2) + e', e' = 0 .. NLV+D-3, the
    // right image's pair of disparities (2qp, 2qp+1) of column v at e' = (v - vlo) + D-2 - 2qp.
    // Sources are clamped into the image; columns a wave sees beyond [0, W1) are then replaced
    // by the edge column's pixel cost (clamp_edges), which is what x clamping means.
    const int vlo = bx0 - SW2;
    const int NRP = NLV + D - 2;
    const int STR = BCOLS + 2 * SW2 + D;
    const int HR = cost_half_r(STR);  // entries per parity half of a staged R plane
    const int BUF = 3 * STR + 6 * HR;
    const uint64_t* PLf = a.pl.L + (size_t)f * a.pl.fstrideL;
    const uint64_t* PRf = a.pl.R + (size_t)f * a.pl.fstrideR;
    const size_t plane = (size_t)H * W;

    // ---- staging: rows of the L splat planes and R pair planes into LDS buffer b ----
    // Loads are unconditional with clamped indices (surplus lanes re-load and re-store the last
    // entry, the same value to the same slot): a guarded load makes hipcc branch around it and
    // wait vmcnt(0) right after the prefetch is issued, exposing the full HBM latency per row.
    constexpr int NPR = K;  // R entries per thread per plane: NRP <= 256 * K
    const int il = min(tid, NLV - 1);
    const int gl = g.minX1 + min(max(vlo + il, 0), W1 - 1);
    const int xr0 = g.minX1 + vlo - g.minD - (D - 2);
    int gr[NPR], pr[NPR];
#pragma unroll
    for (int t = 0; t < NPR; t++) {
        const int ir = min(tid + 256 * t, NRP - 1);
        gr[t] = min(max(xr0 + ir, 0), W - 1);
        pr[t] = (ir & 1) * HR + (ir >> 1);
    }
    uint64_t ql[3], qr[3][NPR];
    auto fetch = [&](int r) {
        const uint64_t* prow = PLf + (size_t)r * W;
        const uint64_t* rrow = PRf + (size_t)r * W;
#pragma unroll
        for (int k = 0; k < 3; k++) ql[k] = prow[k * plane + gl];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int t = 0; t < NPR; t++) qr[k][t] = rrow[k * plane + gr[t]];
    };
    auto put = [&](int b) {
        uint64_t* B = lds + (size_t)b * BUF;
        uint64_t* BR = B + 3 * STR;
#pragma unroll
        for (int k = 0; k < 3; k++) B[k * STR + il] = ql[k];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int t = 0; t < NPR; t++) BR[k * 2 * HR + pr[t]] = qr[k][t];
    };

    // per-lane staged R position of column j: (j & 1) * HR + (wave*CW + j) / 2 + (D-2)/2 - qp
    int rpos[K];
    bool act[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
        const int qp = lane + 64 * i;
        act[i] = 2 * qp < D;
        rpos[i] = 3 * STR + wave * (CW / 2) + (act[i] ? (D - 2) / 2 - qp : 0);
    }
    const int lpos = wave * CW;
    // block-edge waves: first / last in-image column among the wave's NC (NC = none)
    const int j0 = max(0, -(wx0 - SW2));
    const int j1 = min(NC - 1, W1 - 1 - (wx0 - SW2));
    const bool edge = (j0 > 0) | (j1 < NC - 1);

    // virtual rows and outputs
    const int ylim = a.ylim, s0 = a.s0;
    const int tfirst = min(ty0, ylim), tlast = min(yl - 1, ylim);
    const int qbeg = tfirst - SH2, qend = tlast + SH2;
    auto phys = [&](int q) { return min(max(q, s0), H - 1); };

    uint32_t ring[NR][K][CW], sum[K][CW];
#pragma unroll
    for (int s = 0; s < NR; s++)
#pragma unroll
        for (int i = 0; i < K; i++)
#pragma unroll
            for (int c = 0; c < CW; c++) ring[s][i][c] = 0;
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int c = 0; c < CW; c++) sum[i][c] = 0;

    fetch(phys(qbeg));
    put(0);
    if (qbeg + 1 <= qend) fetch(phys(qbeg + 1));
    __syncthreads();

    auto row = [&](const int q, auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        const int b = (q - qbeg) & 1;
        if (q + 1 <= qend) {
            put(b ^ 1);
            if (q + 2 <= qend) fetch(phys(q + 2));
        }
        const uint64_t* B = lds + (size_t)b * BUF;
        const uint64_t* BL = B + lpos;
        // pixel costs of the NC columns of this wave, then the horizontal window sums
        uint32_t hs[K][CW];
        uint32_t pix[K][NC];
#pragma unroll
        for (int j = 0; j < NC; j++) {
            // broadcast LDS reads (every lane the same address) of the L operands
            const uint64_t l0 = BL[j], l1 = BL[STR + j], l2 = BL[2 * STR + j];
            const uint32_t u = (uint32_t)l0, u0 = (uint32_t)(l0 >> 32), u1 = (uint32_t)l1;
            const uint32_t ur = (uint32_t)(l1 >> 32), ur0 = (uint32_t)l2, ur1 = (uint32_t)(l2 >> 32);
#pragma unroll
            for (int i = 0; i < K; i++) {
                const uint64_t* BRj = B + rpos[i] + (j & 1) * HR + (j >> 1);
                const uint64_t r0 = BRj[0], r1 = BRj[2 * HR], r2 = BRj[4 * HR];
                const uint32_t bs = bt_cost(u, u0, u1, (uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1);
                const uint32_t br = bt_cost(ur, ur0, ur1, (uint32_t)(r1 >> 32), (uint32_t)r2, (uint32_t)(r2 >> 32));
                pix[i][j] = pk_add(bs, pk_shr2_u(br));
            }
        }
        if (edge) clamp_edges(pix, j0, j1, std::make_integer_sequence<int, NC>{});
#pragma unroll
        for (int i = 0; i < K; i++) {
            uint32_t h = 0;
#pragma unroll
            for (int k = 0; k < 2 * SW2 + 1; k++) h = pk_add(h, pix[i][k]);
            hs[i][0] = h;
#pragma unroll
            for (int c = 1; c < CW; c++) {
                h = pk_sub(pk_add(h, pix[i][c + 2 * SW2]), pix[i][c - 1]);
                hs[i][c] = h;
            }
#pragma unroll
            for (int c = 0; c < CW; c++) {
                sum[i][c] = pk_sub(pk_add(sum[i][c], hs[i][c]), ring[s][i][c]);
                ring[s][i][c] = hs[i][c];
            }
        }
        // emit the output rows centred on t = q - SH2 once the window is full
        if (q - qbeg >= NR - 1) {
            const int t = q - SH2;
            const int ya = (t == tlast) ? max(t, ty0) : t;
            const int yb = (t == tlast) ? yl : t + 1;
            for (int y = ya; y < yb; y++) emit(y, [&](int i, int c) { return pk_add(sum[i][c], P2x2); });
        }
        __syncthreads();
    };
    int qq = qbeg;
    for (; qq + NR - 1 <= qend; qq += NR) unroll_rows(row, qq, std::make_integer_sequence<int, NR>{});
    unroll_rows_tail(row, qq, qend, std::make_integer_sequence<int, NR>{});
}

template <int NR, int K>
static void launch_cost_t(const Geometry& g, CostArgs a, int F, hipStream_t st) {
    constexpr int BCOLS = 4 * CostCfg<K>::CW;
    const int rows = a.row_end - a.row_begin;
    const int STR = BCOLS + 2 * ((NR - 1) / 2) + g.D;
    const size_t lds = (size_t)2 * (3 * STR + 6 * cost_half_r(STR)) * 8;
    const int colblocks = (g.W1 + BCOLS - 1) / BCOLS;
    if (a.TY <= 0) {
        // one full pass of resident blocks: a partial second pass doubles the kernel time, and
        // each block re-walks NR-1 warm-up rows, so use the tallest row band that fills the chip
        static thread_local size_t key = 0;
        static thread_local int slots = 0;
        if (key != lds) {
            int dev = 0, cus = 0, per_cu = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_cost<NR, K>, 256, lds);
            slots = max(1, cus * max(1, per_cu));
            key = lds;
        }
        const int bands = max(1, slots / max(1, colblocks * F));
        a.TY = max(4, (rows + bands - 1) / bands);
    }
    dim3 grid(colblocks, (rows + a.TY - 1) / a.TY, F);
    hipLaunchKernelGGL((k_cost<NR, K>), grid, dim3(256), lds, st, g, a);
}

bool cost_supported(const Geometry& g) { return g.SH2 == g.SW2 && g.SH2 <= 5 && g.D <= 256; }

void launch_cost(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    if (a.row_end <= a.row_begin) return;
    const int NR = 2 * g.SH2 + 1;
    const bool k2 = g.D > 128;
#define SDR_COST(NRV)                                                 \
    case NRV:                                                         \
        if (k2) launch_cost_t<NRV, 2>(g, a, F, st);                   \
        else launch_cost_t<NRV, 1>(g, a, F, st);                      \
        break;
    switch (NR) {
        SDR_COST(1) SDR_COST(3) SDR_COST(5) SDR_COST(7) SDR_COST(9) SDR_COST(11)
        default: break;
    }
#undef SDR_COST
}

}  // namespace sdr
