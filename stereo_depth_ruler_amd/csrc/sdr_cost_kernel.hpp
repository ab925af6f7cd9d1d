// sdr_cost_kernel.hpp -- the A.2/A.3 cost-volume kernel template (k_cost<NR, K, CN>), shared by
// sdr_cost.hip (gray input, CN = 1) and sdr_cost3.hip (3-channel input, CN = 3) so that the two
// sets of instantiations compile in parallel.  See sdr_cost.hip for the layouts.
#pragma once
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <type_traits>
#include <utility>

namespace sdr {

// ------------------------------------------------------------------------------------------
// A.2 + A.3 cost volume
//   C(y, x, d) = P2 + sum_{|j|<=SH2} hsum(clamp(t(y)+j, s0, H-1), x, d),   t(y) = min(y, ylim)
//   hsum(r, x, d) = sum_{|k|<=SW2} BT(r, clamp(x+k, 0, W1-1), d)
// equals OpenCV's running sums in int16 wrap arithmetic, incl. the bottom rows where the running
// sum stops updating (t clamps at ylim = H-1-SH2) and MODE_HH's untouched P2 rows.  The sums are
// taken in the other order here, vertical first (V(x) = sum over the window's rows of BT(x)),
// then horizontal over the V of the clamped columns: the same int16 wrap sum.
// The window is walked over "virtual" rows q = t-SH2 .. t+SH2 (physical row clamp(q, s0, H-1)),
// so the ring of the last NR rows is a plain sliding window with compile-time slots.
// ------------------------------------------------------------------------------------------
// parity half of a staged R plane, in 8-byte entries: >= ceil(STR/2) and == 8 (mod 16).  A
// ds_write_b64 is serviced in 16-lane groups on 32 banks ((a/4) mod 32): the group's 8 even lanes
// store 64 consecutive bytes into one half and its 8 odd lanes the same bytes of the other, so
// the halves must sit 64 bytes apart mod 128 to take disjoint banks (at == 16 (mod 32), 128 bytes
// apart, every staging store was 2-way conflicted: C2 1.07 M conflict cycles a launch).  The
// reads are ds_read_b64 of 32 consecutive entries, conflict-free at any offset.
__host__ __device__ inline int cost_half_r(int STR) { return ((STR + 1) / 2 + 7) / 16 * 16 + 8; }

template <int NR, int K, int CN>
struct CostCfg {
    static constexpr int SW2 = (NR - 1) / 2;
    static constexpr int BCOLS = K == 1 ? 32 : 16;  // output columns of a block
    // waves per block.  8 (a ring of 5 pixel-cost columns per wave instead of 9: 158 -> 120 VGPRs,
    // 4 waves per SIMD instead of 3) measured slower on C2, 79.3 -> 85.3 us: the row barrier then
    // syncs twice the waves and the horizontal sums read 2 halo columns per 4 outputs, not per 8
    static constexpr int NW = 4;
    static constexpr int NT = 64 * NW;              // threads per block
    static constexpr int CW = BCOLS / NW;           // output columns per wave (horizontal sums)
    static constexpr int NPB = BCOLS + 2 * SW2;     // pixel-cost columns the block needs
    static constexpr int PCW = (NPB + NW - 1) / NW;  // pixel-cost columns per wave: p = wave + NW*jj
    static constexpr int NLV = NW * PCW;             // staged virtual columns
    // row prefetch depth and the row loop's unroll: U covers the ring slot (% NR), the LDS
    // double buffer (% 2) and the prefetch register slot (% PD) statically
    // (two rows: deeper prefetch costs registers, i.e. resident blocks, and measured slower)
#ifndef SDR_COST_PD
#define SDR_COST_PD 2
#endif
    static constexpr int PD = SDR_COST_PD;
    static constexpr int gcd(int a, int b) { return b ? gcd(b, a % b) : a; }
    static constexpr int U = 2 * NR / gcd(2 * NR, PD) * PD;  // lcm(2 NR, PD)
    // LDS bytes: two staging buffers (R: 3 pair planes x 2 parity halves, L: 4 words a column,
    // each per operand set) + two column-sum buffers
    static size_t lds_bytes(int D) {
        return (size_t)2 * 6 * CN * cost_half_r(NLV + D) * 8 + (size_t)2 * NLV * 16 * CN +
               (size_t)2 * NLV * K * 64 * 4;
    }
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
// a 16-bit half of a word broadcast to both halves: folds into the packed op as an op_sel
// operand selection
__device__ __forceinline__ uint32_t half_lo(uint32_t w) {
    const u16x2 v = as_u16x2(w);
    return as_u32(__builtin_shufflevector(v, v, 0, 0));
}
__device__ __forceinline__ uint32_t half_hi(uint32_t w) {
    const u16x2 v = as_u16x2(w);
    return as_u32(__builtin_shufflevector(v, v, 1, 1));
}

template <int NR, int K, int CN, bool EDGE>
__device__ __forceinline__ void cost_block(const Geometry& g, const CostArgs& a, uint64_t* lds,
                                           int bx, int f, int ty0, int ty1) {
    using Cfg = CostCfg<NR, K, CN>;
    constexpr int SW2 = Cfg::SW2, SH2 = SW2, BCOLS = Cfg::BCOLS, CW = Cfg::CW;
    constexpr int PCW = Cfg::PCW, NLV = Cfg::NLV, PD = Cfg::PD, U = Cfg::U;
    static_assert(U % PD == 0 && U % NR == 0 && U % 2 == 0, "static slots");
    const int W = g.W, H = g.H, W1 = g.W1, D = g.D;
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bx0 = bx * BCOLS;
    const uint32_t P2x2 = splat16(g.P2);
    int16_t* out = a.out + (size_t)f * a.out_fstride;

    // output addressing: the wave's first row and column in a buffer resource, rows and columns
    // as scalar offsets, the lane's pair as the one vector offset.  Lanes past the last
    // disparity pair alias it (they compute and store the same value to the same word), so every
    // store is unconditional and the number of stores per row is static: hipcc then counts the
    // outstanding stores exactly and does not wait for the row prefetches behind them.
    const int ox0 = bx0 + wave * CW;
    const int ncols = EDGE ? min(CW, W1 - ox0) : CW;
    const uint32_t colb = (uint32_t)D * 2, rowb = (uint32_t)W1 * colb;
    const Rsrc rO = rsrc_at(out + ((size_t)(ty0 - a.out_row0) * W1 + ox0) * D);
    const Rsrc rSink = rsrc_at(a.sink + (size_t)ox0 * D);
    int qpc[K];
    uint32_t vo[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
        qpc[i] = min(lane + 64 * i, D / 2 - 1);
        vo[i] = 4 * qpc[i];
    }
    auto emit_at = [&](Rsrc r, uint32_t so, auto&& val) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < K; i++)
#pragma unroll
            for (int c = 0; c < CW; c++)
                if (!EDGE || c < ncols) __builtin_amdgcn_raw_buffer_store_b32(val(i, c), r, vo[i], so + c * colb, 0);
    };
    auto emit = [&](int y, auto&& val) __attribute__((always_inline)) { emit_at(rO, (uint32_t)(y - ty0) * rowb, val); };

    // rows [yl, ty1) of MODE_HH keep the initial P2
    int yl = ty1;
    if (a.hh_bottom) yl = max(ty0, min(ty1, max(1, H - SH2)));
    for (int y = yl; y < ty1; y++) emit(y, [&](int, int) { return P2x2; });
    if (yl <= ty0) return;

    // Virtual columns v = vlo + p, p = 0 .. NLV-1; wave w computes the pixel costs of columns
    // p = w + 4*jj.  Left operands are staged for image columns minX1 + clamp(v, 0, W1-1); R pairs
    // for xr = minX1 + vlo - minD - (D-2) + e, e = 0 .. NLV+D-3: the pair of disparities
    // (2qp, 2qp+1) of column p sits at e = p + D-2 - 2qp.  Columns beyond [0, W1) are computed
    // from clamped data and never read: the horizontal sums read the column sums of clamp(v),
    // which is what x clamping means.
    const int vlo = bx0 - SW2;
    const int NRP = NLV + D - 2;
    const int HR = cost_half_r(NLV + D);  // entries per parity half of a staged R plane
    const int BUFR = 6 * HR * CN;                // [3CN planes][2 parity halves][HR]
    uint32_t* LB = (uint32_t*)(lds + 2 * BUFR);  // [2][NLV][CN][4] left operand words
    uint32_t* VB = LB + 2 * NLV * 4 * CN;        // [2][NLV][K][64] column sums
    const uint32_t planeb = (uint32_t)H * W * 8;

    // ---- staging: a row of the R pair planes and of the L pack, global -> registers -> LDS ----
    // Rows are fetched PD rows ahead into PD register slots (slot of row r: (r - qbeg) % PD), so
    // a load has PD row steps to land.  Loads are unconditional with clamped indices and
    // rows (surplus lanes re-load and re-store the last entry, the same value to the same slot):
    // a guarded load makes hipcc branch around it and wait vmcnt(0) right after it is issued.
    // Staging goes through registers, not LDS-direct loads, because the barrier of every row
    // would then wait for all of them.
    constexpr int NT = Cfg::NT, NW = Cfg::NW;
    constexpr int NPR = (NLV + 128 * K - 2 + NT - 1) / NT;  // R entries per thread per plane (NRP <= NLV + D - 2)
    const int xr0 = g.minX1 + vlo - g.minD - (D - 2);
    const Rsrc rR = rsrc_at(a.pl.R + (size_t)f * a.pl.fstrideR);  // < 2 GiB a frame (check_frame)
    const Rsrc rL = rsrc_at(a.pl.L + (size_t)f * a.pl.fstrideL);
    uint32_t gr[NPR];
    int pr[NPR];
#pragma unroll
    for (int t = 0; t < NPR; t++) {
        const int ir = min(tid + NT * t, NRP - 1);
        gr[t] = 8 * min(max(xr0 + ir, 0), W - 1);
        pr[t] = (ir & 1) * HR + (ir >> 1);
    }
    // L word il: column il / 3CN, word il % 3CN (operand set w / 3), staged as 4 words per
    // column and operand set (one 16-byte broadcast)
    constexpr int NLT = (3 * CN * NLV + NT - 1) / NT;  // L words per thread
    uint32_t gl[NLT];
    int pl[NLT];
#pragma unroll
    for (int t = 0; t < NLT; t++) {
        const int il = min(tid + NT * t, 3 * CN * NLV - 1), c = il / (3 * CN), w = il % (3 * CN);
        gl[t] = 4 * (3 * CN * (g.minX1 + min(max(vlo + c, 0), W1 - 1)) + w);
        pl[t] = (c * CN + w / 3) * 4 + w % 3;
    }
    struct Stage {
        uint64_t r[3 * CN][NPR];
        uint32_t l[NLT];
    };
    Stage st[PD];
    auto fetch = [&](int r, Stage& sg) __attribute__((always_inline)) {
        const uint32_t so = (uint32_t)r * W * 8;
#pragma unroll
        for (int k = 0; k < 3 * CN; k++)
#pragma unroll
            for (int t = 0; t < NPR; t++) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rR, gr[t], so + k * planeb, 0);
                sg.r[k][t] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
            }
#pragma unroll
        for (int t = 0; t < NLT; t++)
            sg.l[t] = __builtin_amdgcn_raw_buffer_load_b32(rL, gl[t], (uint32_t)r * W * 12 * CN, 0);
    };
    auto put = [&](int b, const Stage& sg) __attribute__((always_inline)) {
        uint64_t* BR = lds + b * BUFR;
#pragma unroll
        for (int k = 0; k < 3 * CN; k++)
#pragma unroll
            for (int t = 0; t < NPR; t++) BR[k * 2 * HR + pr[t]] = sg.r[k][t];
#pragma unroll
        for (int t = 0; t < NLT; t++) LB[b * NLV * 4 * CN + pl[t]] = sg.l[t];
    };

    // per-lane staged R position of this wave's column jj: (p & 1) * HR + p / 2 + (D-2)/2 - qp
    // with p = wave + NW*jj, i.e. rpos + (NW/2)*jj (interleaved columns: one base register; a wave
    // owning contiguous columns needs two, and hipcc then spends ~40 more VGPRs on the row loop)
    int rpos[K];
#pragma unroll
    for (int i = 0; i < K; i++) rpos[i] = (wave & 1) * HR + (wave >> 1) + (D - 2) / 2 - qpc[i];
    // column sums: written at [p][i][lane], read back for columns clamp(wave*CW + c', plo, phi)
    uint32_t* Vw = VB + (wave * K) * 64 + lane;
    const int plo = SW2 - bx0, phi = W1 - 1 - vlo;

    // virtual rows and outputs
    const int ylim = a.ylim, s0 = a.s0;
    const int tfirst = min(ty0, ylim), tlast = min(yl - 1, ylim);
    const int qbeg = tfirst - SH2, qend = tlast + SH2;
    auto phys = [&](int q) { return min(max(min(q, qend), s0), H - 1); };

    // horizontal sums (+ P2) of the column sums in buffer b
    auto hsum = [&](int b, uint32_t (&hs)[K][CW]) __attribute__((always_inline)) {
        const uint32_t* V = VB + b * (NLV * K * 64) + (wave * CW) * K * 64 + lane;
#pragma unroll
        for (int i = 0; i < K; i++) {
            uint32_t v[CW + 2 * SW2];
#pragma unroll
            for (int c = 0; c < CW + 2 * SW2; c++) {
                int dc = c;  // interior: immediate offsets from one base
                if (EDGE) dc = min(max(wave * CW + c, plo), phi) - wave * CW;
                v[c] = V[(dc * K + i) * 64];
            }
            uint32_t h = P2x2;
#pragma unroll
            for (int k = 0; k < 2 * SW2 + 1; k++) h = pk_add(h, v[k]);
            hs[i][0] = h;
#pragma unroll
            for (int c = 1; c < CW; c++) {
                h = pk_sub(pk_add(h, v[c + 2 * SW2]), v[c - 1]);
                hs[i][c] = h;
            }
        }
    };

    uint32_t ring[NR][K][PCW], vs[K][PCW];
#pragma unroll
    for (int s = 0; s < NR; s++)
#pragma unroll
        for (int i = 0; i < K; i++)
#pragma unroll
            for (int jj = 0; jj < PCW; jj++) ring[s][i][jj] = 0;
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int jj = 0; jj < PCW; jj++) vs[i][jj] = 0;

    fetch(phys(qbeg), st[0]);
    put(0, st[0]);
#pragma unroll
    for (int k = 1; k <= PD; k++) fetch(phys(qbeg + k), st[k % PD]);
    __syncthreads();

    // one barrier per virtual row q = qbeg + j (mod U): (A) horizontal sums + outputs of the
    // column sums row q-1 left in LDS, (B) staging of row q+1 and the fetch of row q+1+PD, (C)
    // pixel costs of row q, the vertical window, its column sums into LDS
    auto row = [&](const int q, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        constexpr int s = j % NR, b = j & 1;
        {
            // output row t = q-1-SH2 < tlast; rows before ty0 (the window's warm-up, or a band in
            // the frozen bottom rows) go to the sink row instead of a branch around the stores
            uint32_t hs[K][CW];
            hsum(b ^ 1, hs);
            const int t = q - 1 - SH2;
            const bool real = t >= ty0;
            emit_at(real ? rO : rSink, real ? (uint32_t)(t - ty0) * rowb : 0u, [&](int i, int c) { return hs[i][c]; });
        }
        put((j + 1) & 1, st[(j + 1) % PD]);
        fetch(phys(q + 1 + PD), st[(j + 1) % PD]);
        const uint64_t* BR = lds + b * BUFR;
        // a broadcast read per column: every lane reads the column's words as one 16-byte access
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* BL = (const u32x4*)(LB + b * NLV * 4 * CN) + wave * CN;
#pragma unroll
        for (int jj = 0; jj < PCW; jj++) {
            uint32_t pix[K];
#pragma unroll
            for (int ch = 0; ch < CN; ch++) {
                // operand set ch (colour: channel ch's Sobel and raw costs add up)
                const u32x4 lw = BL[NW * jj * CN + ch];
                const uint32_t w0 = lw.x, w1 = lw.y, w2 = lw.z;
                const uint32_t u = half_lo(w0), u0 = half_hi(w0), u1 = half_lo(w1);
                const uint32_t ur = half_hi(w1), ur0 = half_lo(w2), ur1 = half_hi(w2);
#pragma unroll
                for (int i = 0; i < K; i++) {
                    const uint64_t* BRj = BR + rpos[i] + (NW / 2) * jj + 6 * ch * HR;
                    const uint64_t r0 = BRj[0], r1 = BRj[2 * HR], r2 = BRj[4 * HR];
                    const uint32_t bs = bt_cost(u, u0, u1, (uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1);
                    const uint32_t br = bt_cost(ur, ur0, ur1, (uint32_t)(r1 >> 32), (uint32_t)r2, (uint32_t)(r2 >> 32));
                    const uint32_t pc = pk_add(bs, pk_shr2_u(br));
                    pix[i] = ch == 0 ? pc : pk_add(pix[i], pc);
                }
            }
#pragma unroll
            for (int i = 0; i < K; i++) {
                vs[i][jj] = pk_sub(pk_add(vs[i][jj], pix[i]), ring[s][i][jj]);
                ring[s][i][jj] = pix[i];
            }
        }
        {
            // (partial sums during the warm-up: their horizontal sums go to the sink)
            uint32_t* Vb = Vw + b * (NLV * K * 64);
#pragma unroll
            for (int jj = 0; jj < PCW; jj++)
#pragma unroll
                for (int i = 0; i < K; i++) Vb[(NW * jj * K + i) * 64] = vs[i][jj];
        }
        __syncthreads();
    };
    int qq = qbeg;
    for (; qq + U - 1 <= qend; qq += U) unroll_rows(row, qq, std::make_integer_sequence<int, U>{});
    unroll_rows_tail(row, qq, qend, std::make_integer_sequence<int, U>{});
    // the last window, t = tlast: its rows [max(tlast, ty0), yl) (the frozen bottom rows repeat it)
    uint32_t hs[K][CW];
    hsum((qend - qbeg) & 1, hs);
    for (int y = max(tlast, ty0); y < yl; y++) emit(y, [&](int i, int c) { return hs[i][c]; });
}

template <int NR, int K, int CN>
__global__ __launch_bounds__((CostCfg<NR, K, CN>::NT)) void k_cost(Geometry g, CostArgs a) {
    using Cfg = CostCfg<NR, K, CN>;
    extern __shared__ uint64_t lds[];
    // column blocks of one row band are consecutive logical blocks: they share an XCD, so the
    // right-image rows they all stage (each block reads D-2 columns of halo) are re-read from L2
    const int gx = gridDim.x, gy = gridDim.y;
    const int l = xcd_block(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
    const int bx = l % gx, by = (l / gx) % gy, f = l / (gx * gy);
    // row bands [0, gy - naux) of the frame; the last naux bands are the 3WAY stripe starts
    const int nmain = gy - a.naux;
    CostArgs aa = a;
    int ty0, ty1;
    if (by < nmain) {
        ty0 = a.row_begin + by * a.TY;
        ty1 = min(ty0 + a.TY, a.row_end);
    } else {
        const CostAux& x = a.aux[by - nmain];
        aa.out = x.out;
        aa.out_fstride = a.aux_fstride;
        aa.out_row0 = x.row0;
        aa.s0 = x.s0;
        aa.ylim = x.ylim;
        aa.hh_bottom = 0;
        ty0 = x.row0;
        ty1 = x.row0 + x.rows;
    }
    if (ty0 >= ty1) return;
    const int bx0 = bx * Cfg::BCOLS;
    const Geometry gf = frame_geom(g, f);
    if (bx0 - Cfg::SW2 < 0 || bx0 + Cfg::BCOLS + Cfg::SW2 > g.W1) cost_block<NR, K, CN, true>(gf, aa, lds, bx, f, ty0, ty1);
    else cost_block<NR, K, CN, false>(gf, aa, lds, bx, f, ty0, ty1);
}

template <int NR, int K, int CN>
static void launch_cost_t(const Geometry& g, CostArgs a, int F, hipStream_t st) {
    using Cfg = CostCfg<NR, K, CN>;
    const int rows = max(a.row_end - a.row_begin, 0);
    const size_t lds = Cfg::lds_bytes(g.D);
    const int colblocks = (g.W1 + Cfg::BCOLS - 1) / Cfg::BCOLS;
    if (a.TY <= 0) {
        // one full pass of resident blocks: a partial second pass doubles the kernel time, and
        // each block re-walks NR-1 warm-up rows, so use the tallest row band that fills the chip
        // blocks per CU: a property of the kernel and its LDS (one gfx950 binary), cached per LDS size
        static thread_local size_t key = 0;
        static thread_local int per_cu = 0;
        if (key != lds) {
            per_cu = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_cost<NR, K, CN>, Cfg::NT, lds);
            key = lds;
        }
        const int slots = max(1, device_cus() * max(1, per_cu));
        // the 3WAY stripe-start bands are extra rows of blocks in the same launch: leave them
        // their slots, or the launch spills into a second pass (C4: 828 blocks on 768 slots,
        // 61 -> 35 us)
        const int per_band = max(1, colblocks * F);
        const int avail = max(per_band, slots - a.naux * per_band);
        const int bands = max(1, avail / per_band);
        a.TY = max(4, (rows + bands - 1) / bands);
    }
    if (rows == 0) a.TY = 1;
    dim3 grid(colblocks, (rows + a.TY - 1) / a.TY + a.naux, F);
    hipLaunchKernelGGL((k_cost<NR, K, CN>), grid, dim3(Cfg::NT), lds, st, g, a);
}

}  // namespace sdr
