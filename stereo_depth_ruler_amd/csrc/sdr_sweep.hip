// sdr_sweep.hip -- batched MODE_HH (A.6) as two row-synchronous sweeps over a frame, one pixel
// per 16-lane DPP row (CDNA4).
//
// OpenCV's MODE_HH sums eight path directions.  k_paths runs E and W (horizontal chains); the
// other six need their predecessor pixel on the previous row, so a workgroup walks the rows of a
// column tile of a frame in path order:
//   up pass   (bottom to top): N, NE, NW -> their saturated sum, one int16 record per cell;
//   down pass (top to bottom): S, SE, SW, and in the same step A.8 -- S = sat(E + W + up + S + SE
//             + SW), first minimum, uniqueness, subpixel, the right view's WTA keys -- so the
//             down directions' path costs and S never reach HBM.
// Per cell that is 2 B (C read) + 2 B (record write) for the up pass and 2 + 6 B (C and the E, W,
// up records read) for the down pass: with k_cost's C write and k_paths' 8, 20 B a cell, against
// 28 for the round-4 data flow (down pass writing a record that k_south_wta read with C and 3
// more) and 2 + 6 * 8 = 50 for SURVEY.md 8(d)'s canonical model.
//
// Layout: a pixel's D disparities sit on one 16-lane row of a wave, lane gl holding disparities
// [gl * 2DW, gl * 2DW + 2DW) as DW packed int16 pairs (DW = 4 for D <= 128, 8 for D <= 256).  A
// path step is then DW independent packed-word updates per lane (no wait states between them),
// the d-1 / d+1 neighbours across lanes are two DPP row shifts, and the per-pixel minimum that the
// P2 term needs is four DPP row folds; the 64-lane layout of round 4 (one pixel across the wave)
// spent six DPP steps and a readlane on every step's minimum.  A wave holds 4 * M columns: lane
// row r has columns x0 + r * M + m (m < M), so the diagonals' predecessors are the same lane's
// neighbouring slot, except at a lane row's first / last slot, whose predecessor lives in another
// lane row (or wave): every wave publishes those slots' path costs in LDS each row (one barrier
// per row) and reads the neighbours' from the row before.
//
// Across tiles a halo wave on each side recomputes diagonal A (predecessor x - 1: NE / SE) over
// the 4 * MH columns left of the tile, or diagonal B (x + 1: NW / SW) right of it.  A halo column
// whose predecessor lies outside the workgroup goes wrong, the error moving one column inwards per
// row, so the halo feeds the tile exact values for 4 * MH - 1 rows; then the halo waves reload
// their state from the neighbour tiles, which publish their edge columns' path costs through a
// global ring (agent-scope atomic stores, then a row counter per publishing wave; the reader polls
// the counters).  Every tile of a frame in flight must be resident (sweep_shape sizes the grid
// from the occupancy; the engine never has two sweeps in flight), and a wait gives up after
// a.spin polls with *err set: the batch's frames are then overwritten as INVALID after the
// post-filter (launch_sweep_verdict) and the handle's status reports SDR_ERR_DEVICE.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <algorithm>
#include <cstdlib>

namespace sdr {

namespace {

constexpr int kDppRowShr1 = 0x111;  // lane i <- lane i-1 within its 16-lane row
constexpr int kDppRowShl1 = 0x101;  // lane i <- lane i+1 within its 16-lane row
constexpr int kSweepXcds = 8;       // MI355X: blocks are dealt round-robin over 8 XCDs

// slots (columns per lane row) of the own waves and the halo waves of a pass
#ifndef SDR_SW_UP_MO
#define SDR_SW_UP_MO 2
#endif
#ifndef SDR_SW_UP_MH
#define SDR_SW_UP_MH 2
#endif
#ifndef SDR_SW_DN_MO
#define SDR_SW_DN_MO 1
#endif
#ifndef SDR_SW_DN_MH
#define SDR_SW_DN_MH 2
#endif
template <int DW, bool UP>
struct SwShape {
    // the up pass keeps N, NE, NW of M = 2 columns per lane row in registers; the down pass adds
    // the E, W and up records of two rows in flight and the WTA, so its own waves hold one
    // column per lane row, and its halo waves (one diagonal each, no records) two
    static constexpr int MO = UP ? SDR_SW_UP_MO : SDR_SW_DN_MO;
    static constexpr int MH = UP ? SDR_SW_UP_MH : SDR_SW_DN_MH;
};

// the path recurrence of one pixel step on a 16-lane row: L = C + min(Lp, min(Lp[d-1], Lp[d+1]) +
// P1, dp) - dp with dp = min(Lp) + P2, for the lane's DW words; m16 = min of L over the lane's
// disparities (low half).  The row's first lane has no d-1 for its first word: it takes its own
// first word there (whose high half, d+1, repeats the d+1 term of the minimum, so the minimum is
// the one +inf would give); the last lane likewise takes its own last word as d+1 (low half d-2,
// the d-1 term again).  A padded D's inactive lanes hold +inf (kMaxPair), so the last active
// lane's d+1 is +inf through the shift itself.
template <int DW, bool PAD>
__device__ __forceinline__ void step16(const uint32_t (&c)[DW], const uint32_t (&Lp)[DW], uint32_t dp,
                                       uint32_t P1x2, bool active, uint32_t (&L)[DW], uint32_t& m16) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)Lp[0], (int)Lp[DW - 1], kDppRowShr1, 0xf, 0xf, false);
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp((int)Lp[DW - 1], (int)Lp[0], kDppRowShl1, 0xf, 0xf, false);
    uint32_t m = kMaxPair;
#pragma unroll
    for (int i = 0; i < DW; i++) {
        const uint32_t dm1 = funnel16(Lp[i], i == 0 ? up : Lp[i == 0 ? 0 : i - 1]);
        const uint32_t dp1 = funnel16(i == DW - 1 ? dn : Lp[i == DW - 1 ? 0 : i + 1], Lp[i]);
        uint32_t t = pk_add_sat(pk_min(dm1, dp1), P1x2);
        t = pk_min(pk_min(t, Lp[i]), dp);
        uint32_t l = pk_sub(pk_add(c[i], t), dp);
        if constexpr (PAD) l = active ? l : kMaxPair;
        L[i] = l;
        m = pk_min(m, l);
    }
    m16 = (uint32_t)__builtin_elementwise_min((unsigned short)(m & 0xffffu), (unsigned short)(m >> 16));
}

// N row minima (one per slot and direction) folded together, one DPP step across all of them at
// a time (each DPP read then sits N - 1 instructions after the write it reads: no wait states);
// returns dp = min * 0x10001 + P2 (both halves)
template <int N>
__device__ __forceinline__ void row_deltas(uint32_t (&m)[N], uint32_t P2x2) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; i++) m[i] = min_u32_dpp<kDppQuadXor1>(m[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; i++) m[i] = min_u32_dpp<kDppQuadXor2>(m[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; i++) m[i] = min_u32_dpp<kDppRowHalfMirror>(m[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; i++) m[i] = min_u32_dpp<kDppRowMirror>(m[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; i++) m[i] = m[i] * 0x00010001u + P2x2;
}

template <int DW>
__device__ __forceinline__ void load16(Rsrc r, uint32_t vofs, uint32_t (&v)[DW]) {
#pragma unroll
    for (int j = 0; j < DW / 4; j++) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, vofs + 16 * j, 0, 0);
        v[4 * j] = t[0]; v[4 * j + 1] = t[1]; v[4 * j + 2] = t[2]; v[4 * j + 3] = t[3];
    }
}

}  // namespace

// the LDS of a sweep workgroup: every row's lane-row edge states, [parity][uint4 chunk][flat lane]
// (16-B accesses of consecutive lanes are bank-conflict free), and the down pass's WTA rows (one S
// row per lane row of each own wave: the subpixel neighbours and the uniqueness minimum are read
// back from it)
template <int DW, bool UP>
struct SweepLds {
    uint4 xA[2][DW / 4][kSweepWaves * 64];
    uint4 xB[2][DW / 4][kSweepWaves * 64];
    uint32_t xdA[2][kSweepWaves * 64], xdB[2][kSweepWaves * 64];
    uint32_t sS[UP ? 1 : kSweepOwn][4][16 * DW + 4];
    // the down pass's per-pixel epilogue queue: 16 rows of each own wave's pixels (wta_flush)
    uint4 wq[UP ? 1 : kSweepOwn][UP ? 1 : 64 * SwShape<DW, false>::MO];
};

enum { kOwn = 0, kLeftHalo = 1, kRightHalo = 2 };

// One wave's whole sweep (every frame of its slot): ROLE kOwn holds M = MO columns per lane row and
// runs the pass's three directions (and the down pass's WTA); the halo waves hold MH columns and
// run diagonal A (left) or B (right) only.  Each role is its own loop, so the registers a wave
// carries from row to row are its role's, not the union of all three.
template <int DW, bool PAD, bool UP, int ROLE>
__device__ __forceinline__ void sweep_wave(const Geometry& g, const SweepArgs& a, const SweepWta& w, int F,
                                           SweepLds<DW, UP>& sh, int wv, int slot, int tile) {
    constexpr int NWV = kSweepWaves, NO = kSweepOwn;
    constexpr int MO = SwShape<DW, UP>::MO, MH = SwShape<DW, UP>::MH;
    constexpr int NCO = 4 * MO, NCH = 4 * MH;  // columns per own / halo wave
    static_assert(NCH % NCO == 0, "the halo spans whole own waves");
    constexpr int NPUB = NCH / NCO;             // own waves publishing a tile edge
    constexpr int RS = NCH - 1;                 // rows between halo reloads
    constexpr int TILE = NCO * NO;
    constexpr bool OWN = ROLE == kOwn, DA = ROLE != kRightHalo, DB = ROLE != kLeftHalo;
    constexpr int M = OWN ? MO : MH;
    constexpr int NV = DW / 4;                  // uint4 per lane per state
    constexpr int RING = 2;                     // cost (and record) rows in registers
    constexpr bool WTA = OWN && !UP;
    const int lane = threadIdx.x & 63;
    const int r = lane >> 4, gl = lane & 15;
    const int flat = wv * 64 + lane;
    const int W1 = g.W1, H = g.H, D = g.D;
    const int tx0 = tile * TILE;
    const int x0w = ROLE == kLeftHalo ? tx0 - NCH : ROLE == kRightHalo ? tx0 + TILE : tx0 + (wv - 1) * NCO;
    constexpr int ncw = 4 * M;
    const bool has_left = tile > 0, has_right = tile + 1 < a.ntiles;
    // a wave whose columns reach outside [0, W1): those slots hold a fresh state (the value a
    // chain's predecessor outside the image has), which is what their neighbours must read
    const bool edge = x0w < 0 || x0w + ncw > W1;
    const bool idle = x0w + ncw <= 0 || x0w >= W1;  // no column inside the image at all
    const bool active = !PAD || gl * 2 * DW < D;
    const int lg = PAD ? min(gl, D / (2 * DW) - 1) : gl;
    const uint32_t lofs = (uint32_t)(lg * 2 * DW * 2);
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    const uint32_t fresh = active ? 0u : kMaxPair;
    auto col = [&](int m) { return x0w + r * M + m; };
    auto inside = [&](int m) { const int x = col(m); return x >= 0 && x < W1; };
    // ring entries of tile t, side (0: its first NCH columns' diagonal B, 1: its last NCH
    // columns' diagonal A), parity: [NCH columns][DW words][16 lanes], then [NCH][16] deltas
    constexpr int EW = NCH * 16 * (DW + 1);
    auto entry = [&](int t, int side, int par) {
        return a.edge + ((((size_t)slot * a.ntiles + t) * 2 + side) * 2 + par) * EW;
    };
    auto flag = [&](int t, int side, int p) { return a.flags + (((size_t)slot * a.ntiles + t) * 2 + side) * NPUB + p; };
    // publishing waves: the first NPUB own waves (side 0), the last NPUB (side 1)
    const int pub0 = OWN && wv - 1 < NPUB ? wv - 1 : -1;
    const int pub1 = OWN && wv >= NO - NPUB + 1 ? wv - (NO - NPUB + 1) : -1;
    bool gave_up = false;
    auto wait = [&](const int* fl, int target) __attribute__((always_inline)) {
        int n = 0;
        while (!gave_up &&
               __builtin_amdgcn_readfirstlane(__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
                   target) {
            if (++n > a.spin) {
                if (lane == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gave_up = true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the ring loads stay after the poll
    };

    for (int f = slot, it = 0; f < F; f += a.nslots, it++) {
        const int base = it * H;  // rows of this slot's earlier frames (the counters run on)
        const char* cframe = (const char*)(a.C + (size_t)f * a.cs_fstride);
        const size_t crow = (size_t)W1 * D * 2, rrow = (size_t)W1 * a.l_pix * 2;
        auto yof = [&](int k) { return UP ? H - 1 - k : k; };
        // per-slot lane offsets into a cost row / a record row (columns clamped into the image)
        uint32_t cofs[M];
#pragma unroll
        for (int m = 0; m < M; m++)
            cofs[m] = (uint32_t)min(max(col(m), 0), W1 - 1) * (uint32_t)(D * 2) + lofs;
        uint32_t Lv[OWN ? M : 1][DW], La[DA ? M : 1][DW], Lb[DB ? M : 1][DW];
        uint32_t dv[OWN ? M : 1], da[DA ? M : 1], db[DB ? M : 1];
#pragma unroll
        for (int m = 0; m < M; m++) {
#pragma unroll
            for (int i = 0; i < DW; i++) {
                if constexpr (OWN) Lv[m][i] = fresh;
                if constexpr (DA) La[m][i] = fresh;
                if constexpr (DB) Lb[m][i] = fresh;
            }
            if constexpr (OWN) dv[m] = P2x2;
            if constexpr (DA) da[m] = P2x2;
            if constexpr (DB) db[m] = P2x2;
        }
        // this tile's edge columns after row count-1 -> the ring, then the wave's counter (the
        // counter store waits for the data stores); data = false: the counter only
        auto publish = [&](int count, bool data) __attribute__((always_inline)) {
            if constexpr (OWN) {
                if (pub0 < 0 && pub1 < 0) return;
                const int side = pub0 >= 0 ? 0 : 1, p = pub0 >= 0 ? pub0 : pub1;
                if (data) {
                    // word i of the 16 lanes of a column are 64 contiguous bytes ([column][word]
                    // [lane]): each agent-scope store below (sc1: written through this XCD's L2)
                    // fills whole 64-byte segments.  With a lane's words contiguous ([column][lane]
                    // [word]) each 4-byte store cost a 32-byte memory write: 6 GB of a C3 batch's
                    // down pass, 3 GB of its up pass
                    // (the side is a constant in each branch: a runtime select between La and Lb
                    // became a select of their addresses, which put both arrays in scratch)
                    uint32_t* e = entry(tile, side, (count / RS) & 1);
                    auto put = [&](const uint32_t(&L)[M][DW], const uint32_t(&dl)[M]) __attribute__((always_inline)) {
#pragma unroll
                        for (int m = 0; m < MO; m++) {
                            const int c = p * NCO + r * MO + m;  // column within the edge group
#pragma unroll
                            for (int i = 0; i < DW; i++)
                                __hip_atomic_store(e + (c * DW + i) * 16 + gl, L[m][i], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(e + NCH * 16 * DW + c * 16 + gl, dl[m], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        }
                    };
                    if (side) put(La, da);
                    else put(Lb, db);
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no compiler motion across the wait
                __builtin_amdgcn_s_waitcnt(0);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if (lane == 0) __hip_atomic_store(flag(tile, side, p), count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        // a halo wave's state: the neighbour's edge columns after row count-1.  The halo's own
        // lane-row boundaries went through LDS at the row before, from the drifted pre-reload
        // state, so the predecessor of each lane row's boundary slot (diagonal A: the column left
        // of its first slot; B: right of its last) comes from the ring too, for this one row
        uint32_t rin[OWN ? 1 : DW], rdin = 0;
        bool reloaded = false;
        auto reload = [&](int count) __attribute__((always_inline)) {
            if constexpr (!OWN) {
                constexpr int side = ROLE == kLeftHalo ? 1 : 0;
                if (ROLE == kLeftHalo ? !has_left : !has_right) return;
                const int nt = ROLE == kLeftHalo ? tile - 1 : tile + 1;
#pragma unroll
                for (int p = 0; p < NPUB; p++) wait(flag(nt, side, p), count);
                const uint32_t* e = entry(nt, side, (count / RS) & 1);
                {
                    // the boundary predecessor: column r * MH - 1 (A) or r * MH + MH (B), inside the
                    // group for all but the group's outer lane row (whose value is never exact)
                    const int cb = ROLE == kLeftHalo ? max(r * MH - 1, 0) : min(r * MH + MH, NCH - 1);
#pragma unroll
                    for (int i = 0; i < DW; i++)
                        rin[i] = __hip_atomic_load(e + (cb * DW + i) * 16 + gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    rdin = __hip_atomic_load(e + NCH * 16 * DW + cb * 16 + gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    reloaded = true;
                }
#pragma unroll
                for (int m = 0; m < MH; m++) {
                    const int c = r * MH + m;
                    uint32_t v[DW];
#pragma unroll
                    for (int i = 0; i < DW; i++)
                        v[i] = __hip_atomic_load(e + (c * DW + i) * 16 + gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t dd =
                        __hip_atomic_load(e + NCH * 16 * DW + c * 16 + gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                    for (int i = 0; i < DW; i++) {
                        if constexpr (ROLE == kLeftHalo) La[m][i] = v[i];
                        else Lb[m][i] = v[i];
                    }
                    if constexpr (ROLE == kLeftHalo) da[m] = dd;
                    else db[m] = dd;
                }
            }
        };

        uint32_t cr[RING][M][DW];
        auto load_row = [&](int k, uint32_t (&dst)[M][DW]) __attribute__((always_inline)) {
            const Rsrc rs = rsrc_at(cframe + (size_t)yof(min(k, H - 1)) * crow);  // past the end: the last row again
#pragma unroll
            for (int m = 0; m < M; m++) load16<DW>(rs, cofs[m], dst[m]);
        };
        // the down pass's E, W and up records of a row (own waves)
        constexpr int ER = WTA ? RING : 1, EM = WTA ? MO : 1;
        uint32_t er[ER][EM][3][DW];
        auto load_rec = [&](int k, uint32_t (&dst)[EM][3][DW]) __attribute__((always_inline)) {
            if constexpr (WTA) {
                const Rsrc rs = rsrc_at((const char*)(w.recs + (size_t)f * a.l_fstride) + (size_t)yof(min(k, H - 1)) * rrow);
#pragma unroll
                for (int m = 0; m < MO; m++) {
                    const uint32_t ro = (uint32_t)min(max(col(m), 0), W1 - 1) * (uint32_t)(a.l_pix * 2) + lofs;
#pragma unroll
                    for (int q = 0; q < 3; q++) load16<DW>(rs, ro + (uint32_t)(q * D * 2), dst[m][q]);
                }
            }
        };
        if (!idle) {
            load_row(0, cr[0]);
            load_rec(0, er[0]);
        }
        // a new frame: the neighbours must be done reading this tile's ring entries of the last one
        if (it > 0) {
            if (ROLE == kLeftHalo && has_left)
                for (int p = 0; p < NPUB; p++) wait(flag(tile - 1, 1, p), base);
            if (ROLE == kRightHalo && has_right)
                for (int p = 0; p < NPUB; p++) wait(flag(tile + 1, 0, p), base);
        }
        // records of the own columns inside the image: stores of other columns and of padding
        // lanes fall outside the resource and are dropped
        const int nin = max(0, min(W1, x0w + ncw) - max(x0w, 0));

        // A.8's per-pixel epilogue (uniqueness, subpixel, the WTA disparity and the right view's
        // key) for the queued pixels of rows (k & ~15) .. k, a pixel a lane: done in each row, a
        // lane row's one pixel kept 60 of the wave's 64 lanes idle through ~45 instructions
        auto wta_flush = [&](int k) __attribute__((always_inline)) {
            if constexpr (WTA) {
                const int kb = k & ~15, nrow = k - kb + 1;
                const int invalid = (g.minD - 1) * 16;
                const bool check_uniq = w.uniq > 0 || !w.uniq_simd;
                // SIMD rule: S[d] < (short)(thresh + 1), thresh = (100*minS)/(100-u); scalar: S*(100-u) < 100*minS
                const double inv100u = 1.0 / (double)(100 - w.uniq) * (1.0 + 0x1p-40);
#pragma unroll
                for (int q = 0; q < MO; q++) {
                    const int e = q * 64 + lane;
                    const int m = e % MO, rq = (e / MO) & 3, kk = e / (4 * MO);
                    const int x = x0w + rq * MO + m;
                    if (kk < nrow && x >= 0 && x < W1) {
                        const uint4 v = sh.wq[wv - 1][e];
                        const int minS = (int)(v.x >> 16), best = (int)(v.x & 0xffffu);
                        const int Sm = (int)(int16_t)(v.y >> 16), Sp = (int)(int16_t)(v.y & 0xffffu);
                        const int min2 = (int)v.z;
                        const int y = yof(kb + kk);
                        const int thr16 = (int)(short)((int)((double)(100 * minS) * inv100u) + 1);
                        const bool reject =
                            check_uniq && (w.uniq_simd ? (min2 < thr16) : (min2 * (100 - w.uniq) < minS * 100));
                        int out = invalid;
                        // every S saturated: OpenCV's first-minimum scan keeps bestDisp = -1 (INVALID)
                        if (!reject && minS < kMaxCost) {
                            const int den = max(Sm + Sp - 2 * minS, 1);
                            const int qq = div_trunc_small((Sm - Sp) * 16 + den, 2 * den);
                            out = best * 16 + (((0 < best) & (best < D - 1)) ? qq : 0) + g.minD * 16;
                            if (w.d2) {
                                const int x2 = x + g.minX1 - g.minD - best;
                                if (x2 >= 0 && x2 < g.W)
                                    atomicMin(&w.d2[(size_t)f * w.disp_fstride + (size_t)y * g.W + x2],
                                              ((uint32_t)minS << 16) | (uint32_t)(0xffff - x));
                            }
                        }
                        w.disp_raw[(size_t)f * w.disp_fstride + (size_t)y * g.W + x + g.minX1] = (int16_t)out;
                    }
                }
            }
        };
        auto row = [&](const int k, auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            if (k > 0 && k % RS == 0) {
                publish(base + k, true);
                reload(base + k);
            }
            if (!idle) {
                load_row(k + 1, cr[(s + 1) % RING]);
                load_rec(k + 1, er[(s + 1) % ER]);
            }
            const uint32_t(&c)[M][DW] = cr[s];
            const int pr = (k + 1) & 1;  // parity of row k-1's edge states
            if (!idle) {
                uint32_t m16[(OWN ? 3 : 1) * M];
                if constexpr (OWN) {
                    // vertical: the same column, the row before
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        uint32_t L[DW];
                        step16<DW, PAD>(c[m], Lv[m], dv[m], P1x2, active, L, m16[m]);
#pragma unroll
                        for (int i = 0; i < DW; i++) Lv[m][i] = L[i];
                    }
                }
                if constexpr (DA) {
                    // diagonal A (predecessor x - 1), slots descending: La[m-1] is still the row
                    // before's; the lane row's first slot takes the previous lane row's (or wave's)
                    // last slot from LDS
                    constexpr int o = OWN ? M : 0;
#pragma unroll
                    for (int m = M - 1; m >= 0; m--) {
                        uint32_t L[DW];
                        if (m > 0) {
                            step16<DW, PAD>(c[m], La[m > 0 ? m - 1 : 0], da[m > 0 ? m - 1 : 0], P1x2, active, L, m16[o + m]);
                        } else {
                            uint32_t in[DW], din = P2x2;
#pragma unroll
                            for (int i = 0; i < DW; i++) in[i] = fresh;
                            if (k > 0 && flat >= 16) {
#pragma unroll
                                for (int j = 0; j < NV; j++) {
                                    const uint4 v = sh.xA[pr][j][flat - 16];
                                    in[4 * j] = v.x; in[4 * j + 1] = v.y; in[4 * j + 2] = v.z; in[4 * j + 3] = v.w;
                                }
                                din = sh.xdA[pr][flat - 16];
                            }
                            if constexpr (!OWN) {
                                if (reloaded) {
#pragma unroll
                                    for (int i = 0; i < DW; i++) in[i] = rin[i];
                                    din = rdin;
                                }
                            }
                            step16<DW, PAD>(c[m], in, din, P1x2, active, L, m16[o + m]);
                        }
#pragma unroll
                        for (int i = 0; i < DW; i++) La[m][i] = L[i];
                    }
                }
                if constexpr (DB) {
                    // diagonal B (predecessor x + 1), slots ascending
                    constexpr int o = OWN ? 2 * M : 0;
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        uint32_t L[DW];
                        if (m < M - 1) {
                            step16<DW, PAD>(c[m], Lb[m < M - 1 ? m + 1 : 0], db[m < M - 1 ? m + 1 : 0], P1x2, active, L, m16[o + m]);
                        } else {
                            uint32_t in[DW], din = P2x2;
#pragma unroll
                            for (int i = 0; i < DW; i++) in[i] = fresh;
                            if (k > 0 && flat + 16 < NWV * 64) {
#pragma unroll
                                for (int j = 0; j < NV; j++) {
                                    const uint4 v = sh.xB[pr][j][flat + 16];
                                    in[4 * j] = v.x; in[4 * j + 1] = v.y; in[4 * j + 2] = v.z; in[4 * j + 3] = v.w;
                                }
                                din = sh.xdB[pr][flat + 16];
                            }
                            if constexpr (!OWN) {
                                if (reloaded) {
#pragma unroll
                                    for (int i = 0; i < DW; i++) in[i] = rin[i];
                                    din = rdin;
                                }
                            }
                            step16<DW, PAD>(c[m], in, din, P1x2, active, L, m16[o + m]);
                        }
#pragma unroll
                        for (int i = 0; i < DW; i++) Lb[m][i] = L[i];
                    }
                }
                row_deltas<(OWN ? 3 : 1) * M>(m16, P2x2);
#pragma unroll
                for (int m = 0; m < M; m++) {
                    if constexpr (OWN) dv[m] = m16[m];
                    if constexpr (DA) da[m] = m16[(OWN ? M : 0) + m];
                    if constexpr (DB) db[m] = m16[(OWN ? 2 * M : 0) + m];
                }
                if (edge) {
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        const bool in = inside(m);
#pragma unroll
                        for (int i = 0; i < DW; i++) {
                            if constexpr (OWN) Lv[m][i] = in ? Lv[m][i] : fresh;
                            if constexpr (DA) La[m][i] = in ? La[m][i] : fresh;
                            if constexpr (DB) Lb[m][i] = in ? Lb[m][i] : fresh;
                        }
                        if constexpr (OWN) dv[m] = in ? dv[m] : P2x2;
                        if constexpr (DA) da[m] = in ? da[m] : P2x2;
                        if constexpr (DB) db[m] = in ? db[m] : P2x2;
                    }
                }
            }
            if constexpr (!OWN) reloaded = false;
            // this row's lane-row edge states for the neighbouring lane rows (diagonal A's last
            // slot, B's first; a role without the diagonal or an idle wave: fresh)
#pragma unroll
            for (int j = 0; j < NV; j++) {
                uint4 va = make_uint4(fresh, fresh, fresh, fresh), vb = va;
                if constexpr (DA) va = make_uint4(La[M - 1][4 * j], La[M - 1][4 * j + 1], La[M - 1][4 * j + 2], La[M - 1][4 * j + 3]);
                if constexpr (DB) vb = make_uint4(Lb[0][4 * j], Lb[0][4 * j + 1], Lb[0][4 * j + 2], Lb[0][4 * j + 3]);
                sh.xA[k & 1][j][flat] = va;
                sh.xB[k & 1][j][flat] = vb;
            }
            if constexpr (DA) sh.xdA[k & 1][flat] = da[M - 1];
            else sh.xdA[k & 1][flat] = P2x2;
            if constexpr (DB) sh.xdB[k & 1][flat] = db[0];
            else sh.xdB[k & 1][flat] = P2x2;
            if constexpr (OWN && UP) {
                if (!idle) {
                    // the pass's record: sat(N + NE + NW)
                    const Rsrc rr = __builtin_amdgcn_make_buffer_rsrc(
                        (char*)(a.rec + (size_t)f * a.l_fstride) + (size_t)yof(k) * rrow + (size_t)max(x0w, 0) * a.l_pix * 2,
                        (short)0, (int)(nin > 0 ? (nin - 1) * a.l_pix * 2 + D * 2 : 0), 0x00020000);
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        Regs<DW> sum;
#pragma unroll
                        for (int i = 0; i < DW; i++) sum.r[i] = pk_add_sat(pk_add_sat(Lv[m][i], La[m][i]), Lb[m][i]);
                        const int xr = col(m) - max(x0w, 0);
                        const uint32_t so = active && inside(m) ? (uint32_t)xr * (uint32_t)(a.l_pix * 2) + lofs : 0x7fffffffu;
                        store_buf_nt<DW>(rr, so, 0, sum);
                    }
                }
            }
            if constexpr (WTA) {
                if (!idle) {
                    // A.8 on S = sat(E + W + up + S + SE + SW) of each own slot
                    const uint32_t(&e)[EM][3][DW] = er[s % ER];
#pragma unroll
                    for (int m = 0; m < M; m++) {
                        uint32_t St[DW];
#pragma unroll
                        for (int i = 0; i < DW; i++) {
                            uint32_t acc = pk_add_sat(pk_add_sat(e[m][0][i], e[m][1][i]), e[m][2][i]);
                            acc = pk_add_sat(pk_add_sat(pk_add_sat(acc, Lv[m][i]), La[m][i]), Lb[m][i]);
                            St[i] = PAD ? (active ? acc : kMaxPair) : acc;
                        }
                        // first minimum: (S << 16 | d) keys (S >= 0: a sum of non-negative path costs)
                        const uint32_t d0 = (uint32_t)(gl * 2 * DW);
                        uint32_t key = 0xffffffffu;
#pragma unroll
                        for (int i = 0; i < DW; i++) {
                            const uint32_t klo = (St[i] << 16) | (d0 + 2 * i);
                            const uint32_t khi = (St[i] & 0xffff0000u) | (d0 + 2 * i + 1);
                            key = min(key, min(klo, khi));
                        }
                        key = row16_min_u32(active ? key : 0xffffffffu);
                        const int minS = (int)(key >> 16);
                        const int best = (int)(key & 0xffff);
                        const int dm = max(best - 1, 0), dp = min(best + 1, D - 1);
                        typedef int16_t __attribute__((may_alias)) s16a;
                        typedef uint32_t __attribute__((may_alias)) u32a;
                        u32a* srow = (u32a*)&sh.sS[UP ? 0 : wv - 1][r][0];
#pragma unroll
                        for (int i = 0; i < DW; i++) srow[gl * DW + i] = St[i];
                        s16a* s16 = (s16a*)srow;
                        const int Sm = s16[dm];
                        const int Sp = s16[dp];
                        s16[dm] = 0x7fff;
                        s16[best] = 0x7fff;
                        s16[dp] = 0x7fff;
                        // uniqueness: min of S[d] over |d - best| > 1 (0 <= S <= 32767: 0x7fff masks a half)
                        uint32_t m2 = kMaxPair;
#pragma unroll
                        for (int i = 0; i < DW; i++) m2 = pk_min(m2, srow[gl * DW + i]);
                        m2 = active ? m2 : kMaxPair;
                        m2 = pk_min(m2, funnel16(m2, m2));
                        m2 = row16_min_u32(m2);
                        const int min2 = (int)(m2 & 0x7fff);
                        // the pixel's epilogue waits in the queue (wta_flush)
                        if (gl == 0)
                            sh.wq[wv - 1][((k & 15) * 4 + r) * MO + m] =
                                make_uint4(((uint32_t)minS << 16) | (uint32_t)best,
                                           ((uint32_t)(uint16_t)Sm << 16) | (uint32_t)(uint16_t)Sp, (uint32_t)min2, 0u);
                    }
                    if ((k & 15) == 15 || k == H - 1) wta_flush(k);
                }
            }
            __syncthreads();
        };
        int k0 = 0;
        for (; k0 + RING <= H; k0 += RING) unroll_rows(row, k0, std::make_integer_sequence<int, RING>{});
        unroll_rows_tail(row, k0, H - 1, std::make_integer_sequence<int, RING - 1>{});
        publish(base + H, false);  // the frame is done: the neighbours may start the next one
    }
}

template <int DW, bool PAD, bool UP>
__global__ __launch_bounds__(64 * kSweepWaves) void k_sweep16(Geometry g, SweepArgs a, SweepWta w, int F) {
    __shared__ SweepLds<DW, UP> sh;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // blocks b and b + 8 share an XCD (its L2): two neighbouring tiles there read the C columns of
    // each other's halo from the L2 the other filled.  For speed only: the ring protocol assumes
    // no placement.  The grid is a multiple of 2 * kSweepXcds; the padding blocks exit at once.
    const int b = (int)blockIdx.x;
    // 1: tile t at blocks b, b + 8, ... of one XCD; 2: tiles 2j and 2j + 1 on one XCD (blocks b and
    // b + 8), the pairs dealt round-robin (the grid is a multiple of 2 * kSweepXcds); 0: linear
    const int lid = a.xcd == 1   ? (b % kSweepXcds) * (int)(gridDim.x / kSweepXcds) + b / kSweepXcds
                    : a.xcd == 2 ? ((b / (2 * kSweepXcds)) * kSweepXcds + b % kSweepXcds) * 2 + (b / kSweepXcds) % 2
                                 : b;
    if (lid >= a.nslots * a.ntiles) return;
    const int slot = lid / a.ntiles, tile = lid - slot * a.ntiles;
    if (wv == 0) sweep_wave<DW, PAD, UP, kLeftHalo>(g, a, w, F, sh, wv, slot, tile);
    else if (wv == kSweepWaves - 1) sweep_wave<DW, PAD, UP, kRightHalo>(g, a, w, F, sh, wv, slot, tile);
    else sweep_wave<DW, PAD, UP, kOwn>(g, a, w, F, sh, wv, slot, tile);
}

template <int DW, bool PAD, bool UP>
static int sweep16_occupancy() {
    static int per_cu = -1;
    if (__atomic_load_n(&per_cu, __ATOMIC_RELAXED) < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)k_sweep16<DW, PAD, UP>, 64 * kSweepWaves, 0) !=
            hipSuccess)
            n = 0;
        __atomic_store_n(&per_cu, n, __ATOMIC_RELAXED);
    }
    return per_cu;
}

SweepShape sweep_shape(const Geometry& g, int F, bool up) {
    SweepShape sh{0, 0, 0, 0, 0};
    if (g.W1 <= 0 || F <= 0 || g.D > 256) return sh;  // 16 disparities per lane at most
    const int cus = device_cus();
    const int dw = g.D <= 128 ? 4 : 8;
    int occ, mo, mh;
    if (dw == 4) {
        occ = up ? (g.D < 128 ? sweep16_occupancy<4, true, true>() : sweep16_occupancy<4, false, true>())
                 : (g.D < 128 ? sweep16_occupancy<4, true, false>() : sweep16_occupancy<4, false, false>());
        mo = up ? SwShape<4, true>::MO : SwShape<4, false>::MO;
        mh = up ? SwShape<4, true>::MH : SwShape<4, false>::MH;
    } else {
        occ = up ? (g.D < 256 ? sweep16_occupancy<8, true, true>() : sweep16_occupancy<8, false, true>())
                 : (g.D < 256 ? sweep16_occupancy<8, true, false>() : sweep16_occupancy<8, false, false>());
        mo = up ? SwShape<8, true>::MO : SwShape<8, false>::MO;
        mh = up ? SwShape<8, true>::MH : SwShape<8, false>::MH;
    }
    const int tile = 4 * mo * kSweepOwn;
    sh.cols = 4 * mo;
    sh.ntiles = (g.W1 + tile - 1) / tile;
    sh.nslots = std::min(F, cus * occ / sh.ntiles);
    sh.npub = mh / mo;
    sh.entry_words = 4 * mh * 16 * (dw + 1);
    return sh;
}

void launch_sweep(const Geometry& g, const SweepArgs& a0, const SweepWta& w, int F, hipStream_t st) {
    // tile -> XCD (profiles/r6_sweep_xcd_ab.txt, one box each; C3 PMC a 32-frame batch, algorithmic
    // down 48.3 GB, up 24.2): linear (0) 55.3 / 27.6 GB, down 10.65 ms, up 5.66; a frame's tiles on
    // one XCD (1) 50.9 / 25.9 GB but down 11.67, up 6.55 ms -- its tiles walk the rows in lockstep,
    // so one XCD's demand comes in bursts where the other orders mix frames at different rows;
    // pairs of tiles on one XCD (2, the default) 52.9 / 26.5 GB (1.10x) at the linear order's times
    static const int xcd = getenv("SDR_SWEEP_XCD") ? atoi(getenv("SDR_SWEEP_XCD")) : 2;
    SweepArgs a = a0;
    a.xcd = xcd;
    const dim3 grid((a.nslots * a.ntiles + 2 * kSweepXcds - 1) / (2 * kSweepXcds) * (2 * kSweepXcds)), block(64 * kSweepWaves);
#define SDR_SWEEP(DW, PAD)                                                                          \
    if (a.up) hipLaunchKernelGGL((k_sweep16<DW, PAD, true>), grid, block, 0, st, g, a, w, F);       \
    else hipLaunchKernelGGL((k_sweep16<DW, PAD, false>), grid, block, 0, st, g, a, w, F);
    if (g.D <= 128) {
        if (g.D < 128) { SDR_SWEEP(4, true) } else { SDR_SWEEP(4, false) }
    } else {
        if (g.D < 256) { SDR_SWEEP(8, true) } else { SDR_SWEEP(8, false) }
    }
#undef SDR_SWEEP
}

__global__ __launch_bounds__(256) void k_sweep_verdict(const int* __restrict__ err, int16_t* __restrict__ disp,
                                                       size_t n, int F, int16_t invalid, int* __restrict__ mins,
                                                       int* __restrict__ sticky) {
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0)
        return;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < n * F; i += nth) disp[i] = invalid;
    if (mins)
        for (size_t i = tid; i < (size_t)F * kMinSlots; i += nth) mins[i] = invalid;
    if (tid == 0) atomicAdd(sticky, 1);  // counts timed-out batches: the host reports each once
}

void launch_sweep_verdict(const int* err, int16_t* disp, size_t n, int F, int16_t invalid, int* mins,
                          int* sticky, hipStream_t st) {
    hipLaunchKernelGGL(k_sweep_verdict, dim3(1024), dim3(256), 0, st, err, disp, n, F, invalid, mins, sticky);
}

}  // namespace sdr
