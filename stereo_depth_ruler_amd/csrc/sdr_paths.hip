// sdr_paths.hip -- A.4-A.9: path aggregation and winner-take-all/LR kernels (CDNA4).
//
// k_paths: every scanline chain of every direction of the mode in ONE launch (a direction table
// in the kernel arguments).  One wave64 = one chain; lane l holds disparities [l*DPL, l*DPL+DPL)
// as DPL/2 packed int16 pairs.  Per step
//     L = C + min(Lp, min(Lp[d-1], Lp[d+1]) + P1, minLp + P2) - (minLp + P2)
// and L is written to the direction's own buffer (every direction but top-to-bottom).  The
// latency-bound chains (E/W: H chains of W1 steps at batch 1) overlap with the bandwidth-bound
// ones instead of running alone.  C loads are software-pipelined LA steps ahead through one
// buffer resource per chain and an SGPR offset; they run into slack rows past the chain's ends
// instead of being clamped.  The per-step minimum is a wave-uniform (SGPR) value.
//
// k_south_wta: the top-to-bottom chains fused with the winner-take-all (S = sat(sum_r L_r),
// first minimum, uniqueness, subpixel, disp2 scatter) as a producer/consumer workgroup;
// k_lr_check then applies the left-right check per pixel.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <algorithm>

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

// Buffer-resource access: the row base lives in a wave-uniform resource descriptor (SGPRs, scalar
// arithmetic), the lane's byte offset in one VGPR, so a load or store costs no vector address math.
#ifndef SDR_PATHS_BUF
#define SDR_PATHS_BUF 1  // k_paths through buffer resources (0: flat global addresses)
#endif
#ifndef SDR_PATHS_KEEPFILL
#define SDR_PATHS_KEEPFILL 1  // boundary lanes of the neighbour shifts kept across steps (0: refilled)
#endif
#ifndef SDR_WMIN_BCAST
#define SDR_WMIN_BCAST 1  // path minimum via DPP row broadcasts + readlane (0: permlane swaps)
#endif
#ifndef SDR_PATHS_SOFF
#define SDR_PATHS_SOFF 1  // k_paths: per-chain resources + SGPR offsets (0: a resource per access)
#endif
#ifndef SDR_SOUTH_BUF
#define SDR_SOUTH_BUF 1  // k_south_wta through buffer resources (0: flat global addresses)
#endif
using Rsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ Rsrc rsrc_at(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}

template <int K>
__device__ __forceinline__ Regs<K> load_buf(Rsrc r, uint32_t vofs) {
    Regs<K> v;
    if constexpr (K == 1) {
        v.r[0] = __builtin_amdgcn_raw_buffer_load_b32(r, vofs, 0, 0);
    } else if constexpr (K == 2) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, vofs, 0, 0);
        v.r[0] = t[0];
        v.r[1] = t[1];
    } else {
        static_assert(K % 4 == 0, "K = 1, 2 or a multiple of 4");
#pragma unroll
        for (int j = 0; j < K / 4; j++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, vofs + 16 * j, 0, 0);
            v.r[4 * j] = t[0]; v.r[4 * j + 1] = t[1]; v.r[4 * j + 2] = t[2]; v.r[4 * j + 3] = t[3];
        }
    }
    return v;
}

// The same with a wave-uniform (SGPR) byte offset: one resource per buffer for a whole chain,
// and one scalar add per step moves every access of the step.
template <int K>
__device__ __forceinline__ Regs<K> load_buf_so(Rsrc r, uint32_t vofs, uint32_t sofs) {
    Regs<K> v;
    if constexpr (K == 1) {
        v.r[0] = __builtin_amdgcn_raw_buffer_load_b32(r, vofs, sofs, 0);
    } else if constexpr (K == 2) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, vofs, sofs, 0);
        v.r[0] = t[0];
        v.r[1] = t[1];
    } else {
        static_assert(K % 4 == 0, "K = 1, 2 or a multiple of 4");
#pragma unroll
        for (int j = 0; j < K / 4; j++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, vofs + 16 * j, sofs, 0);
            v.r[4 * j] = t[0]; v.r[4 * j + 1] = t[1]; v.r[4 * j + 2] = t[2]; v.r[4 * j + 3] = t[3];
        }
    }
    return v;
}
template <int K>
__device__ __forceinline__ void store_buf_nt_so(Rsrc r, uint32_t vofs, uint32_t sofs, const Regs<K>& v) {
    if constexpr (K == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v.r[0], r, vofs, sofs, 2);
    } else if constexpr (K == 2) {
        __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) uint32_t){v.r[0], v.r[1]}, r,
                                              vofs, sofs, 2);
    } else {
#pragma unroll
        for (int j = 0; j < K / 4; j++)
            __builtin_amdgcn_raw_buffer_store_b128(
                (__attribute__((ext_vector_type(4))) uint32_t){v.r[4 * j], v.r[4 * j + 1], v.r[4 * j + 2],
                                                               v.r[4 * j + 3]},
                r, vofs + 16 * j, sofs, 2);
    }
}

// non-temporal (aux = nt) stores of K packed pairs
template <int K>
__device__ __forceinline__ void store_buf_nt(Rsrc r, uint32_t vofs, const Regs<K>& v) {
    if constexpr (K == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v.r[0], r, vofs, 0, 2);
    } else if constexpr (K == 2) {
        __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) uint32_t){v.r[0], v.r[1]}, r,
                                              vofs, 0, 2);
    } else {
#pragma unroll
        for (int j = 0; j < K / 4; j++)
            __builtin_amdgcn_raw_buffer_store_b128(
                (__attribute__((ext_vector_type(4))) uint32_t){v.r[4 * j], v.r[4 * j + 1], v.r[4 * j + 2],
                                                               v.r[4 * j + 3]},
                r, vofs + 16 * j, 0, 2);
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

#ifndef SDR_PATHS_VF
// offset-carrying recurrence (1) or the normalised form (0).  Both are bit-exact on MI355X; the
// shorter serial chain did not pay, twice: C2 single-stream k_paths 322 vs 304-315 us before the
// scalar-minimum rework, 280-282 vs 273-285 us after it, k_south_wta 241-242 us either way (its
// producer's step time is not set by this dependency chain either).
#define SDR_PATHS_VF 0
#endif
// Initial recurrence state before a chain's first pixel (Lp = 0 there, OpenCV's zeroed row).
__device__ __forceinline__ uint32_t path_delta0(uint32_t P2x2) { return SDR_PATHS_VF ? 0u : P2x2; }

// One step of the path recurrence on a wave's packed int16 pairs (lane l: disparities
// [l*2K, l*2K + 2K)); returns L of this pixel.
//
// SDR_PATHS_VF=1 carries V(k) = L(k) + delta(k) instead of L(k) (delta(k) = min_d L(k-1) + P2):
//   V(k+1) = C - delta(k) + min(min(V[d], V[d-1] + P1, V[d+1] + P1), M(k) + P2),
//   delta(k+1) = M(k) - delta(k) + P2,  M(k) = min_d V(k),  L(k) = V(k) - delta(k),
// which is the same integer arithmetic (0 <= L <= V <= 2 Cmax + P2, the range the normalised form
// already needs for C + min(...)), but the wave-wide minimum of a step is taken over the state it
// starts from, so it runs beside the neighbour terms instead of after them: the serial chain from
// one pixel to the next is the reduction plus three ops.  State: Lp = V, delta2 = delta.
// SDR_PATHS_VF=0: Lp := L, delta2 := minL + P2 (both halves).
// upr/dnr: the lane-shifted neighbour words of the previous step.  A wave shift leaves the lane
// without a source (lane 0 / lane 63) unwritten, so passing the previous shift as the DPP's old
// value keeps the kMaxPair boundary there from the first step on, with no refill per step.
template <int K, bool PAD>
__device__ __forceinline__ Regs<K> path_step(Regs<K> c, Regs<K>& Lp, uint32_t& delta2, uint32_t P1x2,
                                             uint32_t P2x2, bool active, uint32_t& upr, uint32_t& dnr) {
    if constexpr (SDR_PATHS_VF) {
        uint32_t m = Lp.r[0];
#pragma unroll
        for (int i = 1; i < K; i++) m = pk_min(m, Lp.r[i]);
        const uint32_t m16 = (uint32_t)__builtin_elementwise_min((unsigned short)(m & 0xffffu),
                                                                  (unsigned short)(m >> 16));
        // M(k) + P2 and delta(k+1) as wave-uniform packed words (equal halves, no carry/borrow
        // crosses them: 0 < delta(k+1) = M(k) + P2 - delta(k) < 0x8000)
        const uint32_t mP2 = wave_min_u32_uniform(m16) * 0x00010001u + P2x2;
        const uint32_t dnew = mP2 - delta2;
        const uint32_t up = upr = lane_from_prev(Lp.r[K - 1], upr);
        const uint32_t dn = dnr = lane_from_next(Lp.r[0], dnr);
        Regs<K> V, L;
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint32_t dm1 = funnel16(Lp.r[i], i == 0 ? up : Lp.r[i == 0 ? 0 : i - 1]);
            const uint32_t dp1 = funnel16(i == K - 1 ? dn : Lp.r[i == K - 1 ? 0 : i + 1], Lp.r[i]);
            const uint32_t t = pk_min(pk_add_sat(pk_min(dm1, dp1), P1x2), Lp.r[i]);
            uint32_t v = pk_add(pk_min(t, mP2), pk_sub(c.r[i], delta2));
            uint32_t l = pk_sub(v, dnew);
            if constexpr (PAD) {
                v = active ? v : kMaxPair;
                l = active ? l : kMaxPair;
            }
            V.r[i] = v;
            L.r[i] = l;
        }
        Lp = V;
        delta2 = dnew;
        return L;
    }
    if constexpr (PAD) {
#pragma unroll
        for (int i = 0; i < K; i++) c.r[i] = active ? c.r[i] : kMaxPair;
    }
    uint32_t up, dn;
    if constexpr (SDR_PATHS_KEEPFILL) {
        up = upr = lane_from_prev(Lp.r[K - 1], upr);
        dn = dnr = lane_from_next(Lp.r[0], dnr);
    } else {
        up = lane_from_prev(Lp.r[K - 1], kMaxPair);
        dn = lane_from_next(Lp.r[0], kMaxPair);
    }
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
    if constexpr (SDR_WMIN_BCAST) {
        // min of the pair into the low half (one SDWA op; L >= 0, so u16 order is int16 order),
        // wave minimum as a wave-uniform value, splatted and offset by P2 in scalar registers
        const uint32_t m16 = (uint32_t)__builtin_elementwise_min((unsigned short)(m & 0xffffu),
                                                                  (unsigned short)(m >> 16));
        delta2 = wave_min_u32_uniform(m16) * 0x00010001u + P2x2;
    } else {
        // both halves := min of the pair; L >= 0, so the u32 order of such words is the int16 order
        m = pk_min(m, funnel16(m, m));
        m = wave_min_u32(m);
        delta2 = pk_add(m, P2x2);
    }
    Lp = L;
    return L;
}

#ifndef SDR_PATHS_LA
#define SDR_PATHS_LA 16  // k_paths lookahead (steps)
#endif
template <int DPL, bool PAD, bool NT = false>
__global__ __launch_bounds__(256) void k_paths(Geometry g, PathLaunch pl) {
    constexpr int K = DPL / 2;
    // C is loaded LA steps ahead into a ring of 2*LA slots: the slot a load fills was consumed
    // LA steps earlier, so every slot keeps one register across the loop's back edge (a ring
    // of LA slots makes the compiler copy the in-flight loads at the back edge, which waits for
    // all of them)
    constexpr int LA = SDR_PATHS_LA;
    constexpr int R = 2 * LA;
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
    // addresses = wave-uniform row base (SGPRs, two scalar adds per step) + 32-bit lane byte
    // offset; inactive (padding) lanes read the pixel's last word and discard it.  Loads run LA
    // steps past either end of a chain into the buffers' slack (kSouthPad rows each side), so
    // neither the addresses nor the stores need a clamp or a branch.
    const uint32_t lofs = (uint32_t)((PAD ? min(lane, D / DPL - 1) : lane) * DPL * 2);
    const ptrdiff_t rowb = (ptrdiff_t)(ch.dy * W1 + ch.dx) * D * 2;
    const size_t p0 = (size_t)f * pl.cs_fstride + ((size_t)ch.y0 * W1 + ch.x0) * D;
    const char* cp = (const char*)(pl.C + p0);  // row k + LA's pixel
    char* op = (char*)(pd.out + p0);            // row k's pixel
    const int last = ch.len - 1;
    // SDR_PATHS_SOFF: one resource per buffer for the whole chain, based at the lowest address
    // the chain's loads touch (row `low`); the SGPR offset of row j is (j - low) * rowb >= 0, and
    // the store resource is shifted so that the store of row k uses the offset of the load of
    // row k + LA, which the step has in hand: one scalar add per step moves both.
    const int low = rowb >= 0 ? 0 : last + LA;
    const Rsrc rC = rsrc_at(cp + (ptrdiff_t)low * rowb);
    const Rsrc rO = rsrc_at(op + (ptrdiff_t)(low - LA) * rowb);
    uint32_t soff = (uint32_t)((ptrdiff_t)(0 - low) * rowb);
    auto cload = [&](const char* base) __attribute__((always_inline)) {
        if constexpr (SDR_PATHS_SOFF) return load_buf_so<K>(rC, lofs, soff);
        else if constexpr (SDR_PATHS_BUF) return load_buf<K>(rsrc_at(base), lofs);
        else return load_regs<K>((const int16_t*)(base + lofs));
    };

    Regs<K> cring[R];
#pragma unroll
    for (int j = 0; j < LA; j++) {
        cring[j] = cload(cp);
        cp += rowb;
        soff += (uint32_t)rowb;
    }

    Regs<K> Lp;
#pragma unroll
    for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    uint32_t delta2 = path_delta0(P2x2);
    uint32_t upr = kMaxPair, dnr = kMaxPair;  // see path_step

    auto step = [&](const int, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const Regs<K> c = cring[j];
        cring[(j + LA) % R] = cload(cp);
        cp += rowb;
        const Regs<K> L = path_step<K, PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr);
        if (active) {  // padding lanes alias the pixel's last word
            if constexpr (NT && SDR_PATHS_SOFF) store_buf_nt_so<K>(rO, lofs, soff, L);
            else if constexpr (NT && SDR_PATHS_BUF) store_buf_nt<K>(rsrc_at(op), lofs, L);
            else if constexpr (NT) store_regs_nt<K>((int16_t*)(op + lofs), L);
            else store_regs<K>((int16_t*)(op + lofs), L);
        }
        op += rowb;
        soff += (uint32_t)rowb;
    };
    int k0 = 0;
    for (; k0 + R <= ch.len; k0 += R) unroll_rows(step, k0, std::make_integer_sequence<int, R>{});
    unroll_rows_tail(step, k0, last, std::make_integer_sequence<int, R - 1>{});
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
// The top-to-bottom direction fused with A.8 (WTA / uniqueness / subpixel / disp2 scatter).
//
// One workgroup per column chain, two roles:
//   wave 0 (producer) runs the serial recurrence of the chain (C loaded kSouthLAB blocks
//     ahead) and stages each row's L in LDS, kSouthRB rows per block, double-buffered;
//   waves 1..3 (consumers) each own 4 rows of a block: a pixel's D disparities sit on one 16-lane
//     DPP row (4 pixels per wave instruction, 16 B per lane per direction), the other P-1
//     directions' L are read from HBM (prefetched whole blocks ahead), the staged L is added
//     from LDS, and the winner-take-all runs on the saturated sums.
// A block is handed over by one barrier.  The serial chain is the only latency-bound part and
// it does nothing but the recurrence; the WTA and the HBM reads of the other directions run on
// three more waves beside it.  L of this direction is never written to HBM, so the pass moves
// 2 + 2(P-1) B/cell.  The uniqueness test needs only the smallest S[d] with |d - best| > 1 (both
// of OpenCV's rules are monotone in S[d]): a masked packed minimum.  disp2 (right-view WTA) is a
// global atomicMin per pixel on (minS << 16 | 0xffff - x) keys (ties -> largest x, OpenCV's
// descending loop); k_lr_check applies A.9.  Loads run past a chain's end into the buffers'
// kSouthPad rows of slack instead of being clamped.
// ------------------------------------------------------------------------------------------
// 1 producer + 3 consumer waves (256 threads): at <= 96 VGPRs five workgroups fit a CU, so
// the 1152 column chains of a 1280x720 d=128 frame are resident in one pass.  2 and 4 consumer
// waves measured the same within noise (C2 single-stream 240-249 us, all three bit-exact).
#ifndef SDR_SOUTH_CONSUMERS
#define SDR_SOUTH_CONSUMERS 3
#endif
constexpr int kSouthConsumers = SDR_SOUTH_CONSUMERS;
constexpr int kSouthRB = 4 * kSouthConsumers;  // rows per block (4 per consumer wave)
#ifndef SDR_SOUTH_LAB
#define SDR_SOUTH_LAB 1
#endif
constexpr int kSouthLAB = SDR_SOUTH_LAB;  // producer lookahead in blocks (D <= 128; 1 above)
#ifndef SDR_SOUTH_PD
#define SDR_SOUTH_PD 0  // consumer prefetch distance in blocks; 0: by register budget
#endif

#ifndef SDR_SOUTH_SOFF
// k_south_wta producer: one resource per chain + SGPR row offset (1) or a resource per load (0).
// Measured C2 single-stream k_south_wta 238-241 us with 1 and 229-232 us with 0 (the compiler
// bunches the offset-addressed loads into one burst per block), so it stays off here.
#define SDR_SOUTH_SOFF 0
#endif
#ifndef SDR_SOUTH_SPAD
#define SDR_SOUTH_SPAD 4  // dword padding of the consumers' staged S rows
#endif
#ifndef SDR_SOUTH_LDSU
#define SDR_SOUTH_LDSU 1  // consumers: S row staged in LDS for subpixel + uniqueness (0: in registers)
#endif
#ifndef SDR_SOUTH_STAMP
#define SDR_SOUTH_STAMP 0  // diagnostic build: per-wave cycles (total, in barriers) into keys2
#endif
// barrier with optional wait-time accounting (SDR_SOUTH_STAMP)
struct StampBarrier {
    uint64_t t0 = 0, wait = 0;
    __device__ __forceinline__ void start() {
        if constexpr (SDR_SOUTH_STAMP) t0 = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void sync() {
        if constexpr (SDR_SOUTH_STAMP) {
            const uint64_t a = __builtin_amdgcn_s_memtime();
            __syncthreads();
            wait += __builtin_amdgcn_s_memtime() - a;
        } else {
            __syncthreads();
        }
    }
    __device__ __forceinline__ void finish(uint32_t* keys, int slot, int lane) {
        if constexpr (SDR_SOUTH_STAMP) {
            const uint64_t tot = __builtin_amdgcn_s_memtime() - t0;
            if (lane == 0) {
                ((uint64_t*)keys)[2 * slot] = tot;
                ((uint64_t*)keys)[2 * slot + 1] = wait;
            }
        }
    }
};

#ifndef SDR_SOUTH_ROTATE
#define SDR_SOUTH_ROTATE 0  // producer role rotated over the wave slots: bit-exact, no change (229-234 us)
#endif
#ifndef SDR_SOUTH_FLAGS
#define SDR_SOUTH_FLAGS 0  // block hand-over by LDS counters over 3 slots (0: a barrier per block)
#endif
// SDR_SOUTH_FLAGS: the producer publishes "blocks staged" and each consumer "blocks consumed" in
// LDS counters, so neither side waits for the other's slowest block as long as a slot is free.
// Spins are bounded: a protocol error ends in wrong results (caught by the parity tests), never
// in a wave that spins forever.  Bit-exact on MI355X but not faster (C2 single-stream 246-247 vs
// 241-242 us with the barrier), so the barrier stays: the waits are not what bounds the pass.
__device__ __forceinline__ void south_wait_ge(int* p, int v) {
    for (int n = 0; n < (1 << 22); n++) {
        const int c = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (c >= v) return;
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ void south_publish(int* p, int v, int lane) {
    if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int DPL, bool PAD, int NP>
__global__ __launch_bounds__(64 * (1 + kSouthConsumers)) void k_south_wta(Geometry g, PathLaunch pl,
                                                                           SouthWtaArgs a) {
    constexpr int K = DPL / 2;
    constexpr int RB = kSouthRB;
    constexpr int LAB = K == 1 ? kSouthLAB : 1;  // producer lookahead in blocks
    constexpr int LA = LAB * RB;                 // ... in rows
    constexpr int NS = 2 * LAB;                  // ring blocks per producer loop body
    constexpr int R = NS * RB;                   // producer ring slots (rows)
    static_assert(LA + RB <= kSouthPad, "load overrun must fit the buffers' row slack");
    constexpr int WDPL = DPL * 4;  // consumer: disparities per lane
    constexpr int WK = WDPL / 2;
    constexpr int DMAX = 64 * DPL;
    constexpr int LSTR = DMAX / 2 + 4;  // dwords per staged row (padded: rows of a wave's 4 pixels)
    // consumer prefetch distance in blocks: the ring (2*PD blocks) of the other directions' L
    constexpr int PD = SDR_SOUTH_PD ? SDR_SOUTH_PD : (NP * WK <= 8 ? 2 : 1);
    static_assert((PD + 1) * RB <= kSouthPad, "consumer load overrun must fit the row slack");
    constexpr int NB = SDR_SOUTH_FLAGS ? 3 : 2;  // LDS slots of staged L blocks
    __shared__ uint32_t sL[NB][RB][LSTR];
    __shared__ int s_prod, s_cons[kSouthConsumers];
    // SDR_SOUTH_LDSU: each consumer row's S staged in LDS for the subpixel neighbours and the
    // uniqueness minimum (one 16-B write per lane, three masking u16 writes, one read back)
    // rows padded by 4 dwords: the four lane groups' 16-B writes start on different banks
    __shared__ uint32_t sS[SDR_SOUTH_LDSU ? kSouthConsumers : 1][4][SDR_SOUTH_LDSU ? DMAX / 2 + SDR_SOUTH_SPAD : 1];
    const int lane = threadIdx.x & 63;
    // role of this wave (0 = producer); SDR_SOUTH_ROTATE moves the producer role to a different
    // hardware wave slot in consecutive workgroups, so the producers of the workgroups sharing a
    // CU do not all sit on the same SIMD if slots map to SIMDs in order
    const int hw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wv = SDR_SOUTH_ROTATE ? (hw + (int)blockIdx.x) % (1 + kSouthConsumers) : hw;
    const int cg = blockIdx.x;
    const int f = blockIdx.y;
    int di = 0;
    while (cg >= pl.prefix[di + 1]) di++;
    const PathDir pd = pl.d[di];
    const Chain ch = make_chain(g, pd, cg - pl.prefix[di]);
    if (ch.len <= 0) return;  // whole workgroup
    const int D = g.D, W1 = g.W1;
    const size_t fofs = (size_t)f * pl.cs_fstride;
    const int last = ch.len - 1;
    const int nblk = (ch.len + RB - 1) / RB;
    StampBarrier sb;
    if constexpr (SDR_SOUTH_FLAGS) {
        if (threadIdx.x == 0) {
            s_prod = 0;
            for (int c = 0; c < kSouthConsumers; c++) s_cons[c] = 0;
        }
        __syncthreads();
    }
    sb.start();
    const int stamp_slot = (blockIdx.y * gridDim.x + blockIdx.x) * (1 + kSouthConsumers) + wv;

    if (wv == 0) {
        // ---------------- producer: the recurrence, L rows to LDS ----------------
        __builtin_amdgcn_s_setprio(2);
        const bool active = !PAD || lane * DPL < D;
        const uint32_t lofs = (uint32_t)((PAD ? min(lane, D / DPL - 1) : lane) * DPL * 2);
        const ptrdiff_t rowb = (ptrdiff_t)W1 * D * 2;
        // 3WAY stripes: a chain starting at aux_row0 reads its first aux_rows (< LA) cost rows
        // from the stripe-local (row-major) buffer; every later row comes from C
        const int naux = pd.Caux ? pd.aux_rows : 0;
        const char* abase = pd.Caux ? (const char*)(pd.Caux + (size_t)f * pl.aux_fstride + (size_t)ch.x0 * D)
                                    : (const char*)pl.C;
        const char* cp = (const char*)(pl.C + fofs + ((size_t)ch.y0 * W1 + ch.x0) * D);  // row k + LA
        auto cload = [&](const char* base) __attribute__((always_inline)) {
            if constexpr (SDR_SOUTH_BUF) return load_buf<K>(rsrc_at(base), lofs);
            else return load_regs<K>((const int16_t*)(base + lofs));
        };
        // in the loop: one resource for the chain's column of C and an SGPR row offset (rows
        // only go down, so offsets from row 0 are non-negative; see k_paths)
        const Rsrc rC = rsrc_at(cp);
        uint32_t soff = 0;
        auto cload_loop = [&]() __attribute__((always_inline)) {
            if constexpr (SDR_SOUTH_SOFF) return load_buf_so<K>(rC, lofs, soff);
            else return cload(cp);
        };
        // ring of 2*LA rows loaded LA ahead (see k_paths: no copies at the loop's back edge)
        Regs<K> cring[R];
#pragma unroll
        for (int j = 0; j < LA; j++) {
            cring[j] = cload(j < naux ? abase + (ptrdiff_t)j * rowb : cp);
            cp += rowb;
            soff += (uint32_t)rowb;
        }
        Regs<K> Lp;
#pragma unroll
        for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
        const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
        uint32_t delta2 = path_delta0(P2x2);
        uint32_t upr = kMaxPair, dnr = kMaxPair;  // see path_step
        // block bb (= slot ic of the ring): RB recurrence steps into LDS slot bb & 1, then hand over
        auto block = [&](const int bb, auto ic) __attribute__((always_inline)) {
            if constexpr (SDR_SOUTH_FLAGS) {
                if (bb >= NB)  // slot bb % NB held block bb - NB: every consumer must be done with it
#pragma unroll
                    for (int c = 0; c < kSouthConsumers; c++) south_wait_ge(&s_cons[c], bb - NB + 1);
            }
            uint32_t* dst = &sL[SDR_SOUTH_FLAGS ? bb % NB : bb & 1][0][lane * K];
            auto st = [&](const int, auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value + decltype(ic)::value * RB;  // ring slot = k % R
                const Regs<K> c = cring[j];
                cring[(j + LA) % R] = cload_loop();
                cp += rowb;
                soff += (uint32_t)rowb;
                const Regs<K> L = path_step<K, PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr);
#pragma unroll
                for (int i = 0; i < K; i++) dst[(j % RB) * LSTR + i] = L.r[i];
            };
            unroll_rows(st, bb * RB, std::make_integer_sequence<int, RB>{});
            if constexpr (SDR_SOUTH_FLAGS) south_publish(&s_prod, bb + 1, lane);
            else sb.sync();
        };
        int b = 0;
        for (; b + NS <= nblk; b += NS) unroll_rows(block, b, std::make_integer_sequence<int, NS>{});
        unroll_rows_tail(block, b, nblk - 1, std::make_integer_sequence<int, NS - 1>{});
        if constexpr (!SDR_SOUTH_FLAGS) sb.sync();  // the consumers' last block
        sb.finish(a.keys2, stamp_slot, lane);
        return;
    }

    // ---------------- consumers: the other directions + WTA, 4 rows per wave ----------------
    const int gl = lane & 15, grp = lane >> 4;
    const int r = (wv - 1) * 4 + grp;  // this lane group's row within a block
    const bool wactive = !PAD || gl * WDPL < D;
    const int wd0 = (PAD ? min(gl, D / WDPL - 1) : gl) * WDPL;
    // row blk*RB + r of the chain: wave-uniform block base + lane byte offset
    const ptrdiff_t bstepb = (ptrdiff_t)RB * W1 * D * 2;
    const uint32_t lofs = (uint32_t)(((size_t)r * W1 * D + wd0) * 2);
    const size_t p0 = fofs + ((size_t)ch.y0 * W1 + ch.x0) * D;
    auto oload = [&](int q, int blk) __attribute__((always_inline)) {
        const char* base = (const char*)(a.L[q] + p0) + (ptrdiff_t)blk * bstepb;
        if constexpr (SDR_SOUTH_BUF) return load_buf<WK>(rsrc_at(base), lofs);
        else return load_regs<WK>((const int16_t*)(base + lofs));
    };
    // rows before kw belong to the previous 3WAY stripe: recurred through, never output
    const int kw = ch.kwrite;
    const int invalid = (g.minD - 1) * 16;
    const bool check_uniq = a.uniq > 0 || !a.uniq_simd;
    const bool uniq_simd = a.uniq_simd != 0;
    const int lhs_scale = 100 - a.uniq;
    const double inv100u = 1.0 / (double)(100 - a.uniq) * (1.0 + 0x1p-40);
    const int x = ch.x0;  // matched-range column of this chain
    int16_t* raw = a.disp_raw + (size_t)f * a.disp_fstride + x + g.minX1;
    uint32_t* keys = a.keys2 + (size_t)f * a.disp_fstride;

    // ring of 2*PD blocks loaded PD ahead (as the producer's: no copies at the back edge);
    // unconditional: blocks past the chain's end read the buffers' row slack (kSouthPad)
    constexpr int OR = 2 * PD;
    Regs<WK> oring[OR][NP];
#pragma unroll
    for (int s = 0; s < PD; s++)
#pragma unroll
        for (int q = 0; q < NP; q++) oring[s][q] = oload(q, s);

    auto consume_sync = [&](const int b, auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        Regs<WK> o[NP];
#pragma unroll
        for (int q = 0; q < NP; q++) o[q] = oring[s][q];
#pragma unroll
        for (int q = 0; q < NP; q++) oring[(s + PD) % OR][q] = oload(q, b + PD);
        // S = sat(sum of the P path costs), the fused direction's L from LDS
        if constexpr (SDR_SOUTH_FLAGS) south_wait_ge(&s_prod, b + 1);  // block b staged
        const uint32_t* ls = &sL[SDR_SOUTH_FLAGS ? b % NB : b & 1][r][wd0 / 2];
        Regs<WK> St;
#pragma unroll
        for (int i = 0; i < WK; i++) {
            uint32_t acc = 0;
#pragma unroll
            for (int p = 0; p <= NP; p++) {
                const uint32_t v = p == kSouthIdx ? ls[i] : o[p < kSouthIdx ? p : p - 1].r[i];
                acc = p == 0 ? v : pk_add_sat(acc, v);
            }
            St.r[i] = acc;
        }
        const int k = b * RB + r;
        const bool rowok = k >= kw && k <= last;
        // first minimum: packed (S + 32768) << 16 | d keys, min over the 16-lane row
        uint32_t key = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < WK; i++) {
            const uint32_t d = (uint32_t)(gl * WDPL + 2 * i);
            const uint32_t lo = (uint32_t)((int)(short)(St.r[i] & 0xffff) + 32768);
            const uint32_t hi = (uint32_t)((int)(short)(St.r[i] >> 16) + 32768);
            key = min(key, min((lo << 16) | d, (hi << 16) | (d + 1)));
        }
        uint32_t* srow = &sS[SDR_SOUTH_LDSU ? wv - 1 : 0][grp][0];
        if constexpr (SDR_SOUTH_LDSU) {
#pragma unroll
            for (int i = 0; i < WK; i++) ((uint32_t __attribute__((may_alias))*)srow)[gl * WK + i] = St.r[i];
        }
        key = row16_min_u32(wactive ? key : 0xffffffffu);
        const int minS = (int)(key >> 16) - 32768;
        const int best = (int)(key & 0xffff);
        const int dm = max(best - 1, 0), dp = min(best + 1, D - 1);
        // uniqueness: min of S[d] over |d - best| > 1 (0 <= S <= 32767: 0x7fff masks a half)
        uint32_t m2 = kMaxPair;
        int Sm_l = 0, Sp_l = 0;
        if constexpr (SDR_SOUTH_LDSU) {
            // the halfword accesses alias the row's 32-bit words: may_alias keeps their order
            typedef int16_t __attribute__((may_alias)) s16a;
            typedef uint32_t __attribute__((may_alias)) u32a;
            s16a* s16 = (s16a*)srow;
            Sm_l = s16[dm];
            Sp_l = s16[dp];
            s16[dm] = 0x7fff;
            s16[best] = 0x7fff;
            s16[dp] = 0x7fff;
#pragma unroll
            for (int i = 0; i < WK; i++) m2 = pk_min(m2, ((u32a*)srow)[gl * WK + i]);
        } else {
#pragma unroll
            for (int i = 0; i < WK; i++) {
                const int t = gl * WDPL + 2 * i - best;
                const uint32_t mk = ((unsigned)(t + 1) <= 2u ? 0x7fffu : 0u) | ((unsigned)(t + 2) <= 2u ? 0x7fff0000u : 0u);
                m2 = pk_min(m2, St.r[i] | mk);
            }
        }
        m2 = wactive ? m2 : kMaxPair;
        m2 = pk_min(m2, funnel16(m2, m2));
        m2 = row16_min_u32(m2);
        const int min2 = (int)(m2 & 0x7fff);
        // SIMD rule: S[d] < (short)(thresh + 1), thresh = (100*minS)/(100-u); scalar: S*(100-u) < 100*minS
        const int thr16 = (int)(short)((int)((double)(100 * minS) * inv100u) + 1);
        const bool reject = check_uniq && (uniq_simd ? (min2 < thr16) : (min2 * lhs_scale < minS * 100));
        // subpixel: d*16 + ((S[d-1]-S[d+1])*16 + den) / (2*den), C truncating division
        uint32_t am = 0, ap = 0;
        if constexpr (!SDR_SOUTH_LDSU) {
            uint32_t wm = St.r[0], wp = St.r[0];
#pragma unroll
            for (int i = 1; i < WK; i++) {
                if (((dm % WDPL) >> 1) == i) wm = St.r[i];
                if (((dp % WDPL) >> 1) == i) wp = St.r[i];
            }
            am = (uint32_t)__shfl((int)wm, grp * 16 + dm / WDPL);
            ap = (uint32_t)__shfl((int)wp, grp * 16 + dp / WDPL);
        }
        if (gl == 0 && rowok) {
            const size_t y = (size_t)(ch.y0 + k);
            int out = invalid;
            // every S saturated: OpenCV's first-minimum scan (strict '<' from MAX_COST) keeps
            // bestDisp = -1, whose value (-1 + minD) * 16 is INVALID and whose disp2 candidate
            // (cost MAX_COST) never replaces the initial one
            if (!reject && minS < kMaxCost) {
                const int Sm = SDR_SOUTH_LDSU ? Sm_l : (int)(short)((dm & 1) ? (am >> 16) : (am & 0xffff));
                const int Sp = SDR_SOUTH_LDSU ? Sp_l : (int)(short)((dp & 1) ? (ap >> 16) : (ap & 0xffff));
                const int den = max(Sm + Sp - 2 * minS, 1);
                const int qq = div_trunc_small((Sm - Sp) * 16 + den, 2 * den);
                out = best * 16 + (((0 < best) & (best < D - 1)) ? qq : 0) + g.minD * 16;
                const int x2 = x + g.minX1 - best - g.minD;
                if (x2 >= 0 && x2 < g.W)
                    atomicMin(&keys[y * g.W + x2], ((uint32_t)minS << 16) | (uint32_t)(0xffff - x));
            }
            raw[y * g.W] = (int16_t)out;
        }
        if constexpr (SDR_SOUTH_FLAGS) south_publish(&s_cons[wv - 1], b + 1, lane);
        else sb.sync();
    };
    if constexpr (!SDR_SOUTH_FLAGS) sb.sync();  // block 0 staged
    int b = 0;
    for (; b + OR <= nblk; b += OR) unroll_rows(consume_sync, b, std::make_integer_sequence<int, OR>{});
    unroll_rows_tail(consume_sync, b, nblk - 1, std::make_integer_sequence<int, OR - 1>{});
    sb.finish(a.keys2, stamp_slot, lane);
}

// disp_raw := invalid, keys2 := no match (per frame, before k_south_wta)
__global__ __launch_bounds__(256) void k_wta_init(int16_t* __restrict__ raw, uint32_t* __restrict__ keys,
                                                  size_t n, int invalid) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        raw[i] = (int16_t)invalid;
        keys[i] = 32767u << 16;
    }
}

// A.9 on the fused pass's outputs: disp2 from the scattered keys, then OpenCV's check
__global__ __launch_bounds__(256) void k_lr_check(Geometry g, const int16_t* __restrict__ raw,
                                                  const uint32_t* __restrict__ keys,
                                                  int16_t* __restrict__ out, size_t fstride,
                                                  int disp12MaxDiff) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y, f = blockIdx.z;
    if (x >= g.W) return;
    const size_t ro = (size_t)f * fstride + (size_t)y * g.W;
    const int invalid = (g.minD - 1) * 16;
    const uint32_t kInit = 32767u << 16;
    auto disp2 = [&](int xx) {
        const uint32_t k = keys[ro + xx];
        return k == kInit ? invalid : ((0xffff - (int)(k & 0xffff)) + g.minX1 - xx);
    };
    int d1 = raw[ro + x];
    if (x >= g.minX1 && x < g.minX1 + g.W1 && d1 != invalid) {
        const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
        const int _x = x - _d, x_ = x - d_;
        if (0 <= _x && _x < g.W && 0 <= x_ && x_ < g.W) {
            const int a2 = disp2(_x), b2 = disp2(x_);
            if (a2 >= g.minD && abs(a2 - _d) > disp12MaxDiff && b2 >= g.minD && abs(b2 - d_) > disp12MaxDiff)
                d1 = invalid;
        }
    }
    out[ro + x] = (int16_t)d1;
}

template <int DPL, bool PAD>
static void launch_south_np(const Geometry& g, const PathLaunch& pl, const SouthWtaArgs& a, int F,
                            hipStream_t st) {
    dim3 grid(pl.prefix[pl.ndirs], F);
    dim3 block(64 * (1 + kSouthConsumers));
    switch (a.npaths) {
    case 3: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 2>), grid, block, 0, st, g, pl, a); break;
    case 5: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 4>), grid, block, 0, st, g, pl, a); break;
    default: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 7>), grid, block, 0, st, g, pl, a); break;
    }
}

void launch_south_wta(const Geometry& g, const PathLaunch& pl, const SouthWtaArgs& a, int F,
                      hipStream_t st) {
    const size_t n = (size_t)F * a.disp_fstride;
    hipLaunchKernelGGL(k_wta_init, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0,
                       st, a.disp_raw, a.keys2, n, (g.minD - 1) * 16);
    if (pl.prefix[pl.ndirs] <= 0) return;
    if (g.D <= 128) {
        if (g.D < 128) launch_south_np<2, true>(g, pl, a, F, st);
        else launch_south_np<2, false>(g, pl, a, F, st);
    } else {
        if (g.D < 256) launch_south_np<4, true>(g, pl, a, F, st);
        else launch_south_np<4, false>(g, pl, a, F, st);
    }
}

void launch_lr_check(const Geometry& g, const int16_t* raw, const uint32_t* keys, int16_t* out,
                     size_t fstride, int disp12MaxDiff, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_lr_check, dim3((g.W + 255) / 256, g.H, F), dim3(256), 0, st, g, raw, keys, out,
                       fstride, disp12MaxDiff);
}

}  // namespace sdr
