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
// first minimum, uniqueness, subpixel) as a producer/consumer workgroup; it leaves each pixel's
// WTA disparity and folds its (minS, x) into the right view's WTA keys (disp2) by atomicMin; the
// left-right check (lr_at) is then computed by the median's tiles from those two maps.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <algorithm>

namespace sdr {

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

// The per-word recurrence of one step: L = C + min(Lp, min(Lp[d-1], Lp[d+1]) + P1, delta2) -
// delta2 for the lane's K words, and m = the minimum of L's pairs.  (Issuing two words' packed ops
// alternately -- 4 x int16 vector ops, no packed op right after the one it reads, so none of
// gfx950's wait states -- removed ~40 % of the path kernels' s_nops and measured no faster: at
// 3-4 waves per SIMD the other waves fill those slots; profiles/r4_ab_variants.txt.)
template <int K, bool PAD>
__device__ __forceinline__ void step_words(const Regs<K>& c, const Regs<K>& Lp, uint32_t delta2, uint32_t P1x2,
                                           bool active, uint32_t up, uint32_t dn, Regs<K>& L, uint32_t& m) {
    m = kMaxPair;
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
}

// One step of the path recurrence on a wave's packed int16 pairs (lane l: disparities
// [l*2K, l*2K + 2K)); returns L of this pixel.  State: Lp := L, delta2 := minL + P2 (both
// halves).  upr/dnr: the lane-shifted neighbour words of the previous step -- a wave shift leaves
// the lane without a source (lane 0 / lane 63) unwritten, so passing the previous shift as the
// DPP's old value keeps the kMaxPair boundary there from the first step on, with no refill.
// (An offset-carrying form that takes the wave minimum off the serial chain was bit-exact and
// not faster on MI355X)  The wave minimum is a wave-uniform (SGPR) value.
template <int K, bool PAD>
__device__ __forceinline__ Regs<K> path_step(Regs<K> c, Regs<K>& Lp, uint32_t& delta2, uint32_t P1x2,
                                             uint32_t P2x2, bool active, uint32_t& upr, uint32_t& dnr) {
    if constexpr (PAD) {
#pragma unroll
        for (int i = 0; i < K; i++) c.r[i] = active ? c.r[i] : kMaxPair;
    }
    const uint32_t up = upr = lane_from_prev(Lp.r[K - 1], upr);
    const uint32_t dn = dnr = lane_from_next(Lp.r[0], dnr);
    Regs<K> L;
    uint32_t m;
    step_words<K, PAD>(c, Lp, delta2, P1x2, active, up, dn, L, m);
    // min of the pair into the low half (one SDWA op; L >= 0, so u16 order is int16 order), the
    // wave minimum as a wave-uniform value, splatted and offset by P2 in scalar registers
    const uint32_t m16 = (uint32_t)__builtin_elementwise_min((unsigned short)(m & 0xffffu),
                                                              (unsigned short)(m >> 16));
    delta2 = wave_min_u32_uniform(m16) * 0x00010001u + P2x2;
    Lp = L;
    return L;
}

// k_paths lookahead (steps).  32 steps at D <= 128 measured slower on the class path's 640x360
// frames (k_paths 75 -> 82 us for both matchers; C2 unchanged): its E/W chains wait on the
// memory system (3.4 TB/s over the launch), not on the lookahead.
// (8 at D > 256: four pairs per lane, a 16-slot ring is already 64 VGPRs)
template <int DPL>
constexpr int paths_la() { return DPL == 8 ? 8 : 16; }
// k_paths loads C with the default cache policy: the launch's four directions (and k_south_wta
// after it) re-read C, and the 212 MB volume of a C2 frame is served partly from the 256 MB
// Infinity Cache -- non-temporal C loads there measured 274 -> 340 us.
// k_south_wta is the last reader of both C and the L records, and loads them non-temporal: the
// consumers' L records (849 MB a C2 frame) then stop evicting C and each other from the caches,
// 219 -> 183 us (MI355X, scripts/kbench.py A/B, bit-exact).
constexpr int kLoadNT = 2;

template <int DPL, bool PAD>
__global__ __launch_bounds__(256) void k_paths(Geometry g, PathLaunch pl) {
    constexpr int K = DPL / 2;
    // C is loaded LA steps ahead into a ring of 2*LA slots: the slot a load fills was consumed
    // LA steps earlier, so every slot keeps one register across the loop's back edge (a ring
    // of LA slots makes the compiler copy the in-flight loads at the back edge, which waits for
    // all of them)
    constexpr int LA = paths_la<DPL>();
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
    // addresses = wave-uniform chain base (a buffer resource) + SGPR row offset + 32-bit lane
    // byte offset; inactive (padding) lanes read the pixel's last word and discard it.  Loads run
    // LA steps past either end of a chain into the buffers' slack (kSouthPad rows each side), so
    // neither the addresses nor the stores need a clamp or a branch.
    const uint32_t lofs = (uint32_t)((PAD ? min(lane, D / DPL - 1) : lane) * DPL * 2);
    const ptrdiff_t rowb = (ptrdiff_t)(ch.dy * W1 + ch.dx) * D * 2;          // C, per step
    const ptrdiff_t rowl = (ptrdiff_t)(ch.dy * W1 + ch.dx) * pl.l_pix * 2;   // L records, per step
    const char* cp = (const char*)(pl.C + (size_t)f * pl.cs_fstride + ((size_t)ch.y0 * W1 + ch.x0) * D);
    if (pd.dir == DIR_E || pd.dir == DIR_W) {
        // a short last 3WAY stripe's output rows: its own cost rows (RowRedirect)
        for (int i = 0; i < pl.nredir; i++)
            if (ch.y0 >= pl.redir[i].lo && ch.y0 < pl.redir[i].hi)
                cp = (const char*)(pl.redir[i].aux + (size_t)f * pl.aux_fstride +
                                   ((size_t)(ch.y0 - pl.redir[i].s0) * W1 + ch.x0) * D);
    }
    char* op = (char*)(pd.out + (size_t)f * pl.l_fstride + ((size_t)ch.y0 * W1 + ch.x0) * pl.l_pix);
    const int last = ch.len - 1;
    // C: one resource for the whole chain, based at the lowest address the chain's loads touch
    // (row `low`); the SGPR offset of row j is (j - low) * rowb >= 0 (below 2^31: the engine
    // refuses frames whose chain span passes it).  L: the record stride is P-1 times larger, so
    // the store resource is re-based at every ring period (R steps) instead.
    const int low = rowb >= 0 ? 0 : last + LA;
    const Rsrc rC = rsrc_at(cp + (ptrdiff_t)low * rowb);
    uint32_t soff = (uint32_t)((ptrdiff_t)(0 - low) * rowb);
    Rsrc rO;
    uint32_t soffl = 0;
    auto rebase = [&](int k0) __attribute__((always_inline)) {
        const int lo = rowl >= 0 ? k0 : k0 + R - 1;
        rO = rsrc_at(op + (ptrdiff_t)lo * rowl);
        soffl = (uint32_t)((ptrdiff_t)(k0 - lo) * rowl);
    };

    Regs<K> cring[R];
#pragma unroll
    for (int j = 0; j < LA; j++) {
        cring[j] = load_buf<K>(rC, lofs, soff);
        soff += (uint32_t)rowb;
    }

    Regs<K> Lp;
#pragma unroll
    for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    uint32_t delta2 = P2x2;                   // minLp = 0 before a chain's first pixel
    uint32_t upr = kMaxPair, dnr = kMaxPair;  // see path_step

    // path-cost stores are non-temporal: measured on MI355X (C2, 2 frames in flight) +4 % fps
    // over default-policy stores, the WTA's re-reads of the L buffers getting faster.
    // The store is unconditional: padding lanes (which alias the last word on loads) get a lane
    // offset past the resource's num_records, so the hardware drops their writes.  A store under
    // `if (active)` put a branch in every step, and the compiler's vmcnt accounting then had to
    // assume the path where no store was issued: every step waited until only 15 memory ops
    // were outstanding, i.e. for the C load of ~8 steps back instead of 16 -- the E/W chains of
    // the padded D = 80 class path ran at the memory latency / 8 per step.
    const uint32_t sofs_st = active ? lofs : 0x80000000u;
    auto step = [&](const int, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const Regs<K> c = cring[j];
        cring[(j + LA) % R] = load_buf<K>(rC, lofs, soff);
        soff += (uint32_t)rowb;
        const Regs<K> L = path_step<K, PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr);
        store_buf_nt<K>(rO, sofs_st, soffl, L);
        soffl += (uint32_t)rowl;
        // one scheduling region per step (as the branch used to make it): scheduled across the
        // whole unrolled ring, the steps' loads and stores were reordered and the ring registers
        // copied, with vmcnt(0) waits inside the loop
        __builtin_amdgcn_sched_barrier(0);
    };
    int k0 = 0;
    for (; k0 + R <= ch.len; k0 += R) {
        rebase(k0);
        unroll_rows(step, k0, std::make_integer_sequence<int, R>{});
    }
    rebase(k0);
    unroll_rows_tail(step, k0, last, std::make_integer_sequence<int, R - 1>{});
}

// k_paths with TWO chains per wave (lanes 0-31: chain 2w, lanes 32-63: chain 2w+1 of the same
// direction), four disparities (two packed pairs) per lane, for the latency-bound launches: D <=
// 128 and more chains than SIMDs but few enough that each chain waits on its own serial steps.
// The class path's paired 3WAY matchers at 640x360 have 1440 E/W chains of 560 steps: one per
// wave, 416 SIMDs held two and every such chain ran ~1.6x slower (C4 k_paths 85 us, against 54
// for the 720 chains of one matcher); two per wave, all 720 waves have a SIMD to themselves, and a
// step costs about the same instructions for two chains as the one-chain step for one.
//   - the d +- 1 neighbours cross lanes by the same DPP wave shifts, with lane 32 (31) given the
//     chain's boundary value instead of the other chain's lane 31 (32);
//   - the per-chain minimum: DPP row minima, row_bcast:15 into rows 1 and 3 (lanes 31 and 63 then
//     hold the two halves' minima), two readlanes, and the half's delta selected per lane;
//   - one buffer resource per wave based at chain A; chain B's lanes carry the (non-negative)
//     distance to chain B in their offset.  Only directions whose chains all have one length (E, W,
//     N, S) take this kernel, so the two chains step together.
// One step of two chains (lanes 0-31: chain A, 32-63: chain B; two packed pairs per lane):
// path_step with the chains' boundary lanes fed their own fill and a per-half minimum.
template <bool PAD>
__device__ __forceinline__ Regs<2> path_step_tc(Regs<2> c, Regs<2>& Lp, uint32_t& delta2, uint32_t P1x2,
                                                uint32_t P2x2, bool active, uint32_t& upr, uint32_t& dnr,
                                                int lane) {
    constexpr int K = 2;
    if constexpr (PAD) {
#pragma unroll
        for (int i = 0; i < K; i++) c.r[i] = active ? c.r[i] : kMaxPair;
    }
    upr = lane_from_prev(Lp.r[K - 1], upr);
    dnr = lane_from_next(Lp.r[0], dnr);
    const uint32_t up = lane == 32 ? kMaxPair : upr;  // chain B's first lane: its own boundary
    const uint32_t dn = lane == 31 ? kMaxPair : dnr;
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
    // the two chains' minima, in every lane of each half: 16-lane row minima (DPP), then rows 0+1
    // and 2+3 by one v_permlane16_swap (rows 0 <-> 1, 2 <-> 3); no readlane / scalar round trip
    uint32_t m16 = (uint32_t)__builtin_elementwise_min((unsigned short)(m & 0xffffu), (unsigned short)(m >> 16));
    m16 = row16_min_u32(m16);
    const auto p16 = __builtin_amdgcn_permlane16_swap(m16, m16, false, false);
    m16 = min((uint32_t)p16[0], (uint32_t)p16[1]);
    delta2 = m16 * 0x00010001u + P2x2;
    Lp = L;
    return L;
}

template <bool PAD>
__global__ __launch_bounds__(256) void k_paths_tc(Geometry g, PathLaunch pl) {
    constexpr int DPL = 4, K = 2;
    constexpr int LA = paths_la<DPL>();
    constexpr int R = 2 * LA;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5, hl = lane & 31;
    const int wg = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int f = blockIdx.y;
    int di = 0, w0 = 0;
    for (; di < pl.ndirs; di++) {
        const int nw = (pl.d[di].nchains + 1) / 2;
        if (wg < w0 + nw) break;
        w0 += nw;
    }
    if (di >= pl.ndirs) return;
    const PathDir pd = pl.d[di];
    const int ca = 2 * (wg - w0);
    const bool hasB = ca + 1 < pd.nchains;
    const Chain ch = make_chain(g, pd, ca);
    const Chain chB = make_chain(g, pd, hasB ? ca + 1 : ca);
    if (ch.len <= 0) return;

    const int D = g.D, W1 = g.W1;
    const bool active = (half == 0 || hasB) && (!PAD || hl * DPL < D);
    const uint32_t lofs = (uint32_t)((PAD ? min(hl, D / DPL - 1) : hl) * DPL * 2);
    const ptrdiff_t pixB = (ptrdiff_t)(chB.y0 - ch.y0) * W1 + (chB.x0 - ch.x0);  // >= 0
    const ptrdiff_t rowb = (ptrdiff_t)(ch.dy * W1 + ch.dx) * D * 2;
    const ptrdiff_t rowl = (ptrdiff_t)(ch.dy * W1 + ch.dx) * pl.l_pix * 2;
    const uint32_t vld = lofs + (half ? (uint32_t)(pixB * D * 2) : 0u);
    const uint32_t vst = active ? lofs + (half ? (uint32_t)(pixB * pl.l_pix * 2) : 0u) : 0x80000000u;
    const char* cp = (const char*)(pl.C + (size_t)f * pl.cs_fstride + ((size_t)ch.y0 * W1 + ch.x0) * D);
    char* op = (char*)(pd.out + (size_t)f * pl.l_fstride + ((size_t)ch.y0 * W1 + ch.x0) * pl.l_pix);
    const int last = ch.len - 1;
    const int low = rowb >= 0 ? 0 : last + LA;
    const Rsrc rC = rsrc_at(cp + (ptrdiff_t)low * rowb);
    uint32_t soff = (uint32_t)((ptrdiff_t)(0 - low) * rowb);
    Rsrc rO;
    uint32_t soffl = 0;
    auto rebase = [&](int k0) __attribute__((always_inline)) {
        const int lo = rowl >= 0 ? k0 : k0 + R - 1;
        rO = rsrc_at(op + (ptrdiff_t)lo * rowl);
        soffl = (uint32_t)((ptrdiff_t)(k0 - lo) * rowl);
    };
    Regs<K> cring[R];
#pragma unroll
    for (int j = 0; j < LA; j++) {
        cring[j] = load_buf<K>(rC, vld, soff);
        soff += (uint32_t)rowb;
    }
    Regs<K> Lp;
#pragma unroll
    for (int i = 0; i < K; i++) Lp.r[i] = active ? 0u : kMaxPair;
    const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
    uint32_t delta2 = P2x2;
    uint32_t upr = kMaxPair, dnr = kMaxPair;
    auto step = [&](const int, auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const Regs<K> c = cring[j];
        cring[(j + LA) % R] = load_buf<K>(rC, vld, soff);
        soff += (uint32_t)rowb;
        const Regs<K> L = path_step_tc<PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr, lane);
        store_buf_nt<K>(rO, vst, soffl, L);
        soffl += (uint32_t)rowl;
        __builtin_amdgcn_sched_barrier(0);
    };
    int k0 = 0;
    for (; k0 + R <= ch.len; k0 += R) {
        rebase(k0);
        unroll_rows(step, k0, std::make_integer_sequence<int, R>{});
    }
    rebase(k0);
    unroll_rows_tail(step, k0, last, std::make_integer_sequence<int, R - 1>{});
}

// the two-chain kernel for this launch?  D <= 128, no redirected 3WAY rows, every direction with
// chains of one length, and more chains than the chip's SIMDs (with fewer, one chain per wave
// already has a SIMD each and the one-chain step is the cheaper one)
static bool paths_two_chain(const Geometry& g, const PathLaunch& pl, int F) {
    if (g.D > 128 || pl.nredir > 0) return false;
    for (int i = 0; i < pl.ndirs; i++)
        if (pl.d[i].dir != DIR_E && pl.d[i].dir != DIR_W && pl.d[i].dir != DIR_N) return false;
    return (long)pl.prefix[pl.ndirs] * F > 4L * device_cus();
}

void launch_paths(const Geometry& g, const PathLaunch& pl, int F, hipStream_t st) {
    const int total = pl.prefix[pl.ndirs];
    if (total <= 0) return;
    if (paths_two_chain(g, pl, F)) {
        int waves = 0;
        for (int i = 0; i < pl.ndirs; i++) waves += (pl.d[i].nchains + 1) / 2;
        const dim3 grid2((waves + 3) / 4, F);
        if (g.D < 128) hipLaunchKernelGGL((k_paths_tc<true>), grid2, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths_tc<false>), grid2, dim3(256), 0, st, g, pl);
        return;
    }
    dim3 grid((total + 3) / 4, F);
    if (g.D <= 128) {
        if (g.D < 128) hipLaunchKernelGGL((k_paths<2, true>), grid, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths<2, false>), grid, dim3(256), 0, st, g, pl);
    } else if (g.D <= 256) {
        if (g.D < 256) hipLaunchKernelGGL((k_paths<4, true>), grid, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths<4, false>), grid, dim3(256), 0, st, g, pl);
    } else {
        if (g.D < 512) hipLaunchKernelGGL((k_paths<8, true>), grid, dim3(256), 0, st, g, pl);
        else hipLaunchKernelGGL((k_paths<8, false>), grid, dim3(256), 0, st, g, pl);
    }
}

// ------------------------------------------------------------------------------------------
// The top-to-bottom direction fused with A.8 (WTA / uniqueness / subpixel).
//
// One workgroup per column chain, two roles:
//   wave 0 (producer) runs the serial recurrence of the chain (C loaded kSouthLAB blocks
//     ahead) and stages each row's L in LDS, kSouthRB rows per block, double-buffered;
//   waves 1..3 (consumers) each own 4 rows of a block: a pixel's D disparities sit on one 16-lane
//     DPP row (4 pixels per wave instruction, 16 B per lane per direction), the other P-1
//     directions' L are read from HBM (prefetched whole blocks ahead), the staged L is added
//     from LDS, and the winner-take-all runs on the saturated sums.
// A block is handed over by one barrier.  L of this direction is never written to HBM, so the
// pass moves 2 + 2(P-1) B/cell.  The uniqueness test needs only the smallest S[d] with
// |d - best| > 1 (both of OpenCV's rules are monotone in S[d]): a masked packed minimum.
// Each pixel's results -- the WTA disparity and (minS << 16 | bestDisp) for the right-view WTA --
// are staged in LDS and written out once per kStageBlocks blocks, so no global store or atomic
// sits in the consumers' vector-memory queue between a block's loads and their use (a per-block
// global atomic there made every block wait for its round trip).  Loads run past a chain's end
// into the buffers' kSouthPad rows of slack instead of being clamped.
// ------------------------------------------------------------------------------------------
// 1 producer + 3 consumer waves (256 threads): the 1152 column chains of a 1280x720 d=128 frame
// are resident in one pass.  2 and 4 consumer waves measured the same within noise.
#ifndef SDR_SOUTH_CONS
#define SDR_SOUTH_CONS 3
#endif
#ifndef SDR_SOUTH_LAB
#define SDR_SOUTH_LAB 2
#endif
constexpr int kSouthConsumers = SDR_SOUTH_CONS;
constexpr int kSouthRPW = 4;                           // rows per consumer wave and block (4 per pass;
                                                       // 8 rows x 2 consumers measured the same)
constexpr int kSouthRB = kSouthRPW * kSouthConsumers;  // rows per block
constexpr int kSouthLAB = SDR_SOUTH_LAB;       // producer lookahead in blocks (C0 -28 %, C2 -3 % vs 1)
constexpr int kSouthSPad = 4;                  // dword padding of the consumers' staged S rows
constexpr int kStageBlocks = 32;               // blocks per output staging window
constexpr int kStageRows = kStageBlocks * kSouthRB;
constexpr uint32_t kNoWrite = 0xfffffffeu;     // staged row outside this chain's output rows
constexpr uint32_t kRejected = 0xffffffffu;    // no disp2 candidate

// TC (two columns per workgroup, D <= 128, DPL = 2): the producer wave runs the chains of two
// adjacent columns of one direction entry, lanes 0-31 and 32-63 with four disparities each (the
// k_paths_tc step), and the consumers take both columns' pixels of a block (two passes).  The
// class path's 3WAY stripes at 640x360 are 4480 short chains of ~100 rows, each a workgroup whose
// producer's serial steps bound the pass; two per workgroup halves the workgroups to run.
template <int DPL, bool PAD, int NP, bool TC = false>
__global__ __launch_bounds__(64 * (1 + kSouthConsumers)) void k_south_wta(Geometry g0, PathLaunch pl,
                                                                           SouthWtaArgs a) {
    static_assert(!TC || DPL == 2, "two columns per workgroup: the D <= 128 layout");
    const Geometry g = frame_geom(g0, blockIdx.y);
    constexpr int K = DPL / 2;
    constexpr int NCOL = TC ? 2 : 1;   // columns per workgroup
    constexpr int PK = TC ? 2 : K;     // producer words per lane
    constexpr int RB = kSouthRB;
    constexpr int LAB = kSouthLAB;
    constexpr int LA = LAB * RB;  // producer lookahead in rows
    // ring of LA slots, unrolled by LA steps: a slot is reloaded (row k + LA) as soon as row k
    // is taken from it, so its register is static and never copied at the loop's back edge
    constexpr int NS = LAB;       // ring blocks per producer loop body
    constexpr int R = NS * RB;    // producer ring slots (rows) = LA
    static_assert(LA + RB <= kSouthPad, "load overrun must fit the buffers' row slack");
    constexpr int WDPL = DPL * 4;  // consumer: disparities per lane
    constexpr int WK = WDPL / 2;
    constexpr int DMAX = 64 * DPL;
    constexpr int LSTR = DMAX / 2 + 4;  // dwords per staged row (padded: rows of a wave's 4 pixels)
    // consumer prefetch distance in blocks (= ring slots) of the other directions' L
    // (two blocks while the ring fits 64 VGPRs; 1 block -- a ring of 56 VGPRs -- for 8 paths at D > 128)
#ifndef SDR_SOUTH_TC_PD
#define SDR_SOUTH_TC_PD 2
#endif
    constexpr int PD = TC ? SDR_SOUTH_TC_PD : NP * WK * kSouthRPW <= 128 ? 2 : 1;
    static_assert((PD + 1) * RB <= kSouthPad, "consumer load overrun must fit the row slack");
    __shared__ uint32_t sL[2][RB][NCOL][LSTR];
    // each consumer row's S staged for the subpixel neighbours and the uniqueness minimum (one
    // 16-B write per lane, three masking u16 writes, one read back); rows padded by 4 dwords so
    // the four lane groups' 16-B writes start on different banks
    __shared__ uint32_t sS[kSouthConsumers][4][DMAX / 2 + kSouthSPad];
    // per-row outputs, two windows of kStageRows rows
    __shared__ int16_t sRaw[2][NCOL][kStageRows];
    __shared__ uint32_t sKey[2][NCOL][kStageRows];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // role (0 = producer)
    const int cg = blockIdx.x;
    const int f = blockIdx.y;
    int di = 0, c0i = 0;
    bool hasB = false;
    if constexpr (TC) {
        // workgroups per direction entry: ceil(chains / 2)
        int w0 = 0;
        for (; di < pl.ndirs; di++) {
            const int nw = (pl.d[di].nchains + 1) / 2;
            if (cg < w0 + nw) break;
            w0 += nw;
        }
        if (di >= pl.ndirs) return;
        c0i = 2 * (cg - w0);
        hasB = c0i + 1 < pl.d[di].nchains;
    } else {
        while (cg >= pl.prefix[di + 1]) di++;
        c0i = cg - pl.prefix[di];
    }
    const PathDir pd = pl.d[di];
    const Chain ch = make_chain(g, pd, c0i);  // TC: the second column is ch.x0 + 1, same rows
    if (ch.len <= 0) return;  // whole workgroup
    const int D = g.D, W1 = g.W1;
    const size_t fofs = (size_t)f * pl.cs_fstride;
    const int last = ch.len - 1;
    const int nblk = (ch.len + RB - 1) / RB;

    if (wv == 0) {
        // ---------------- producer: the recurrence, L rows to LDS ----------------
        __builtin_amdgcn_s_setprio(2);
        // TC: half h of the wave runs column x0 + h (its lanes' offsets one pixel further)
        const int half = TC ? lane >> 5 : 0, hl = TC ? lane & 31 : lane;
        constexpr int PDPL = 2 * PK;  // producer disparities per lane
        const bool active = (!TC || half == 0 || hasB) && (!PAD || hl * PDPL < D);
        const uint32_t lofs = (uint32_t)((PAD ? min(hl, D / PDPL - 1) : hl) * PDPL * 2) + (uint32_t)(half * D * 2);
        const ptrdiff_t rowb = (ptrdiff_t)W1 * D * 2;
        // 3WAY stripes: a chain starting at aux_row0 reads its first aux_rows (< LA) cost rows
        // from the stripe-local (row-major) buffer; every later row comes from C
        const int naux = pd.Caux ? pd.aux_rows : 0;
        const char* abase = pd.Caux ? (const char*)(pd.Caux + (size_t)f * pl.aux_fstride + (size_t)ch.x0 * D)
                                    : (const char*)pl.C;
        const char* c0 = (const char*)(pl.C + fofs + ((size_t)ch.y0 * W1 + ch.x0) * D);
        // a resource per load: the compiler then bunches the loads into one burst per block
        // (measured faster than one resource per chain with an SGPR row offset here).  Rows past
        // the chain's end re-read its last row (an L2 hit) instead of the buffer's slack rows:
        // the class path's 3WAY stripes are ~100 rows, and a lookahead of LA rows past each
        // stripe's end was a quarter of the pass's HBM reads there
        auto crow = [&](int k) { return c0 + (ptrdiff_t)min(k, last) * rowb; };
        Regs<PK> cring[R];
#pragma unroll
        for (int j = 0; j < LA; j++)
            cring[j] = load_buf<PK>(rsrc_at(j < naux ? abase + (ptrdiff_t)j * rowb : crow(j)), lofs);
        Regs<PK> Lp;
#pragma unroll
        for (int i = 0; i < PK; i++) Lp.r[i] = active ? 0u : kMaxPair;
        const uint32_t P1x2 = splat16(g.P1), P2x2 = splat16(g.P2);
        uint32_t delta2 = P2x2;
        uint32_t upr = kMaxPair, dnr = kMaxPair;  // see path_step
        // block bb (= slot ic of the ring): RB recurrence steps into LDS slot bb & 1, then hand over
        auto block = [&](const int bb, auto ic) __attribute__((always_inline)) {
            uint32_t* dst = &sL[bb & 1][0][half][hl * PK];
            auto st = [&](const int, auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value + decltype(ic)::value * RB;  // ring slot = k % R
                const Regs<PK> c = cring[j];
                cring[(j + LA) % R] = load_buf<PK, kLoadNT>(rsrc_at(crow(bb * RB + (j % RB) + LA)), lofs);
                Regs<PK> L;
                if constexpr (TC) L = path_step_tc<PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr, lane);
                else L = path_step<K, PAD>(c, Lp, delta2, P1x2, P2x2, active, upr, dnr);
#pragma unroll
                for (int i = 0; i < PK; i++) dst[(j % RB) * NCOL * LSTR + i] = L.r[i];
            };
            unroll_rows(st, bb * RB, std::make_integer_sequence<int, RB>{});
            __syncthreads();
        };
        int b = 0;
        for (; b + NS <= nblk; b += NS) unroll_rows(block, b, std::make_integer_sequence<int, NS>{});
        unroll_rows_tail(block, b, nblk - 1, std::make_integer_sequence<int, NS - 1>{});
        __syncthreads();  // the consumers' last block
        return;
    }

    // ---------------- consumers: the other directions + WTA, RPW rows per wave ----------------
    // passes of 4 pixels (one per 16-lane group): the wave's RPW rows of each column
    constexpr int RPASS = kSouthRPW / 4;
    constexpr int NPASS = NCOL * RPASS;
    const int gl = lane & 15, grp = lane >> 4;
    // D > 256: 32 disparities per lane, so the last active lane may hold fewer than 32 (D is a
    // multiple of 16): it reads its own offset and masks the pairs past D (see ssum)
    const bool wactive = !PAD || gl * WDPL < D;
    const int wd0 = (PAD ? min(gl, (D - 1) / WDPL) : gl) * WDPL;
    // row blk*RB + r of the chain: wave-uniform block base + lane byte offset; the NP
    // directions of a pixel are one contiguous record (q*D*2 folds into the instruction offset)
    const ptrdiff_t bstepb = (ptrdiff_t)RB * W1 * pl.l_pix * 2;
    int rr[NPASS];          // this lane group's row within a block, per pass
    uint32_t lofs[NPASS];
#pragma unroll
    for (int ps = 0; ps < NPASS; ps++) {
        const int col = ps / RPASS;  // TC: passes of the second column are one pixel further on
        rr[ps] = (wv - 1) * kSouthRPW + (ps % RPASS) * 4 + grp;
        lofs[ps] = (uint32_t)((((size_t)rr[ps] * W1 + col) * pl.l_pix + wd0) * 2);
    }
    const char* lbase = (const char*)(a.L + (size_t)f * pl.l_fstride + ((size_t)ch.y0 * W1 + ch.x0) * pl.l_pix);
    // blocks past the chain's last one re-read that block (L2 hits), not the buffers' slack
    // a block whose rows all lie before the chain's first output row (a 3WAY stripe's overlap
    // rows: recurred through by the producer, never output) reads its records from an empty
    // resource -- zeros, no memory traffic, no branch (its sums are never output)
    auto oload = [&](int q, int blk, int ps) __attribute__((always_inline)) {
        const bool need = blk * RB + RB > ch.kwrite;
        const Rsrc r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<char*>(lbase + (ptrdiff_t)min(blk, nblk - 1) * bstepb), (short)0, need ? 0x7fffffff : 0,
            0x00020000);
        return load_buf<WK, kLoadNT>(r, lofs[ps] + (uint32_t)(q * D * 2));
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
    uint32_t* d2 = a.d2 ? a.d2 + (size_t)f * a.disp_fstride : nullptr;
    const int x2base = x + g.minX1 - g.minD;  // the right-view column of disparity index 0

    // window w of staged outputs (rows [w*kStageRows, ...)) to HBM, by the consumer lanes
    auto flush = [&](int w) __attribute__((always_inline)) {
        const int r0 = w * kStageRows;
        const int n = min(kStageRows, ch.len - r0);
#pragma unroll
        for (int col = 0; col < NCOL; col++) {
            if (col > 0 && !hasB) break;  // uniform
            for (int i = (wv - 1) * 64 + lane; i < n; i += 64 * kSouthConsumers) {
                const uint32_t key = sKey[w & 1][col][i];
                if (key == kNoWrite) continue;
                const size_t y = (size_t)(ch.y0 + r0 + i);
                raw[y * g.W + col] = sRaw[w & 1][col][i];
                if (d2 && key < kNoWrite) {
                    // A.8's disp2 candidate of this pixel (no return value: a fire-and-forget atomic)
                    const int x2 = x2base + col - (int)(key & 0xffff);
                    if (x2 >= 0 && x2 < g.W)
                        atomicMin(&d2[y * g.W + x2], (key & 0xffff0000u) | (uint32_t)(0xffff - (x + col)));
                }
            }
        }
    };

    // one 4-row pass of block b: S of row k = b*RB + r, the WTA, its outputs staged in LDS
    // S = sat(sum of the P path costs) of row r of block b, the fused direction's L from LDS
    auto ssum = [&](const int b, const int r, const int col, const Regs<WK> (&o)[NP]) __attribute__((always_inline)) {
        const uint32_t* ls = &sL[b & 1][r][col][wd0 / 2];
        Regs<WK> St;
#pragma unroll
        for (int i = 0; i < WK; i++) {
            uint32_t acc = 0;
#pragma unroll
            for (int p = 0; p <= NP; p++) {
                const uint32_t v = p == kSouthIdx ? ls[i] : o[p < kSouthIdx ? p : p - 1].r[i];
                acc = p == 0 ? v : pk_add_sat(acc, v);
            }
            if constexpr (PAD && DPL == 8) acc = wd0 + 2 * i < D ? acc : kMaxPair;  // past D: never a minimum
            St.r[i] = acc;
        }
        return St;
    };
    auto rows = [&](const int b, const int r, const int col, const Regs<WK>& St) __attribute__((always_inline)) {
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
        uint32_t* srow = &sS[wv - 1][grp][0];
#pragma unroll
        for (int i = 0; i < WK; i++) ((uint32_t __attribute__((may_alias))*)srow)[gl * WK + i] = St.r[i];
        key = row16_min_u32(wactive ? key : 0xffffffffu);
        const int minS = (int)(key >> 16) - 32768;
        const int best = (int)(key & 0xffff);
        const int dm = max(best - 1, 0), dp = min(best + 1, D - 1);
        // uniqueness: min of S[d] over |d - best| > 1 (0 <= S <= 32767: 0x7fff masks a half);
        // the halfword accesses alias the row's 32-bit words: may_alias keeps their order
        typedef int16_t __attribute__((may_alias)) s16a;
        typedef uint32_t __attribute__((may_alias)) u32a;
        s16a* s16 = (s16a*)srow;
        const int Sm = s16[dm];
        const int Sp = s16[dp];
        s16[dm] = 0x7fff;
        s16[best] = 0x7fff;
        s16[dp] = 0x7fff;
        uint32_t m2 = kMaxPair;
#pragma unroll
        for (int i = 0; i < WK; i++) m2 = pk_min(m2, ((u32a*)srow)[gl * WK + i]);
        m2 = wactive ? m2 : kMaxPair;
        m2 = pk_min(m2, funnel16(m2, m2));
        m2 = row16_min_u32(m2);
        const int min2 = (int)(m2 & 0x7fff);
        // SIMD rule: S[d] < (short)(thresh + 1), thresh = (100*minS)/(100-u); scalar: S*(100-u) < 100*minS
        const int thr16 = (int)(short)((int)((double)(100 * minS) * inv100u) + 1);
        const bool reject = check_uniq && (uniq_simd ? (min2 < thr16) : (min2 * lhs_scale < minS * 100));
        if (gl == 0 && k <= last) {
            int out = invalid;
            uint32_t okey = kNoWrite;
            if (rowok) {
                okey = kRejected;
                // every S saturated: OpenCV's first-minimum scan (strict '<' from MAX_COST) keeps
                // bestDisp = -1, whose value (-1 + minD) * 16 is INVALID and whose disp2
                // candidate (cost MAX_COST) never replaces the initial one
                if (!reject && minS < kMaxCost) {
                    // subpixel: d*16 + ((S[d-1]-S[d+1])*16 + den) / (2*den), C truncating division
                    const int den = max(Sm + Sp - 2 * minS, 1);
                    const int qq = div_trunc_small((Sm - Sp) * 16 + den, 2 * den);
                    out = best * 16 + (((0 < best) & (best < D - 1)) ? qq : 0) + g.minD * 16;
                    okey = ((uint32_t)minS << 16) | (uint32_t)best;
                }
            }
            sRaw[(k / kStageRows) & 1][col][k % kStageRows] = (int16_t)out;
            sKey[(k / kStageRows) & 1][col][k % kStageRows] = okey;
        }
    };

    // ring of PD blocks: slot s holds block b (b = s mod PD) until its sum is taken, then the
    // load of block b + PD goes into the same registers, so each block's loads have PD block
    // periods to land (the loop is unrolled by PD: static slots, no copies at the back edge);
    // unconditional: blocks past the chain's end re-read its last block (oload clamps)
    Regs<WK> oring[PD][NPASS][NP];
#pragma unroll
    for (int s = 0; s < PD; s++)
#pragma unroll
        for (int ps = 0; ps < NPASS; ps++)
#pragma unroll
            for (int q = 0; q < NP; q++) oring[s][ps][q] = oload(q, s, ps);

    auto consume_sync = [&](const int b, auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
#pragma unroll
        for (int ps = 0; ps < NPASS; ps++) {
            const Regs<WK> St = ssum(b, rr[ps], ps / RPASS, oring[s][ps]);
#pragma unroll
            for (int q = 0; q < NP; q++) oring[s][ps][q] = oload(q, b + PD, ps);
            if (ps < RPASS || hasB) rows(b, rr[ps], ps / RPASS, St);  // TC: a second column exists
        }
        __syncthreads();
        // the window this block completes (or the chain's last, partial one) goes out now that
        // every consumer's rows of it are staged; its buffer is rewritten kStageBlocks blocks on
        if (b % kStageBlocks == kStageBlocks - 1 || b == nblk - 1) flush(b / kStageBlocks);
    };
    __syncthreads();  // block 0 staged
    int b = 0;
    for (; b + PD <= nblk; b += PD) unroll_rows(consume_sync, b, std::make_integer_sequence<int, PD>{});
    unroll_rows_tail(consume_sync, b, nblk - 1, std::make_integer_sequence<int, PD>{});
}

// A.9 materialised (the debug stage of the LR-checked map; the pipeline's median computes it
// per tile instead)
__global__ __launch_bounds__(256) void k_lr_apply(Geometry g0, const int16_t* __restrict__ raw,
                                                  const uint32_t* __restrict__ d2,
                                                  int16_t* __restrict__ out, size_t fstride, int d12) {
    const Geometry g = frame_geom(g0, blockIdx.y);
    const int y = blockIdx.x, f = blockIdx.y;
    const size_t fo = (size_t)f * fstride;
    for (int x = threadIdx.x; x < g.W; x += 256)
        out[fo + (size_t)y * g.W + x] = (int16_t)lr_at(g, raw + fo, d2 + fo, x, y, d12);
}

template <int DPL, bool PAD>
static void launch_south_np(const Geometry& g, const PathLaunch& pl, const SouthWtaArgs& a, int F,
                            hipStream_t st) {
    dim3 grid(pl.prefix[pl.ndirs], F);
    dim3 block(64 * (1 + kSouthConsumers));
    if constexpr (DPL == 2) {
        // two columns per workgroup when the chains far outnumber what the chip holds at once
        // (short, latency-bound chains: the class path's 3WAY stripes), up to 5 paths
        const int cus = device_cus();
        if (a.npaths <= 5 && (long)pl.prefix[pl.ndirs] * F > 8L * cus) {
            int wgs = 0;
            for (int i = 0; i < pl.ndirs; i++) wgs += (pl.d[i].nchains + 1) / 2;
            const dim3 grid2(wgs, F);
            switch (a.npaths) {
            case 3: hipLaunchKernelGGL((k_south_wta<2, PAD, 2, true>), grid2, block, 0, st, g, pl, a); return;
            case 4: hipLaunchKernelGGL((k_south_wta<2, PAD, 3, true>), grid2, block, 0, st, g, pl, a); return;
            default: hipLaunchKernelGGL((k_south_wta<2, PAD, 4, true>), grid2, block, 0, st, g, pl, a); return;
            }
        }
    }
    switch (a.npaths) {
    case 3: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 2>), grid, block, 0, st, g, pl, a); break;
    case 4: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 3>), grid, block, 0, st, g, pl, a); break;
    case 5: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 4>), grid, block, 0, st, g, pl, a); break;
    default: hipLaunchKernelGGL((k_south_wta<DPL, PAD, 7>), grid, block, 0, st, g, pl, a); break;
    }
}

void launch_south_wta(const Geometry& g, const PathLaunch& pl, const SouthWtaArgs& a, int F,
                      hipStream_t st) {
    if (pl.prefix[pl.ndirs] <= 0) return;
    if (g.D <= 128) {
        if (g.D < 128) launch_south_np<2, true>(g, pl, a, F, st);
        else launch_south_np<2, false>(g, pl, a, F, st);
    } else if (g.D <= 256) {
        if (g.D < 256) launch_south_np<4, true>(g, pl, a, F, st);
        else launch_south_np<4, false>(g, pl, a, F, st);
    } else {
        if (g.D < 512) launch_south_np<8, true>(g, pl, a, F, st);
        else launch_south_np<8, false>(g, pl, a, F, st);
    }
}

void launch_lr_apply(const Geometry& g, const int16_t* raw, const uint32_t* d2, int16_t* out,
                     size_t fstride, int disp12MaxDiff, int F, hipStream_t st) {
    hipLaunchKernelGGL(k_lr_apply, dim3(g.H, F), dim3(256), 0, st, g, raw, d2, out, fstride, disp12MaxDiff);
}

}  // namespace sdr
