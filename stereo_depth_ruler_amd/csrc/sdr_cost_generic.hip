// sdr_cost_generic.hip -- the A.2/A.3 cost volume for block sizes past k_cost's register ring
// (blockSize 13..17: SH2 = SW2 > 5; larger windows always leave the int16 cost domain, which the
// engine refuses).  Same arithmetic as k_cost (sdr_cost_kernel.hpp), in two passes through a
// scratch volume instead of one:
//   k_hsum_generic  H1(r, x, d) = sum_{|k|<=SW2} BT(r, clamp(x+k, 0, W1-1), d) for every physical
//                   row r: a thread owns one disparity pair and slides along a strip of columns
//                   (one pixel cost in, one out per step: two BT evaluations per output)
//   k_vsum_generic  C(y, x, d) = P2 + sum_{|j|<=SH2} H1(clamp(t(y)+j, s0, H-1), x, d), t(y) =
//                   min(y, ylim), MODE_HH's frozen bottom rows P2; a thread owns one (column,
//                   disparity pair) and slides down a chunk of rows (two loads per output)
// Sums are packed int16 with wrap-around, as in k_cost and OpenCV's CostType arithmetic.
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

namespace sdr {

namespace {

constexpr int kHsumStrip = 64;  // columns per thread in k_hsum_generic
constexpr int kVsumChunk = 32;  // output rows per thread in k_vsum_generic

__device__ __forceinline__ uint32_t bt_pair(uint32_t u, uint32_t u0, uint32_t u1, uint32_t v,
                                            uint32_t v0, uint32_t v1) {
    const uint32_t c0 = pk_max_u(pk_sub_usat(u, v1), pk_sub_usat(v0, u));
    const uint32_t c1 = pk_max_u(pk_sub_usat(v, u1), pk_sub_usat(u0, v));
    return pk_min_u(c0, c1);
}
__device__ __forceinline__ uint32_t splat_lo(uint32_t w) { return (w & 0xffffu) * 0x10001u; }
__device__ __forceinline__ uint32_t splat_hi(uint32_t w) { return (w >> 16) * 0x10001u; }

// the packed pixel cost of disparities (2qp, 2qp+1) at matched column xc of row r (both in range)
template <int CN>
__device__ __forceinline__ uint32_t pixel_cost(const Geometry& g, const Planes& pl, int f, int r, int xc, int qp) {
    const uint32_t* Lw = pl.L + (size_t)f * pl.fstrideL + ((size_t)r * g.W + g.minX1 + xc) * 3 * CN;
    const size_t plane = (size_t)g.H * g.W;
    const int xr = g.minX1 + xc - g.minD - 2 * qp;  // the right pixel of d = 2qp (d + 1: xr - 1)
    const uint64_t* Rw = pl.R + (size_t)f * pl.fstrideR + (size_t)r * g.W + xr;
    uint32_t pc = 0;
#pragma unroll
    for (int ch = 0; ch < CN; ch++) {
        const uint32_t w0 = Lw[3 * ch], w1 = Lw[3 * ch + 1], w2 = Lw[3 * ch + 2];
        const uint64_t r0 = Rw[3 * ch * plane], r1 = Rw[(3 * ch + 1) * plane], r2 = Rw[(3 * ch + 2) * plane];
        const uint32_t bs = bt_pair(splat_lo(w0), splat_hi(w0), splat_lo(w1), (uint32_t)r0, (uint32_t)(r0 >> 32),
                                    (uint32_t)r1);
        const uint32_t br = bt_pair(splat_hi(w1), splat_lo(w2), splat_hi(w2), (uint32_t)(r1 >> 32), (uint32_t)r2,
                                    (uint32_t)(r2 >> 32));
        pc = pk_add(pc, pk_add(bs, pk_shr2_u(br)));
    }
    return pc;
}

template <int CN>
__global__ __launch_bounds__(256) void k_hsum_generic(Geometry g0, Planes pl, uint32_t* __restrict__ h1) {
    const int f = blockIdx.z, r = blockIdx.y;
    const Geometry g = frame_geom(g0, f);
    const int npair = g.D / 2, W1 = g.W1, SW2 = g.SW2;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int qp = t % npair, strip = t / npair;
    const int x0 = strip * kHsumStrip;
    if (x0 >= W1) return;
    const int x1 = min(x0 + kHsumStrip, W1);
    auto pc = [&](int x) { return pixel_cost<CN>(g, pl, f, r, min(max(x, 0), W1 - 1), qp); };
    uint32_t hs = 0;
    for (int k = -SW2; k <= SW2; k++) hs = pk_add(hs, pc(x0 + k));
    uint32_t* out = h1 + (((size_t)f * g.H + r) * W1) * (g.D / 2) + qp;
    for (int x = x0; x < x1; x++) {
        out[(size_t)x * npair] = hs;
        hs = pk_sub(pk_add(hs, pc(x + 1 + SW2)), pc(x - SW2));
    }
}

// grid.y: the main rows in chunks of kVsumChunk, then one band per 3WAY stripe start (a.aux)
__global__ __launch_bounds__(256) void k_vsum_generic(Geometry g0, CostArgs a, const uint32_t* __restrict__ h1,
                                                      int nmain) {
    const int f = blockIdx.z;
    const Geometry g = frame_geom(g0, f);
    const int npair = g.D / 2, W1 = g.W1, H = g.H, SH2 = g.SH2;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= W1 * npair) return;
    const int x = t / npair, qp = t % npair;
    int16_t* outb;
    int row0, ty0, ty1, s0, ylim, hh;
    if ((int)blockIdx.y < nmain) {
        outb = a.out + (size_t)f * a.out_fstride;
        row0 = a.out_row0;
        ty0 = a.row_begin + blockIdx.y * kVsumChunk;
        ty1 = min(ty0 + kVsumChunk, a.row_end);
        s0 = a.s0;
        ylim = a.ylim;
        hh = a.hh_bottom;
    } else {
        const CostAux& b = a.aux[blockIdx.y - nmain];
        outb = b.out + (size_t)f * a.aux_fstride;
        row0 = b.row0;
        ty0 = b.row0;
        ty1 = b.row0 + b.rows;
        s0 = b.s0;
        ylim = b.ylim;
        hh = 0;
    }
    if (ty0 >= ty1) return;
    const uint32_t P2x2 = splat16(g.P2);
    const uint32_t* col = h1 + ((size_t)f * H * W1 + x) * npair + qp;
    const size_t rstride = (size_t)W1 * npair;
    auto hv = [&](int q) { return col[(size_t)min(max(q, s0), H - 1) * rstride]; };
    // MODE_HH: rows y > 0 with y + SH2 >= H keep the initial P2
    const int yl = hh ? max(ty0, min(ty1, max(1, H - SH2))) : ty1;
    uint32_t* out = (uint32_t*)(outb + ((size_t)(ty0 - row0) * W1 + x) * g.D) + qp;
    const size_t ostride = (size_t)W1 * npair;
    int tcur = min(ty0, ylim);
    uint32_t s = 0;
    for (int j = -SH2; j <= SH2; j++) s = pk_add(s, hv(tcur + j));
    for (int y = ty0; y < ty1; y++) {
        const int ty = min(y, ylim);
        while (tcur < ty) {  // the window moves down one row (t stops at ylim)
            s = pk_sub(pk_add(s, hv(tcur + 1 + SH2)), hv(tcur - SH2));
            tcur++;
        }
        out[(size_t)(y - ty0) * ostride] = y < yl ? pk_add(s, P2x2) : P2x2;
    }
}

}  // namespace

size_t cost_generic_scratch_bytes(const Geometry& g, int F) { return (size_t)F * g.H * g.W1 * g.D * 2; }

void launch_cost_generic(const Geometry& g, const CostArgs& a, int F, uint32_t* h1, hipStream_t st) {
    const int npair = g.D / 2;
    const int strips = (g.W1 + kHsumStrip - 1) / kHsumStrip;
    const dim3 gh((unsigned)((strips * npair + 255) / 256), g.H, F);
    if (a.pl.cn == 3) hipLaunchKernelGGL(k_hsum_generic<3>, gh, dim3(256), 0, st, g, a.pl, h1);
    else hipLaunchKernelGGL(k_hsum_generic<1>, gh, dim3(256), 0, st, g, a.pl, h1);
    const int rows = max(a.row_end - a.row_begin, 0);
    const int nmain = (rows + kVsumChunk - 1) / kVsumChunk;
    if (nmain + a.naux == 0) return;
    const dim3 gv((unsigned)((g.W1 * npair + 255) / 256), nmain + a.naux, F);
    hipLaunchKernelGGL(k_vsum_generic, gv, dim3(256), 0, st, g, a, (const uint32_t*)h1, nmain);
}

}  // namespace sdr
