// sdr_cost.hip -- A.1 prefilter + BT operands and A.2/A.3 cost volume kernels (CDNA4).
//
//   L pack    u32 [F][H][W][3cn]  the left image's BT operands at x as 16-bit halves, per channel:
//                                 {sob | sob_lo<<16} {sob_hi | raw<<16} {raw_lo | raw_hi<<16}
//   planes R  u64 [F][3cn][H][W]  int16 PAIRS of the right image's operands: q(x) | q(x-1) << 16, so
//                                 a lane holding disparities (d, d+1) reads one word for xr = x-d, x-d-1
//   (cn = 1 for gray input, 3 for CV_8UC3: calcPixelCostBT sums the channels' costs)
//   C         s16 [F][H][W1][D] P2 + blockSize^2 box sum of the BT pixel cost
//
// Cost kernel: lanes = disparity pairs (as in the path kernels).  A block owns BCOLS output
// columns and the BCOLS + 2*SW2 pixel-cost columns their windows need; each pixel cost is
// computed once (the four waves own interleaved columns), summed vertically in registers (a ring
// of the last NR rows, static slots by unrolling the row loop by the window height), and the
// column sums are exchanged through LDS for the horizontal sums.  A pixel's left operands are
// the same for all lanes: they are read from LDS as 16-byte broadcasts (one per column and
// channel) and reach the packed ops through op_sel half selection.  The kernel template itself is
// in sdr_cost_kernel.hpp (gray instantiations here, colour ones in sdr_cost3.hip).  The right image's pair planes are staged per row (split into even/odd-x
// halves so that lane p reading entry x - 2p is bank-conflict free), fetched two rows ahead
// through registers and double-buffered in LDS.  One barrier per row.
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
// channels = tab[0] = ftzero; rows replicate) + half-sample envelopes (calcPixelCostBT), per
// channel of an image with pl.cn (1 or 3) interleaved channels: channel c's operands go to the
// c-th operand set (R planes 3c..3c+2, L words 3c..3c+2 of a pixel).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prefilter(const uint8_t* __restrict__ Limg,
                                                   const uint8_t* __restrict__ Rimg, size_t stride,
                                                   size_t fstride, int W, int H, int ftzero,
                                                   Planes pl, int split, uint32_t* d2fill) {
    extern __shared__ uint64_t q6[];  // [W] 6 bytes per pixel, then the 3 input rows [3][W*cn] bytes
    const int y = blockIdx.x, img = blockIdx.y, f = blockIdx.z;
    const int cn = pl.cn, WB = W * cn;
    // paired matchers: frame f >= split is frame f - split of the pair with L and R swapped
    const bool swap = f >= split;
    const uint8_t* base = ((img != 0) != swap ? Rimg : Limg) + (size_t)(swap ? f - split : f) * fstride;
    {
        // the row and its neighbours (replicated at the borders) staged in LDS: one coalesced
        // byte load per pixel and row instead of eleven scattered ones
        const uint8_t* gr = base + (size_t)y * stride;
        const uint8_t* gn = y > 0 ? gr - stride : gr;
        const uint8_t* gs = y < H - 1 ? gr + stride : gr;
        uint8_t* rows = (uint8_t*)(q6 + W);
        if (((WB | (int)stride | (int)fstride | (int)(uintptr_t)base) & 3) == 0) {
            // dword-aligned rows (the class path's half-size images, typical frames): four bytes a
            // lane, the three rows' loads issued together (the LDS rows start 8-byte aligned and
            // are WB apart, a multiple of 4)
            uint32_t* rw = (uint32_t*)rows;
            const int nw = WB >> 2;
            for (int x = threadIdx.x; x < nw; x += blockDim.x) {
                const uint32_t a = ((const uint32_t*)gn)[x], b = ((const uint32_t*)gr)[x], c = ((const uint32_t*)gs)[x];
                rw[x] = a;
                rw[nw + x] = b;
                rw[2 * nw + x] = c;
            }
        } else {
            for (int x = threadIdx.x; x < WB; x += blockDim.x) {
                rows[x] = gn[x];
                rows[WB + x] = gr[x];
                rows[2 * WB + x] = gs[x];
            }
        }
        __syncthreads();
    }
    if (d2fill && img == 0) {
        // the right-view keys of this row start empty (k_south_wta's atomics fold into them)
        uint32_t* d2 = d2fill + ((size_t)f * H + y) * W;
        for (int x = threadIdx.x; x < W; x += blockDim.x) d2[x] = kD2None;
    }
    const uint8_t* n = (const uint8_t*)(q6 + W);
    const uint8_t* r = n + WB;
    const uint8_t* s = r + WB;
    const size_t plane = (size_t)H * W;
    for (int ch = 0; ch < cn; ch++) {
        for (int x = threadIdx.x; x < W; x += blockDim.x) {
            int sv[3], rv[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                int xx = x + k - 1;
                // OpenCV's clip table is uchar: past preFilterCap 127 its entries (and the border's
                // tab[0] = ftzero past 255) wrap mod 256
                if (xx <= 0 || xx >= W - 1) {
                    sv[k] = ftzero & 0xff;
                    rv[k] = ftzero & 0xff;
                } else {
                    const int a = (xx + 1) * cn + ch, b = (xx - 1) * cn + ch;
                    int gr = 2 * (r[a] - r[b]) + n[a] - n[b] + s[a] - s[b];
                    gr = gr < -ftzero ? -ftzero : (gr > ftzero ? ftzero : gr);
                    sv[k] = (gr + ftzero) & 0xff;
                    rv[k] = r[xx * cn + ch];
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
        for (int x = threadIdx.x; x < W; x += blockDim.x) {
            const uint64_t a = q6[x];
            const uint64_t b = q6[x > 0 ? x - 1 : 0];
            uint32_t w[6];
#pragma unroll
            for (int c = 0; c < 6; c++) {
                const uint32_t va = (uint32_t)(a >> (8 * c)) & 0xff, vb = (uint32_t)(b >> (8 * c)) & 0xff;
                w[c] = img ? (va | (vb << 16)) : va * 0x10001u;
            }
            if (img) {
                uint64_t* dst = pl.R + (size_t)f * pl.fstrideR + 3 * ch * plane + (size_t)y * W + x;
                dst[0] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
                dst[plane] = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
                dst[2 * plane] = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
            } else {
                // one 12-byte store per pixel and channel (gray: a wave writes 768 contiguous bytes)
                typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
                const u32x3 v = {(w[0] & 0xffffu) | (w[1] << 16), (w[2] & 0xffffu) | (w[3] << 16),
                                 (w[4] & 0xffffu) | (w[5] << 16)};
                *(u32x3*)(pl.L + (size_t)f * pl.fstrideL + ((size_t)y * W + x) * 3 * cn + 3 * ch) = v;
            }
        }
        if (ch + 1 < cn) __syncthreads();  // q6 is rewritten by the next channel
    }
}

void launch_prefilter(const uint8_t* L, const uint8_t* R, size_t stride, size_t fstride, int W,
                      int H, int F, int ftzero, const Planes& pl, hipStream_t st, int split,
                      uint32_t* d2fill) {
    hipLaunchKernelGGL(k_prefilter, dim3(H, 2, F), dim3(256), (size_t)W * (8 + 3 * pl.cn), st, L, R,
                       stride, fstride, W, H, ftzero, pl, split, d2fill);
}

}  // namespace sdr

#include "sdr_cost_kernel.hpp"

namespace sdr {

// one output row of the widest column-block span (racing garbage from every block)
size_t cost_sink_bytes(const Geometry& g) { return (size_t)(g.W1 + 64) * g.D * 2; }

// SH2 <= 5 and D <= 256: k_cost (one pass, register ring); otherwise launch_cost_generic
bool cost_supported(const Geometry& g) { return g.SH2 == g.SW2 && g.D <= 512; }

void launch_cost(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    if (a.row_end <= a.row_begin && a.naux == 0) return;
    if (a.pl.cn == 3) return launch_cost_cn3(g, a, F, st);
    const int NR = 2 * g.SH2 + 1;
    const bool k2 = g.D > 128;
#define SDR_COST(NRV)                                                 \
    case NRV:                                                         \
        if (k2) launch_cost_t<NRV, 2, 1>(g, a, F, st);                \
        else launch_cost_t<NRV, 1, 1>(g, a, F, st);                   \
        break;
    switch (NR) {
        SDR_COST(1) SDR_COST(3) SDR_COST(5) SDR_COST(7) SDR_COST(9) SDR_COST(11)
        default: break;
    }
#undef SDR_COST
}

}  // namespace sdr
