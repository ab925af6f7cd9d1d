// Read-bandwidth probe for k_south_wta's access pattern (not product code): 1152 column chains,
// each reading its 1 KB record of every row of a [H][W1][1 KB] volume, vs one linear stream of the
// same bytes.  usage: read_pattern  (prints GB/s of each)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one WG per chain; wave w reads rows w, w+4, ...: 64 lanes x 16 B = the row's 1 KB record
template <int UNR>
__global__ __launch_bounds__(256) void k_chain(const u32x4* __restrict__ v, int H, int W1, unsigned* out) {
    const int x = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t rowv = (size_t)W1 * 64;  // u32x4 per row
    const u32x4* p = v + (size_t)x * 64 + lane;
    unsigned acc = 0;
    for (int y0 = w; y0 < H; y0 += 4 * UNR) {
        u32x4 t[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) {
            const int y = min(y0 + 4 * u, H - 1);
            t[u] = p[(size_t)y * rowv];
        }
#pragma unroll
        for (int u = 0; u < UNR; u++) acc += t[u].x ^ t[u].y ^ t[u].z ^ t[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// k_south_wta's consumer pattern: 3 waves, 12-row blocks, wave c owns rows 4c..4c+3 of a block;
// ROWMAJOR=false: instruction q reads direction q (256 B) of the 4 rows (lane group g = row g);
// ROWMAJOR=true: instruction r reads row r's whole 1 KB record
template <bool ROWMAJOR>
__global__ __launch_bounds__(192) void k_south_like(const u32x4* __restrict__ v, int H, int W1, unsigned* out) {
    const int x = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t rowv = (size_t)W1 * 64;
    const u32x4* p = v + (size_t)x * 64;
    unsigned acc = 0;
    for (int b = 0; b < (H + 11) / 12; b++) {
        u32x4 t[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int y, e;
            if (ROWMAJOR) { y = b * 12 + 4 * w + q; e = lane; }
            else { y = b * 12 + 4 * w + (lane >> 4); e = q * 16 + (lane & 15); }
            y = min(y, H - 1);
            t[q] = p[(size_t)y * rowv + e];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) acc += t[q].x ^ t[q].y ^ t[q].z ^ t[q].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// the same + a producer wave streaming its 256 B row of a second [H][W1][256 B] volume (C)
template <int LA>
__global__ __launch_bounds__(256) void k_south_like_c(const u32x4* __restrict__ v, const unsigned* __restrict__ c,
                                                      int H, int W1, unsigned* out) {
    const int x = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned acc = 0;
    if (w == 3) {
        const unsigned* p = c + (size_t)x * 64 + lane;
        const size_t rowc = (size_t)W1 * 64;
        unsigned ring[LA];
#pragma unroll
        for (int j = 0; j < LA; j++) ring[j] = p[(size_t)j * rowc];
        for (int y0 = 0; y0 < H; y0 += LA) {
#pragma unroll
            for (int j = 0; j < LA; j++) {
                acc = (acc ^ ring[j]) * 3u + 1u;  // a serial dependency like the recurrence
                ring[j] = p[(size_t)min(y0 + j + LA, H - 1) * rowc];
            }
        }
    } else {
        const size_t rowv = (size_t)W1 * 64;
        const u32x4* p = v + (size_t)x * 64;
        for (int b = 0; b < (H + 11) / 12; b++) {
            u32x4 t[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int y = min(b * 12 + 4 * w + (lane >> 4), H - 1);
                t[q] = p[(size_t)y * rowv + q * 16 + (lane & 15)];
            }
#pragma unroll
            for (int q = 0; q < 4; q++) acc += t[q].x ^ t[q].y ^ t[q].z ^ t[q].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// linear: grid-stride over the volume
template <int UNR>
__global__ __launch_bounds__(256) void k_linear(const u32x4* __restrict__ v, size_t n, unsigned* out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = (size_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * UNR) {
        u32x4 t[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) {
            size_t i = i0 + u * stride;
            t[u] = v[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < UNR; u++) acc += t[u].x ^ t[u].y ^ t[u].z ^ t[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const int H = 720, W1 = 1152;
    const size_t bytes = (size_t)H * W1 * 1024;
    u32x4* v;
    unsigned* out;
    hipMalloc(&v, bytes);
    hipMalloc(&out, 4);
    hipMemset(v, 1, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        hipEventRecord(a);
        const int it = 20;
        for (int i = 0; i < it; i++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-28s %8.1f us  %7.0f GB/s\n", name, ms * 1000 / it, bytes / (ms / it * 1e-3) / 1e9);
    };
    timeit("chain unroll 1", [&] { hipLaunchKernelGGL(k_chain<1>, dim3(W1), dim3(256), 0, 0, v, H, W1, out); });
    timeit("chain unroll 2", [&] { hipLaunchKernelGGL(k_chain<2>, dim3(W1), dim3(256), 0, 0, v, H, W1, out); });
    timeit("chain unroll 4", [&] { hipLaunchKernelGGL(k_chain<4>, dim3(W1), dim3(256), 0, 0, v, H, W1, out); });
    timeit("chain unroll 8", [&] { hipLaunchKernelGGL(k_chain<8>, dim3(W1), dim3(256), 0, 0, v, H, W1, out); });
    timeit("south-like, dir per instr", [&] { hipLaunchKernelGGL(k_south_like<false>, dim3(W1), dim3(192), 0, 0, v, H, W1, out); });
    timeit("south-like, row per instr", [&] { hipLaunchKernelGGL(k_south_like<true>, dim3(W1), dim3(192), 0, 0, v, H, W1, out); });
    unsigned* cvol;
    hipMalloc(&cvol, bytes / 4);
    hipMemset(cvol, 2, bytes / 4);
    {
        const size_t b0 = bytes;
        timeit("south-like + C LA 12", [&] { hipLaunchKernelGGL(k_south_like_c<12>, dim3(W1), dim3(256), 0, 0, v, cvol, H, W1, out); });
        timeit("south-like + C LA 24", [&] { hipLaunchKernelGGL(k_south_like_c<24>, dim3(W1), dim3(256), 0, 0, v, cvol, H, W1, out); });
        timeit("south-like + C LA 48", [&] { hipLaunchKernelGGL(k_south_like_c<48>, dim3(W1), dim3(256), 0, 0, v, cvol, H, W1, out); });
        (void)b0;
    }
    const size_t n = bytes / 16;
    timeit("linear 1024 WG unroll 4", [&] { hipLaunchKernelGGL(k_linear<4>, dim3(1024), dim3(256), 0, 0, v, n, out); });
    timeit("linear 4096 WG unroll 4", [&] { hipLaunchKernelGGL(k_linear<4>, dim3(4096), dim3(256), 0, 0, v, n, out); });
    timeit("linear 1152 WG unroll 8", [&] { hipLaunchKernelGGL(k_linear<8>, dim3(1152), dim3(256), 0, 0, v, n, out); });
    return 0;
}
