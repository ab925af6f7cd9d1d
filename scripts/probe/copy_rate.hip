// Copy / read / write rates of a 2 GiB buffer pair under several access shapes, to pick the
// streaming probe's form (sdr_stream_probe).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// grid-stride over workgroup spans of 256*U vectors
template <int U, int NT>
__global__ __launch_bounds__(256) void k_copy_gs(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t span = (size_t)256 * U;
    for (size_t b = (size_t)blockIdx.x * span; b + span <= n; b += (size_t)gridDim.x * span) {
        u4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT & 1 ? __builtin_nontemporal_load(&s[b + u * 256 + threadIdx.x]) : s[b + u * 256 + threadIdx.x];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT & 2) __builtin_nontemporal_store(v[u], &d[b + u * 256 + threadIdx.x]);
            else d[b + u * 256 + threadIdx.x] = v[u];
        }
    }
}
// each workgroup a contiguous chunk of n / grid vectors
template <int U, int NT>
__global__ __launch_bounds__(256) void k_copy_chunk(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t per = n / gridDim.x, b0 = blockIdx.x * per, span = (size_t)256 * U;
    for (size_t b = b0; b + span <= b0 + per; b += span) {
        u4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT & 1 ? __builtin_nontemporal_load(&s[b + u * 256 + threadIdx.x]) : s[b + u * 256 + threadIdx.x];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT & 2) __builtin_nontemporal_store(v[u], &d[b + u * 256 + threadIdx.x]);
            else d[b + u * 256 + threadIdx.x] = v[u];
        }
    }
}
template <int U>
__global__ __launch_bounds__(256) void k_read(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t span = (size_t)256 * U;
    u4 acc = {0, 0, 0, 0};
    for (size_t b = (size_t)blockIdx.x * span; b + span <= n; b += (size_t)gridDim.x * span) {
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= s[b + u * 256 + threadIdx.x];
    }
    if (acc.x == 0x12345678u && acc.y == 0x9abcdefu) d[threadIdx.x] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void k_write(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
    const size_t span = (size_t)256 * U;
    const u4 v = {1u, 2u, 3u, (unsigned)blockIdx.x};
    for (size_t b = (size_t)blockIdx.x * span; b + span <= n; b += (size_t)gridDim.x * span) {
#pragma unroll
        for (int u = 0; u < U; u++) d[b + u * 256 + threadIdx.x] = v;
    }
}

typedef void (*fn)(const u4*, u4*, size_t);
int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 16;
    u4 *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipMemset(b, 2, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct V { const char* name; fn f; int kind; };  // kind 0 copy (2x bytes), 1 read, 2 write
    std::vector<V> vs = {
        {"gs U4 plain", k_copy_gs<4, 0>, 0},   {"gs U4 ntld", k_copy_gs<4, 1>, 0},  {"gs U4 ntst", k_copy_gs<4, 2>, 0},
        {"gs U4 nt both", k_copy_gs<4, 3>, 0}, {"gs U8 plain", k_copy_gs<8, 0>, 0}, {"gs U8 ntld", k_copy_gs<8, 1>, 0},
        {"gs U8 nt both", k_copy_gs<8, 3>, 0}, {"gs U16 plain", k_copy_gs<16, 0>, 0}, {"gs U1 plain", k_copy_gs<1, 0>, 0},
        {"chunk U4 plain", k_copy_chunk<4, 0>, 0}, {"chunk U8 plain", k_copy_chunk<8, 0>, 0},
        {"chunk U8 ntld", k_copy_chunk<8, 1>, 0}, {"chunk U8 nt both", k_copy_chunk<8, 3>, 0},
        {"read U4", k_read<4>, 1}, {"read U8", k_read<8>, 1}, {"write U4", k_write<4>, 2}, {"write U8", k_write<8>, 2}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& v : vs)
        for (int wpc : {2, 4, 8, 16, 32}) {
            const dim3 grid(cus * wpc);
            hipLaunchKernelGGL(v.f, grid, dim3(256), 0, 0, a, b, n);
            hipEventRecord(e0, 0);
            const int it = 10;
            for (int i = 0; i < it; i++) hipLaunchKernelGGL(v.f, grid, dim3(256), 0, 0, a, b, n);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double by = (v.kind == 0 ? 2.0 : 1.0) * bytes * it;
            printf("%-18s wg/CU %2d  %7.1f GB/s\n", v.name, wpc, by / (ms * 1e-3) / 1e9);
        }
    return 0;
}
