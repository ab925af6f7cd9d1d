// Probe: dependent-chain cycles per VALU op for one wave (s_memtime), f32 scalar vs packed f32, and
// LDS read->use latency.  hipcc --offload-arch=gfx950 -O3 -o valu_lat valu_lat.hip && ./valu_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
constexpr int N = 4096;
__global__ void k_fma(float* out, unsigned long long* t, float a, float b) {
    float x = threadIdx.x * 1e-3f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < N; i++) x = __builtin_fmaf(x, a, b);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_fma2(float* out, unsigned long long* t, float a, float b) {
    float x = threadIdx.x * 1e-3f, y = x + 1.0f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < N; i++) {
        x = __builtin_fmaf(x, a, b);
        y = __builtin_fmaf(y, a, b);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x + y;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_pk(float* out, unsigned long long* t, float a, float b) {
    f2 x = {threadIdx.x * 1e-3f, threadIdx.x * 2e-3f};
    const f2 va = {a, a}, vb = {b, b};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < N; i++) x = __builtin_elementwise_fma(x, va, vb);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x.x + x.y;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_mulsub(float* out, unsigned long long* t, float a, float b) {
    float x = threadIdx.x * 1e-3f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < N; i++) x = b - a * x;
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_lds(float* out, unsigned long long* t, float a, float b) {
    __shared__ int s[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) s[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    int p = threadIdx.x & 15;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N / 16; i++) p = s[p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = (float)p;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}
int main() {
    float* out;
    unsigned long long *t, h;
    hipMalloc(&out, 4096 * 4);
    hipMalloc(&t, 8);
    struct K { const char* name; void (*f)(float*, unsigned long long*, float, float); int ops; };
    K ks[] = {{"v_fma_f32 chain", k_fma, N}, {"2 interleaved v_fma_f32 chains (per step)", k_fma2, N},
              {"v_pk_fma_f32 chain", k_pk, N}, {"mul+sub chain (per step)", k_mulsub, N},
              {"ds_read_b32 pointer chase", k_lds, N / 16}};
    for (int lanes : {64, 16}) {
        for (auto& k : ks) {
            for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k.f, dim3(1), dim3(lanes), 0, 0, out, t, 0.999f, 0.5f);
            hipDeviceSynchronize();
            hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
            printf("block %2d threads  %-44s %6.2f cycles per step\n", lanes, k.name, (double)h / k.ops);
        }
    }
    return 0;
}
