// Dependent-chain latency of the cross-lane moves on one wave (round 6): v_permlane16_swap,
// v_permlane32_swap, DPP row_shr:1 (v_mov_dpp), ds_swizzle, and v_add for scale.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int STEPS = 4096;
template <int V>
__global__ __launch_bounds__(64) void k(int* out, unsigned long long* t) {
    int v = threadIdx.x * 7 + 1, d = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < STEPS; i++) {
        if (V == 0) v = v + d;
        if (V == 1) v = (int)__builtin_amdgcn_permlane16_swap(d, v, false, false)[0];
        if (V == 2) v = (int)__builtin_amdgcn_permlane32_swap(d, v, false, false)[0];
        if (V == 3) v = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
        if (V == 4) v = __builtin_amdgcn_ds_swizzle(v, 0x041F);
        if (V == 5) v = (int)__builtin_amdgcn_permlane16_swap(d, v, false, false)[0] + d;
        if (V == 6) v = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false) + d;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 + threadIdx.x] = v;
}
template <int V>
void run(const char* name) {
    int* o;
    unsigned long long* t;
    hipMalloc(&o, 64 * 64 * 4);
    hipMalloc(&t, 64 * 8);
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k<V>, dim3(64), dim3(64), 0, 0, o, t);
    hipDeviceSynchronize();
    unsigned long long h[64];
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 64; i++) s += h[i];
    printf("%-32s %6.2f cycles per step\n", name, s / 64 / STEPS);
}
int main() {
    run<0>("v_add chain");
    run<1>("permlane16_swap chain");
    run<2>("permlane32_swap chain");
    run<3>("dpp row_shr:1 mov chain");
    run<4>("ds_swizzle chain");
    run<5>("permlane16_swap + add chain");
    run<6>("dpp mov + add chain");
    return 0;
}
