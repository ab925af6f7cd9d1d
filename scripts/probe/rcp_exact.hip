// Probe: is r1 = fma(fma(-d, r0, 1), r0, r0), r0 = v_rcp_f32(d), the correctly rounded 1/d for every
// mantissa of d (d in [2^e, 2^(e+1)) for several e)?  Compared with the IEEE division 1.0f / d.
// hipcc --offload-arch=gfx950 -O3 -o rcp_exact rcp_exact.hip && ./rcp_exact
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)
__global__ void k(int e, unsigned long long* bad, unsigned long long* bad0, uint32_t* first) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float d = __builtin_bit_cast(float, (uint32_t)(127 + e) << 23 | m);
    const float ref = 1.0f / d;
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r1 = __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
    if (__builtin_bit_cast(uint32_t, r0) != __builtin_bit_cast(uint32_t, ref)) atomicAdd(bad0, 1ull);
    if (__builtin_bit_cast(uint32_t, r1) != __builtin_bit_cast(uint32_t, ref)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, m);
    }
}
int main() {
    unsigned long long *bad, *bad0, hb, hb0;
    uint32_t *first, hf;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&bad0, 8);
    (void)hipMalloc(&first, 4);
    for (int e : {0, 1, 7, 13, 20, 30, 45, 59, 100, 125}) {
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(bad0, 0, 8);
        (void)hipMemset(first, 0xff, 4);
        hipLaunchKernelGGL(k, dim3((1 << 23) / 256), dim3(256), 0, 0, e, bad, bad0, first);
        (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&hb0, bad0, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
        printf("d in [2^%d, 2^%d): v_rcp_f32 differs from 1/d for %llu mantissas; one Newton step: %llu (first 0x%06x)\n",
               e, e + 1, hb0, hb, hb ? hf : 0);
    }
    return 0;
}
