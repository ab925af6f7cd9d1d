// The FGS coefficient job's dependent chain on one wave (round 6): cycles a sample of
//   den = omc - aa * (1 + t); r = rcp + Newton; q0 = cc * r; t = fma(-fma(q0, den, -cc), r, q0)
// with the operands in registers (V0), with the IEEE division instead of the Markstein form (V1),
// the chain without the reciprocal's Newton step (V2, wrong results: the rcp latency's share), and
// the pass's 5-op forward chain for scale (V3).
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
constexpr int STEPS = 2048;
template <int V>
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* tm, float a0, float c0) {
    float t = 0.0f, aa = a0 * (1 + threadIdx.x * 1e-3f), cc = c0 * (1 + threadIdx.x * 1e-3f), omc = 1.0f - cc;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < STEPS; i++) {
        const float den = omc - aa * (1.0f + t);
        if (V == 0 || V == 2) {
            const float r0 = __builtin_amdgcn_rcpf(den);
            const float r = V == 2 ? r0 : __builtin_fmaf(__builtin_fmaf(-den, r0, 1.0f), r0, r0);
            const float q0 = cc * r;
            t = __builtin_fmaf(-__builtin_fmaf(q0, den, -cc), r, q0);
        } else if (V == 1) {
            t = cc / den;
        } else {
            const float x = omc - aa * t;
            const float q0 = x * cc;
            t = __builtin_fmaf(-__builtin_fmaf(q0, aa, -x), cc, q0);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) tm[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 + threadIdx.x] = t;
}
template <int V>
void run(const char* name) {
    float* o;
    unsigned long long* t;
    hipMalloc(&o, 64 * 64 * 4);
    hipMalloc(&t, 64 * 8);
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k<V>, dim3(64), dim3(64), 0, 0, o, t, -3.0f, -2.0f);
    hipDeviceSynchronize();
    unsigned long long h[64];
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    unsigned long long m = h[0];
    for (int i = 1; i < 64; i++) m = h[i] < m ? h[i] : m;
    printf("%-44s %.1f cycles a sample\n", name, (double)m / STEPS);
    hipFree(o);
    hipFree(t);
}
int main() {
    run<0>("job chain (rcp + Newton, Markstein)");
    run<1>("job chain with the IEEE division");
    run<2>("job chain without the Newton step (wrong)");
    run<3>("pass forward chain (5 ops)");
    return 0;
}
