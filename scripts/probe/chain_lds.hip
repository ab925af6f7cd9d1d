// Probe: cycles per step of the sequential FGS forward step on one wave: the 5-op packed chain
// alone, + its LDS operand reads (8 samples ahead), + the LDS result row, + the tiny-key check.
// hipcc --offload-arch=gfx950 -O3 -o chain_lds chain_lds.hip && ./chain_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <type_traits>
#pragma clang fp contract(off)
constexpr int STEPS = 1024, PF = 8;
template <int V>
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* t) {
    __shared__ __attribute__((aligned(16))) char lds[256 * 16 * 8 + 256 * 16 * 16 + 64 * 16 * 8];
    const int lane = threadIdx.x;
    const int ln = lane & 15;
    for (int i = lane; i < (int)sizeof(lds) / 4; i += 64) ((float*)lds)[i] = 0.5f + (i & 7) * 0.01f;
    __syncthreads();
    const char* U = lds;
    const char* Q = lds + 256 * 16 * 8;
    char* W = lds + 256 * 16 * 8 + 256 * 16 * 16;
    float2 ru[PF];
    float4 rq[PF];
    for (int j = 0; j < PF; j++) {
        ru[j] = *(const float2*)(U + (j * 16 + ln) * 8);
        rq[j] = *(const float4*)(Q + (j * 16 + ln) * 16);
    }
    float p0 = 0, p1 = 0;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < STEPS / 64 - 1; c++) {
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const int r = j % PF;
            float2 xu = {0.7f, 0.3f};
            float4 xq = {-0.2f, 1.5f, 0.66666f, 0.1f};
            if (V >= 1) {
                xu = ru[r];
                xq = rq[r];
                const int s = (c * 64 + j + PF) & 255;
                ru[r] = *(const float2*)(U + (s * 16 + ln) * 8);
                rq[r] = *(const float4*)(Q + (s * 16 + ln) * 16);
                if (V >= 4) __builtin_amdgcn_sched_barrier(0);
            }
            const float x0 = xu.x - xq.x * p0, x1 = xu.y - xq.x * p1;
            const float q00 = x0 * xq.z, q01 = x1 * xq.z;
            p0 = __builtin_fmaf(-__builtin_fmaf(q00, xq.y, -x0), xq.z, q00);
            p1 = __builtin_fmaf(-__builtin_fmaf(q01, xq.y, -x1), xq.z, q01);
            if (V >= 3) key = min(key, min(__builtin_bit_cast(uint32_t, q00) * 2u - 1u, __builtin_bit_cast(uint32_t, q01) * 2u - 1u));
            if (V >= 2) *(float2*)(W + ((j & 63) * 16 + ln) * 8) = make_float2(p0, p1);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = p0 + p1 + (float)key;
    if (lane == 0) t[0] = t1 - t0;
}
// quad layout: lane = 4 * line + s, lane s of a quad holding sample 4m + s of its line; per step the
// quad's operands are broadcast from lane (step mod 4) by DPP; results collected one per lane and
// written once per 4 steps
template <int S> __device__ __forceinline__ float bc(float v) {
    // quad_perm [S,S,S,S]
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), S * 0x55, 0xF, 0xF, false));
}
template <int V>
__global__ __launch_bounds__(64) void kq(float* out, unsigned long long* t) {
    __shared__ __attribute__((aligned(16))) char lds[256 * 16 * 8 + 256 * 16 * 16 + 64 * 16 * 8];
    const int lane = threadIdx.x;
    const int s = lane & 3, l = lane >> 2;
    for (int i = lane; i < (int)sizeof(lds) / 4; i += 64) ((float*)lds)[i] = 0.5f + (i & 7) * 0.01f;
    __syncthreads();
    const char* U = lds;
    const char* Q = lds + 256 * 16 * 8;
    char* W = lds + 256 * 16 * 8 + 256 * 16 * 16;
    constexpr int G = 2;  // groups of 4 samples ahead
    float2 ru[G];
    float4 rq[G];
    for (int g = 0; g < G; g++) {
        ru[g] = *(const float2*)(U + ((4 * g + s) * 16 + l) * 8);
        rq[g] = *(const float4*)(Q + ((4 * g + s) * 16 + l) * 16);
    }
    float p0 = 0, p1 = 0, w0 = 0, w1 = 0;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < STEPS / 64 - 1; c++) {
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const int r = m % G;
            const float2 gu = ru[r];
            const float4 gq = rq[r];
            const int sm = ((c * 16 + m + G) * 4 + s) & 255;
            ru[r] = *(const float2*)(U + (sm * 16 + l) * 8);
            rq[r] = *(const float4*)(Q + (sm * 16 + l) * 16);
            auto step = [&](auto SP) __attribute__((always_inline)) {
                constexpr int sp = decltype(SP)::value;
                const float ux = bc<sp>(gu.x), uy = bc<sp>(gu.y), qa = bc<sp>(gq.x), qd = bc<sp>(gq.y), qr = bc<sp>(gq.z);
                const float x0 = ux - qa * p0, x1 = uy - qa * p1;
                const float q00 = x0 * qr, q01 = x1 * qr;
                p0 = __builtin_fmaf(-__builtin_fmaf(q00, qd, -x0), qr, q00);
                p1 = __builtin_fmaf(-__builtin_fmaf(q01, qd, -x1), qr, q01);
                if (V >= 1) key = min(key, min(__builtin_bit_cast(uint32_t, q00) * 2u - 1u, __builtin_bit_cast(uint32_t, q01) * 2u - 1u));
                w0 = s == sp ? p0 : w0;
                w1 = s == sp ? p1 : w1;
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
            *(float2*)(W + (((m * 4 + s) & 63) * 16 + l) * 8) = make_float2(w0, w1);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = p0 + p1 + (float)key;
    if (lane == 0) t[0] = t1 - t0;
}

int main() {
    float* out;
    unsigned long long *t, h;
    (void)hipMalloc(&out, 4096 * 4);
    (void)hipMalloc(&t, 8);
    void (*ks[])(float*, unsigned long long*) = {k<0>, k<1>, k<2>, k<3>, k<4>};
    const char* names[] = {"chain only (5 packed ops)", "+ LDS operand reads (8 ahead)", "+ LDS result row", "+ tiny key",
                           "all + sched_barrier after the reads"};
    for (int lanes : {64})
    for (int v = 0; v < 5; v++) {
        for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(ks[v], dim3(1), dim3(lanes), 0, 0, out, t);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
        printf("%2d lanes %-34s %6.1f cycles per step\n", lanes, names[v], (double)h / (STEPS - 64));
    }
    void (*kqs[])(float*, unsigned long long*) = {kq<0>, kq<1>};
    const char* qn[] = {"quad layout (reads, rows, no key)", "quad layout + tiny key"};
    for (int v = 0; v < 2; v++) {
        for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(kqs[v], dim3(1), dim3(64), 0, 0, out, t);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
        printf("%-34s %6.1f cycles per step\n", qn[v], (double)h / (STEPS - 64));
    }
    return 0;
}
