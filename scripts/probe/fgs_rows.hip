// Probe (round 6): cycles per line-sample of the sequential FGS forward + back steps on one wave,
// one right-hand side per wave, in two lane layouts:
//   V0  lanes 0-15 = 16 lines, one sample per step, operands read per sample (round-5 style)
//   V1  4 rows x 16 lines: row r holds samples 4*pos(r)+e of each 16-sample group; the chain value
//       visits the rows in the order 0,1,3,2 (permlane16/32 swaps), each row's 4 steps under an
//       exec mask; operands read 4 samples a lane-instruction, results kept per row
// plus 2 waves at once (two right-hand sides on two SIMDs).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)
constexpr int N = 384;  // samples a line
constexpr int L = 16;   // lines

__device__ __forceinline__ float mdiv(float x, float den, float r) {
    const float q0 = x * r;
    return __builtin_fmaf(-__builtin_fmaf(q0, den, -x), r, q0);
}
__device__ __forceinline__ uint32_t tkey(float q) { return __builtin_bit_cast(uint32_t, q) * 2u - 1u; }

// LDS: coef float4 [N][L] (a, den, r, t); u float [N][L] per wave-image (k-major), results in place
template <int V, int KEY>
__global__ __launch_bounds__(128) void k(float* out, unsigned long long* t, int nw) {
    __shared__ __attribute__((aligned(16))) float4 coef[N * L];
    __shared__ __attribute__((aligned(16))) float u[2][N * L];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < N * L; i += blockDim.x) {
        coef[i] = make_float4(-0.2f - (i & 3) * 0.01f, 1.5f + (i & 7) * 0.1f, 0.0f, 0.1f);
        coef[i].z = 1.0f / coef[i].y;
        u[0][i] = 0.7f + (i & 15) * 0.01f;
        u[1][i] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15, row = lane >> 4;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    if (V == 0) {
        if (lane < 16) {
            float p = 0.0f;
#pragma unroll 16
            for (int k = 0; k < N; k++) {
                const float4 q = coef[k * L + l];
                const float x = uu[k * L + l] - q.x * p;
                p = mdiv(x, q.y, q.z);
                if (KEY) key = min(key, tkey(x * q.z));
                uu[k * L + l] = p;
            }
            t1 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
            for (int k = N - 2; k >= 0; k--) {
                p = uu[k * L + l] - coef[k * L + l].w * p;
                uu[k * L + l] = p;
            }
        }
    } else {
        // pos(row): 0->0, 1->1, 3->2, 2->3
        const int pos = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
        float p = 0.0f;
        for (int g = 0; g < N / 16; g++) {
            const int kb = g * 16 + 4 * pos;
            float4 q[4];
            float x[4], res[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                q[e] = coef[(kb + e) * L + l];
                x[e] = uu[(kb + e) * L + l];
            }
#define PHASE(R)                                                   \
    if (row == R) {                                                \
        _Pragma("unroll") for (int e = 0; e < 4; e++) {            \
            const float xx = x[e] - q[e].x * p;                    \
            p = mdiv(xx, q[e].y, q[e].z);                          \
            if (KEY) key = min(key, tkey(xx * q[e].z));            \
            res[e] = p;                                            \
        }                                                          \
    }
            PHASE(0)
            p = __builtin_amdgcn_permlane16_swap(p, p, false, false)[0];  // row 0 -> 1
            PHASE(1)
            p = __builtin_amdgcn_permlane32_swap(p, p, false, false)[0];  // row 1 -> 3
            PHASE(3)
            p = __builtin_amdgcn_permlane16_swap(p, p, false, false)[1];  // row 3 -> 2
            PHASE(2)
            p = __builtin_amdgcn_permlane32_swap(p, p, false, false)[1];  // row 2 -> 0
#pragma unroll
            for (int e = 0; e < 4; e++) uu[(kb + e) * L + l] = res[e];
        }
        t1 = __builtin_amdgcn_s_memtime();
        // back: groups from the end, rows in the reverse order 2,3,1,0
        p = __builtin_amdgcn_permlane32_swap(p, p, false, false)[0];  // the last value (row 0... ) -> row 2
        for (int g = N / 16 - 1; g >= 0; g--) {
            const int kb = g * 16 + 4 * pos;
            float tt[4], x[4], res[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                tt[e] = coef[(kb + e) * L + l].w;
                x[e] = uu[(kb + e) * L + l];
            }
#define BPHASE(R)                                                  \
    if (row == R) {                                                \
        _Pragma("unroll") for (int e = 3; e >= 0; e--) {           \
            p = x[e] - tt[e] * p;                                  \
            res[e] = p;                                            \
        }                                                          \
    }
            BPHASE(2)
            p = __builtin_amdgcn_permlane16_swap(p, p, false, false)[0];  // row 2 -> 3
            BPHASE(3)
            p = __builtin_amdgcn_permlane32_swap(p, p, false, false)[1];  // row 3 -> 1
            BPHASE(1)
            p = __builtin_amdgcn_permlane16_swap(p, p, false, false)[1];  // row 1 -> 0
            BPHASE(0)
            p = __builtin_amdgcn_permlane32_swap(p, p, false, false)[0];  // row 0 -> 2
#pragma unroll
            for (int e = 0; e < 4; e++) uu[(kb + e) * L + l] = res[e];
        }
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

// V2: V1 with the chain value moved by bit (not numeric conversion), the next group's operands
// loaded during the current group, and the swap's second operand a dead register
__device__ __forceinline__ float mv16a(float dead, float p) {  // row 0 -> 1 (and 2 -> 3)
    auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, dead), __builtin_bit_cast(int, p), false, false);
    return __builtin_bit_cast(float, (int)r[0]);
}
__device__ __forceinline__ float mv16b(float p, float dead) {  // row 1 -> 0 (and 3 -> 2)
    auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, p), __builtin_bit_cast(int, dead), false, false);
    return __builtin_bit_cast(float, (int)r[1]);
}
__device__ __forceinline__ float mv32a(float dead, float p) {  // rows 0,1 -> 2,3
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, dead), __builtin_bit_cast(int, p), false, false);
    return __builtin_bit_cast(float, (int)r[0]);
}
__device__ __forceinline__ float mv32b(float p, float dead) {  // rows 2,3 -> 0,1
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, p), __builtin_bit_cast(int, dead), false, false);
    return __builtin_bit_cast(float, (int)r[1]);
}

template <int KEY>
__global__ __launch_bounds__(128) void k2(float* out, unsigned long long* t, int nw) {
    __shared__ __attribute__((aligned(16))) float4 coef[N * L];
    __shared__ __attribute__((aligned(16))) float u[2][N * L];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < N * L; i += blockDim.x) {
        coef[i] = make_float4(-0.2f - (i & 3) * 0.01f, 1.5f + (i & 7) * 0.1f, 0.0f, 0.1f);
        coef[i].z = 1.0f / coef[i].y;
        u[0][i] = 0.7f + (i & 15) * 0.01f;
        u[1][i] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15, row = lane >> 4;
    const int pos = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    float p = 0.0f, dead = 0.0f;
    float4 q[4], qn[4];
    float x[4], xn[4], res[4];
    auto ld = [&](int g, float4* qq, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            qq[e] = coef[(kb + e) * L + l];
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    ld(0, q, x);
    for (int g = 0; g < N / 16; g++) {
        if (g + 1 < N / 16) ld(g + 1, qn, xn);
#define PHASE2(R)                                                  \
    if (row == R) {                                                \
        _Pragma("unroll") for (int e = 0; e < 4; e++) {            \
            const float xx = x[e] - q[e].x * p;                    \
            p = mdiv(xx, q[e].y, q[e].z);                          \
            if (KEY) key = min(key, tkey(xx * q[e].z));            \
            res[e] = p;                                            \
        }                                                          \
    }
        PHASE2(0)
        p = mv16a(dead, p);
        PHASE2(1)
        p = mv32a(dead, p);
        PHASE2(3)
        p = mv16b(p, dead);
        PHASE2(2)
        p = mv32b(p, dead);
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            uu[(kb + e) * L + l] = res[e];
            q[e] = qn[e];
            x[e] = xn[e];
        }
    }
    t1 = __builtin_amdgcn_s_memtime();
    p = mv32a(dead, p);  // row 0 -> row 2
    float tt[4], tn[4];
    auto ldb = [&](int g, float* t4, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            t4[e] = coef[(kb + e) * L + l].w;
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    ldb(N / 16 - 1, tt, x);
    for (int g = N / 16 - 1; g >= 0; g--) {
        if (g > 0) ldb(g - 1, tn, xn);
#define BPHASE2(R)                                                 \
    if (row == R) {                                                \
        _Pragma("unroll") for (int e = 3; e >= 0; e--) {           \
            p = x[e] - tt[e] * p;                                  \
            res[e] = p;                                            \
        }                                                          \
    }
        BPHASE2(2)
        p = mv16a(dead, p);  // row 2 -> 3
        BPHASE2(3)
        p = mv32b(p, dead);  // row 3 -> 1
        BPHASE2(1)
        p = mv16b(p, dead);  // row 1 -> 0
        BPHASE2(0)
        p = mv32a(dead, p);  // row 0 -> 2
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            uu[(kb + e) * L + l] = res[e];
            tt[e] = tn[e];
            x[e] = xn[e];
        }
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

template <int KEY>
__global__ __launch_bounds__(128) void k3(float* out, unsigned long long* t, int nw) {
    __shared__ __attribute__((aligned(16))) float4 coef[N * L];
    __shared__ __attribute__((aligned(16))) float u[2][N * L];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < N * L; i += blockDim.x) {
        coef[i] = make_float4(-0.2f - (i & 3) * 0.01f, 1.5f + (i & 7) * 0.1f, 0.0f, 0.1f);
        coef[i].z = 1.0f / coef[i].y;
        u[0][i] = 0.7f + (i & 15) * 0.01f;
        u[1][i] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15, row = lane >> 4;
    const int pos = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    float p = 0.0f, dead = 0.0f;
    float4 qa[4], qb[4];
    float xa[4], xb[4], res[4];
    auto ld = [&](int g, float4* qq, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            qq[e] = coef[(kb + e) * L + l];
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    auto grp = [&](int g, const float4* q, const float* x) __attribute__((always_inline)) {
        PHASE2(0)
        p = mv16a(dead, p);
        PHASE2(1)
        p = mv32a(dead, p);
        PHASE2(3)
        p = mv16b(p, dead);
        PHASE2(2)
        p = mv32b(p, dead);
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) uu[(kb + e) * L + l] = res[e];
    };
    ld(0, qa, xa);
    for (int g = 0; g < N / 16; g += 2) {
        ld(g + 1, qb, xb);
        grp(g, qa, xa);
        if (g + 2 < N / 16) ld(g + 2, qa, xa);
        grp(g + 1, qb, xb);
    }
    t1 = __builtin_amdgcn_s_memtime();
    p = mv32a(dead, p);  // row 0 -> row 2
    auto ldb = [&](int g, float* t4, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            t4[e] = coef[(kb + e) * L + l].w;
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    auto grpb = [&](int g, const float* tt, const float* x) __attribute__((always_inline)) {
        BPHASE2(2)
        p = mv16a(dead, p);
        BPHASE2(3)
        p = mv32b(p, dead);
        BPHASE2(1)
        p = mv16b(p, dead);
        BPHASE2(0)
        p = mv32a(dead, p);
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) uu[(kb + e) * L + l] = res[e];
    };
    float ta[4], tb[4];
    ldb(N / 16 - 1, ta, xa);
    for (int g = N / 16 - 1; g >= 0; g -= 2) {
        ldb(g - 1, tb, xb);
        grpb(g, ta, xa);
        if (g - 2 >= 0) ldb(g - 2, ta, xa);
        grpb(g - 1, tb, xb);
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

// V4: no exec masks: every row computes every step (same issue cost), the chain value valid in
// the active row; per-phase result and key registers, each row's own selected at the group's end
template <int KEY>
__global__ __launch_bounds__(128) void k4(float* out, unsigned long long* t, int nw) {
    __shared__ __attribute__((aligned(16))) float4 coef[N * L];
    __shared__ __attribute__((aligned(16))) float u[2][N * L];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < N * L; i += blockDim.x) {
        coef[i] = make_float4(-0.2f - (i & 3) * 0.01f, 1.5f + (i & 7) * 0.1f, 0.0f, 0.1f);
        coef[i].z = 1.0f / coef[i].y;
        u[0][i] = 0.7f + (i & 15) * 0.01f;
        u[1][i] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15, row = lane >> 4;
    const int pos = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
    const bool r0 = row == 0, r1 = row == 1, r3 = row == 3;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    float p = 0.0f, dead = 0.0f;
    float4 qa[4], qb[4];
    float xa[4], xb[4];
    auto ld = [&](int g, float4* qq, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            qq[e] = coef[(kb + e) * L + l];
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    auto grp = [&](int g, const float4* q, const float* x) __attribute__((always_inline)) {
        float res[4][4];
        uint32_t kk[4] = {~0u, ~0u, ~0u, ~0u};
        auto ph = [&](int ri) __attribute__((always_inline)) {
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float xx = x[e] - q[e].x * p;
                const float q0 = xx * q[e].z;
                p = __builtin_fmaf(-__builtin_fmaf(q0, q[e].y, -xx), q[e].z, q0);
                if (KEY) kk[ri] = min(kk[ri], tkey(q0));
                res[ri][e] = p;
            }
        };
        ph(0);
        p = mv16a(dead, p);
        ph(1);
        p = mv32a(dead, p);
        ph(2);  // row 3
        p = mv16b(p, dead);
        ph(3);  // row 2
        p = mv32b(p, dead);
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++)
            uu[(kb + e) * L + l] = r0 ? res[0][e] : r1 ? res[1][e] : r3 ? res[2][e] : res[3][e];
        if (KEY) key = min(key, r0 ? kk[0] : r1 ? kk[1] : r3 ? kk[2] : kk[3]);
    };
    ld(0, qa, xa);
    for (int g = 0; g < N / 16; g += 2) {
        ld(g + 1, qb, xb);
        grp(g, qa, xa);
        if (g + 2 < N / 16) ld(g + 2, qa, xa);
        grp(g + 1, qb, xb);
    }
    t1 = __builtin_amdgcn_s_memtime();
    p = mv32a(dead, p);  // row 0 -> row 2
    auto ldb = [&](int g, float* t4, float* xx) __attribute__((always_inline)) {
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            t4[e] = coef[(kb + e) * L + l].w;
            xx[e] = uu[(kb + e) * L + l];
        }
    };
    auto grpb = [&](int g, const float* tt, const float* x) __attribute__((always_inline)) {
        float res[4][4];
        auto ph = [&](int ri) __attribute__((always_inline)) {
#pragma unroll
            for (int e = 3; e >= 0; e--) {
                p = x[e] - tt[e] * p;
                res[ri][e] = p;
            }
        };
        ph(3);  // row 2
        p = mv16a(dead, p);
        ph(2);  // row 3
        p = mv32b(p, dead);
        ph(1);
        p = mv16b(p, dead);
        ph(0);
        p = mv32a(dead, p);
        const int kb = g * 16 + 4 * pos;
#pragma unroll
        for (int e = 0; e < 4; e++)
            uu[(kb + e) * L + l] = r0 ? res[0][e] : r1 ? res[1][e] : r3 ? res[2][e] : res[3][e];
    };
    float ta[4], tb[4];
    ldb(N / 16 - 1, ta, xa);
    for (int g = N / 16 - 1; g >= 0; g -= 2) {
        ldb(g - 1, tb, xb);
        grpb(g, ta, xa);
        if (g - 2 >= 0) ldb(g - 2, ta, xa);
        grpb(g - 1, tb, xb);
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

// V5: lane = line (16 lines, all rows the same lines: only row 0's results used), LINE-MAJOR
// operands: u[l][k], coef as [l][k/4][a0..3 den0..3 r0..3], t[l][k]: one b128 read gives a lane 4
// consecutive samples; results written 4 at a time; no cross-lane moves
template <int KEY>
__global__ __launch_bounds__(128) void k5(float* out, unsigned long long* t, int nw) {
    __shared__ __attribute__((aligned(16))) float cf[L * N * 3];  // [l][k/4][12]
    __shared__ __attribute__((aligned(16))) float tt[L * N];      // [l][k]
    __shared__ __attribute__((aligned(16))) float u[2][L * N];    // [l][k]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < L * N; i += blockDim.x) {
        const int l = i / N, k = i % N;
        const float den = 1.5f + (i & 7) * 0.1f;
        float* c = cf + (l * (N / 4) + k / 4) * 12 + (k & 3);
        c[0] = -0.2f - (i & 3) * 0.01f;
        c[4] = den;
        c[8] = 1.0f / den;
        tt[i] = 0.1f;
        u[0][i] = 0.7f + (i & 15) * 0.01f;
        u[1][i] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    float p = 0.0f;
    const float4* U4 = (const float4*)(uu + l * N);
    float4* W4 = (float4*)(uu + l * N);
    const float4* C4 = (const float4*)(cf + l * N * 3);
    const float4* T4 = (const float4*)(tt + l * N);
    float4 xa = U4[0], aa = C4[0], da = C4[1], ra = C4[2];
#pragma unroll 4
    for (int b = 0; b < N / 4; b++) {
        const int bn = b + 1 < N / 4 ? b + 1 : b;
        const float4 xn = U4[bn], an = C4[3 * bn], dn = C4[3 * bn + 1], rn = C4[3 * bn + 2];
        float4 o;
        const float xv[4] = {xa.x, xa.y, xa.z, xa.w}, av[4] = {aa.x, aa.y, aa.z, aa.w};
        const float dv[4] = {da.x, da.y, da.z, da.w}, rv[4] = {ra.x, ra.y, ra.z, ra.w};
        float ov[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float x = xv[e] - av[e] * p;
            const float q0 = x * rv[e];
            p = __builtin_fmaf(-__builtin_fmaf(q0, dv[e], -x), rv[e], q0);
            if (KEY) key = min(key, tkey(q0));
            ov[e] = p;
        }
        o = make_float4(ov[0], ov[1], ov[2], ov[3]);
        W4[b] = o;
        xa = xn; aa = an; da = dn; ra = rn;
    }
    t1 = __builtin_amdgcn_s_memtime();
    float4 xb = W4[N / 4 - 1], tb = T4[N / 4 - 1];
#pragma unroll 4
    for (int b = N / 4 - 1; b >= 0; b--) {
        const int bn = b > 0 ? b - 1 : 0;
        const float4 xn = W4[bn], tn = T4[bn];
        const float xv[4] = {xb.x, xb.y, xb.z, xb.w}, tv[4] = {tb.x, tb.y, tb.z, tb.w};
        float ov[4];
#pragma unroll
        for (int e = 3; e >= 0; e--) {
            p = xv[e] - tv[e] * p;
            ov[e] = p;
        }
        W4[b] = make_float4(ov[0], ov[1], ov[2], ov[3]);
        xb = xn; tb = tn;
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

template <int KEY>
__global__ __launch_bounds__(128) void k6(float* out, unsigned long long* t, int nw) {
    constexpr int NP = N + 4, CP = N * 3 + 12;  // padded line strides: lanes on distinct banks
    __shared__ __attribute__((aligned(16))) float cf[L * CP];  // [l][k/4][12]
    __shared__ __attribute__((aligned(16))) float tt[L * NP];  // [l][k]
    __shared__ __attribute__((aligned(16))) float u[2][L * NP];    // [l][k]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < L * N; i += blockDim.x) {
        const int l = i / N, k = i % N;
        const float den = 1.5f + (i & 7) * 0.1f;
        float* c = cf + l * CP + (k / 4) * 12 + (k & 3);
        c[0] = -0.2f - (i & 3) * 0.01f;
        c[4] = den;
        c[8] = 1.0f / den;
        tt[l * NP + k] = 0.1f;
        u[0][l * NP + k] = 0.7f + (i & 15) * 0.01f;
        u[1][l * NP + k] = 0.3f + (i & 31) * 0.01f;
    }
    __syncthreads();
    if (w >= nw) return;
    float* uu = u[w];
    const int l = lane & 15;
    uint32_t key = ~0u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
    float p = 0.0f;
    const float4* U4 = (const float4*)(uu + l * NP);
    float4* W4 = (float4*)(uu + l * NP);
    const float4* C4 = (const float4*)(cf + l * CP);
    const float4* T4 = (const float4*)(tt + l * NP);
    float4 xa = U4[0], aa = C4[0], da = C4[1], ra = C4[2];
#pragma unroll 4
    for (int b = 0; b < N / 4; b++) {
        const int bn = b + 1 < N / 4 ? b + 1 : b;
        const float4 xn = U4[bn], an = C4[3 * bn], dn = C4[3 * bn + 1], rn = C4[3 * bn + 2];
        float4 o;
        const float xv[4] = {xa.x, xa.y, xa.z, xa.w}, av[4] = {aa.x, aa.y, aa.z, aa.w};
        const float dv[4] = {da.x, da.y, da.z, da.w}, rv[4] = {ra.x, ra.y, ra.z, ra.w};
        float ov[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float x = xv[e] - av[e] * p;
            const float q0 = x * rv[e];
            p = __builtin_fmaf(-__builtin_fmaf(q0, dv[e], -x), rv[e], q0);
            if (KEY) key = min(key, tkey(q0));
            ov[e] = p;
        }
        o = make_float4(ov[0], ov[1], ov[2], ov[3]);
        W4[b] = o;
        xa = xn; aa = an; da = dn; ra = rn;
    }
    t1 = __builtin_amdgcn_s_memtime();
    float4 xb = W4[N / 4 - 1], tb = T4[N / 4 - 1];
#pragma unroll 4
    for (int b = N / 4 - 1; b >= 0; b--) {
        const int bn = b > 0 ? b - 1 : 0;
        const float4 xn = W4[bn], tn = T4[bn];
        const float xv[4] = {xb.x, xb.y, xb.z, xb.w}, tv[4] = {tb.x, tb.y, tb.z, tb.w};
        float ov[4];
#pragma unroll
        for (int e = 3; e >= 0; e--) {
            p = xv[e] - tv[e] * p;
            ov[e] = p;
        }
        W4[b] = make_float4(ov[0], ov[1], ov[2], ov[3]);
        xb = xn; tb = tn;
    }
    t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        t[(blockIdx.x * 2 + w) * 2] = t1 - t0;
        t[(blockIdx.x * 2 + w) * 2 + 1] = t2 - t1;
    }
    out[blockIdx.x * 128 + threadIdx.x] = uu[lane] + (float)(key & 1);
}

template <int V, int KEY>
void run(const char* name, int nw) {
    float* o;
    unsigned long long* t;
    hipMalloc(&o, 1024 * 128 * 4);
    hipMalloc(&t, 1024 * 4 * 8);
    for (int it = 0; it < 3; it++) {
        if (V == 2) hipLaunchKernelGGL((k2<KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
        else if (V == 3) hipLaunchKernelGGL((k3<KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
        else if (V == 4) hipLaunchKernelGGL((k4<KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
        else if (V == 5) hipLaunchKernelGGL((k5<KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
        else if (V == 6) hipLaunchKernelGGL((k6<KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
        else hipLaunchKernelGGL((k<V, KEY>), dim3(64), dim3(128), 0, 0, o, t, nw);
    }
    hipDeviceSynchronize();
    unsigned long long h[64 * 4];
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    double f = 0, b = 0;
    for (int i = 0; i < 64; i++) {
        f += h[i * 4];
        b += h[i * 4 + 1];
    }
    printf("%-40s waves %d: fwd %6.1f  back %6.1f cycles per sample\n", name, nw, f / 64 / N, b / 64 / N);
    hipFree(o);
    hipFree(t);
}

int main() {
    for (int nw = 1; nw <= 2; nw++) {
        run<0, 0>("V0 16 lanes, no key", nw);
        run<0, 1>("V0 16 lanes, key", nw);
        run<1, 0>("V1 4 rows, no key", nw);
        run<1, 1>("V1 4 rows, key", nw);
        run<2, 0>("V2 4 rows, moves by bit, prefetch, no key", nw);
        run<2, 1>("V2 4 rows, moves by bit, prefetch, key", nw);
        run<3, 0>("V3 = V2 + two groups a trip, no key", nw);
        run<3, 1>("V3 = V2 + two groups a trip, key", nw);
        run<4, 0>("V4 no exec masks, no key", nw);
        run<4, 1>("V4 no exec masks, key", nw);
        run<5, 0>("V5 lane = line, line-major b128, no key", nw);
        run<5, 1>("V5 lane = line, line-major b128, key", nw);
        run<6, 0>("V6 = V5 with padded line strides, no key", nw);
        run<6, 1>("V6 = V5 with padded line strides, key", nw);
    }
    return 0;
}
