// sdr_device.hpp -- CDNA4 (gfx950) device helpers for the stereo disparity engine.
//
// Costs and path values are int16 (OpenCV's CostType = short).  A 32-bit VGPR holds a packed
// pair of disparities (lo = d, hi = d + 1) so one v_pk_{add,sub,min,max}_i16 advances two
// disparities; a wave64 covers 64 * DPL disparities of one pixel.  Neighbours d-1 / d+1 across
// lanes come from DPP wave_shr:1 / wave_shl:1 moves + v_alignbit, and per-pixel minima from
// DPP butterflies + v_permlane{16,32}_swap (all in-register, no LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace sdr {

typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr int kMaxCost = 32767;
constexpr uint32_t kMaxPair = 0x7fff7fffu;

__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return as_u32(as_s16x2(a) + as_s16x2(b));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
    return as_u32(as_s16x2(a) - as_s16x2(b));
}
__device__ __forceinline__ uint32_t pk_add_sat(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_add_sat(as_s16x2(a), as_s16x2(b)));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_min(as_s16x2(a), as_s16x2(b)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_max(as_s16x2(a), as_s16x2(b)));
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// unsigned saturating a - b per half (v_pk_sub_u16 clamp)
__device__ __forceinline__ uint32_t pk_sub_usat(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_sub_sat(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_max_u(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_max(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_min_u(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_min(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_shr2_u(uint32_t a) { return as_u32(as_u16x2(a) >> (unsigned short)2); }
__device__ __forceinline__ uint32_t splat16(int v) {
    return (uint32_t)(v & 0xffff) * 0x00010001u;
}
// {hi:lo} = {b.lo : a.hi}  i.e. (a >> 16) | (b << 16)
__device__ __forceinline__ uint32_t funnel16(uint32_t b, uint32_t a) {
    return __builtin_amdgcn_alignbit(b, a, 16);
}

// DPP controls (GFX9 encoding)
constexpr int kDppQuadXor1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowMirror = 0x140;
constexpr int kDppWaveShl1 = 0x130;     // lane i <- lane i+1
constexpr int kDppWaveShr1 = 0x138;     // lane i <- lane i-1

// lane i receives lane i-1's value; lane 0 receives `fill`
__device__ __forceinline__ uint32_t lane_from_prev(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, kDppWaveShr1, 0xf, 0xf, false);
}
// lane i receives lane i+1's value; lane 63 receives `fill`
__device__ __forceinline__ uint32_t lane_from_next(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, kDppWaveShl1, 0xf, 0xf, false);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

// Packed-int16 minimum over all 64 lanes, broadcast to every lane (both halves hold the same
// value when the input's halves do).
__device__ __forceinline__ uint32_t wave_min_pk(uint32_t m) {
    m = pk_min(m, dpp_mov<kDppQuadXor1>(m));
    m = pk_min(m, dpp_mov<kDppQuadXor2>(m));
    m = pk_min(m, dpp_mov<kDppRowHalfMirror>(m));
    m = pk_min(m, dpp_mov<kDppRowMirror>(m));
    auto p16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m = pk_min(p16[0], p16[1]);
    auto p32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return pk_min(p32[0], p32[1]);
}

// min(v, v from the DPP-permuted lane) as ONE v_min_u32_dpp: the identity (all ones) as the
// update's old value lets the compiler fold the DPP move into the min.
template <int CTRL>
__device__ __forceinline__ uint32_t min_u32_dpp(uint32_t v) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, CTRL, 0xf, 0xf, false);
    return min(v, t);
}

// Unsigned 32-bit minimum over all 64 lanes, broadcast.  Also the minimum of packed non-negative
// int16 pairs whose two halves are equal (u32 order = int16 order there).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t m) {
    m = min_u32_dpp<kDppQuadXor1>(m);
    m = min_u32_dpp<kDppQuadXor2>(m);
    m = min_u32_dpp<kDppRowHalfMirror>(m);
    m = min_u32_dpp<kDppRowMirror>(m);
    auto p16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m = min((uint32_t)p16[0], (uint32_t)p16[1]);
    auto p32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return min((uint32_t)p32[0], (uint32_t)p32[1]);
}

// The same minimum as a wave-uniform value: row minima by DPP, then the GFX9 row broadcasts
// (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3) leave the wave's minimum in
// lane 63, read into an SGPR.  Four fewer VALU ops than the permlane-swap tail, and the result
// feeds the next ops as a scalar operand.
__device__ __forceinline__ uint32_t wave_min_u32_uniform(uint32_t m) {
    m = min_u32_dpp<kDppQuadXor1>(m);
    m = min_u32_dpp<kDppQuadXor2>(m);
    m = min_u32_dpp<kDppRowHalfMirror>(m);
    m = min_u32_dpp<kDppRowMirror>(m);
    uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)m, 0x142, 0xa, 0xf, false);
    m = min(m, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)m, 0x143, 0xc, 0xf, false);
    m = min(m, t);
    return (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
}

// Unsigned 32-bit minimum over each 16-lane DPP row, broadcast within the row.
__device__ __forceinline__ uint32_t row16_min_u32(uint32_t m) {
    m = min_u32_dpp<kDppQuadXor1>(m);
    m = min_u32_dpp<kDppQuadXor2>(m);
    m = min_u32_dpp<kDppRowHalfMirror>(m);
    return min_u32_dpp<kDppRowMirror>(m);
}

template <int K>
struct Regs {
    uint32_t r[K];
};

// Buffer-resource access: the row base lives in a wave-uniform resource descriptor (SGPRs, scalar
// arithmetic), the lane's byte offset in one VGPR, so a load or store costs no vector address math.
using Rsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ Rsrc rsrc_at(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}

// K packed pairs at the lane's byte offset vofs plus a wave-uniform (SGPR) byte offset sofs: one
// resource per buffer for a whole chain, and one scalar add per step moves every access of the step
// (AUX: the cache-policy bits; 2 = non-temporal)
template <int K, int AUX = 0>
__device__ __forceinline__ Regs<K> load_buf(Rsrc r, uint32_t vofs, uint32_t sofs = 0) {
    Regs<K> v;
    if constexpr (K == 1) {
        v.r[0] = __builtin_amdgcn_raw_buffer_load_b32(r, vofs, sofs, AUX);
    } else if constexpr (K == 2) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, vofs, sofs, AUX);
        v.r[0] = t[0];
        v.r[1] = t[1];
    } else {
        static_assert(K % 4 == 0, "K = 1, 2 or a multiple of 4");
#pragma unroll
        for (int j = 0; j < K / 4; j++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, vofs + 16 * j, sofs, AUX);
            v.r[4 * j] = t[0]; v.r[4 * j + 1] = t[1]; v.r[4 * j + 2] = t[2]; v.r[4 * j + 3] = t[3];
        }
    }
    return v;
}

// non-temporal (aux = nt) stores of K packed pairs (k_paths' L records: default-policy stores
// measured 274 -> 300 us there and made k_south_wta's reads 181 -> 200 us; sc0/sc1 variants of
// the loads and stores measured the same as nt within noise)
template <int K, int AUX = 2>
__device__ __forceinline__ void store_buf_nt(Rsrc r, uint32_t vofs, uint32_t sofs, const Regs<K>& v) {
    if constexpr (K == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v.r[0], r, vofs, sofs, AUX);
    } else if constexpr (K == 2) {
        __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) uint32_t){v.r[0], v.r[1]}, r,
                                              vofs, sofs, AUX);
    } else {
#pragma unroll
        for (int j = 0; j < K / 4; j++)
            __builtin_amdgcn_raw_buffer_store_b128(
                (__attribute__((ext_vector_type(4))) uint32_t){v.r[4 * j], v.r[4 * j + 1], v.r[4 * j + 2],
                                                               v.r[4 * j + 3]},
                r, vofs + 16 * j, sofs, AUX);
    }
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// CUs of the current device (host side), cached per device id: a thread may drive handles on
// several devices, so a per-thread cache of the first device's count would be wrong on another
inline int device_cus() {
    static int cache[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    int cus = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (cus <= 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        __atomic_store_n(&cache[dev], cus, __ATOMIC_RELAXED);
    }
    return cus;
}

// Dispatch-order block index h (of n) -> logical index such that consecutive logical blocks share
// an XCD (and its L2): blocks are dealt round-robin over the 8 XCDs, so h and h + 8 share one
// (MI355X_MICROARCH.md, workgroup dispatch); the XCD of h % 8 gets a contiguous logical range.
__device__ __forceinline__ int xcd_block(int h, int n) {
    const int q = n >> 3, r = n & 7, x = h & 7, k = h >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// Compile-time unrolling of a step functor f(k, integral_constant<J>) over J = 0..N-1 (all steps)
// or over the J with k0 + J <= klast (tail); J is the static ring slot of step k0 + J.
template <typename F, int... J>
__device__ __forceinline__ void unroll_rows(F& f, int k0, std::integer_sequence<int, J...>) {
    (f(k0 + J, std::integral_constant<int, J>{}), ...);
}
template <typename F, int... J>
__device__ __forceinline__ void unroll_rows_tail(F& f, int k0, int klast, std::integer_sequence<int, J...>) {
    ((k0 + J <= klast ? f(k0 + J, std::integral_constant<int, J>{}) : void()), ...);
}

// trunc(n / d) for d >= 1 and |n / d| < 2^20 without a divide loop: float estimate, then one
// exact integer correction step (the subpixel quotients are in [-9, 9]).
__device__ __forceinline__ int div_trunc_small(int n, int d) {
    const int an = abs(n);
    int q = (int)((float)an * __builtin_amdgcn_rcpf((float)d));
    const int r = an - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return n < 0 ? -q : q;
}


// ------------------------------------------------------------------------------------------
// A.12 reprojectImageTo3D of one pixel (sdr_post.hip's kernels, the class path's fused WLS
// epilogue in sdr_wls.hip): double math, sequential sums from 0, no contraction, Vec3f then
// *(1.0/h3) rounded to float; handleMissing: Z = 10000 where |d - min(disp)| <= FLT_EPSILON.
// ------------------------------------------------------------------------------------------
struct Q16 {
    double q[16];
};

__device__ __forceinline__ void reproject_px(const Q16& Q, int x, int y, double d, double mind,
                                             int hm, float* o) {
#pragma clang fp contract(off)
    const double v0 = (double)x, v1 = (double)y;
    double h[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double s = 0.0;
        s += Q.q[i * 4 + 0] * v0;
        s += Q.q[i * 4 + 1] * v1;
        s += Q.q[i * 4 + 2] * d;
        s += Q.q[i * 4 + 3] * 1.0;
        h[i] = s;
    }
    const double ia = 1.0 / h[3];
    const float X = (float)((double)(float)h[0] * ia);
    const float Y = (float)((double)(float)h[1] * ia);
    float Z = (float)((double)(float)h[2] * ia);
    if (hm && fabs(d - mind) <= (double)FLT_EPSILON) Z = 10000.f;
    o[0] = X;
    o[1] = Y;
    o[2] = Z;
}

}  // namespace sdr
