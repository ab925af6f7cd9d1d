// sdr_cloud.hip -- the point-cloud emit after the hot path:
//   convertCVMatToPCL(pointCloud_CV, left)       reference point_cloud/src/pcd_write.cpp:17-51,119
//   pcl::VoxelGrid<PointXYZRGB>::filter          pcd_write.cpp:122-130
//   pcl::io::savePCDFileBinary                   pcd_write.cpp:141
// restating PCL 1.14 the way oracle/pcl_oracle.c does (the checker; parity with PCL unpinned).
//
// Points are PointXYZRGB as savePCDFileBinary lays them out: 16-byte records {x, y, z, rgba}.
//   k_xyz_to_cloud   thread per pixel: 12 B XYZ + 3 B BGR in, 16 B out (HBM-bound, streaming)
//   voxel grid       k_minmax (two-stage, exact float min/max over finite points) -> host decides
//                    PCL's int32-overflow passthrough -> k_voxel_keys (64-bit key = voxel index <<
//                    32 | point index, non-finite last) -> the sort of those keys: a stable LSD
//                    radix sort of the voxel indices (8-bit digits, as many passes as the largest
//                    index needs; points start in index order, so stability gives PCL's (index,
//                    point) order) -> k_voxel_heads + an exclusive scan -> k_voxel_centroid (one
//                    thread per voxel sums its run in point order: the oracle's order, so
//                    centroids match bit for bit).  Sort and scan are hand-written (k_rs_*, k_scan_*):
//                    no library on the path.
#include "../../include/sdr/sdr.h"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#pragma clang fp contract(off)

namespace sdr {

__device__ __forceinline__ bool finite3(float x, float y, float z) {
    return isfinite(x) && isfinite(y) && isfinite(z);
}

__global__ __launch_bounds__(256) void k_xyz_to_cloud(const float* __restrict__ xyz,
                                                      const uint8_t* __restrict__ bgr, int W, int H,
                                                      size_t bstride, size_t bfstride, size_t n,
                                                      float4* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        uint32_t rgba = 0xFF000000u;
        float4 o;
        if (finite3(x, y, z)) {
            o.x = x;
            o.y = y;
            o.z = z;
            if (bgr) {
                const size_t f = i / ((size_t)W * H), r = i % ((size_t)W * H);
                const uint8_t* px = bgr + f * bfstride + (r / W) * bstride + (r % W) * 3;
                rgba |= (uint32_t)px[2] << 16 | (uint32_t)px[1] << 8 | px[0];
            }
        } else {
            o.x = o.y = o.z = __uint_as_float(0x7FC00000u);
        }
        o.w = __uint_as_float(rgba);
        out[i] = o;
    }
}

constexpr int kMinMaxBlocks = 512;

// partial[b] = {min x, y, z, max x, y, z, finite count (as float bits)}
__global__ __launch_bounds__(256) void k_minmax(const float4* __restrict__ p, int n,
                                                float* __restrict__ partial) {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    int cnt = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const float4 q = p[i];
        if (!finite3(q.x, q.y, q.z)) continue;
        cnt++;
        mn[0] = fminf(mn[0], q.x); mn[1] = fminf(mn[1], q.y); mn[2] = fminf(mn[2], q.z);
        mx[0] = fmaxf(mx[0], q.x); mx[1] = fmaxf(mx[1], q.y); mx[2] = fmaxf(mx[2], q.z);
    }
    __shared__ float s[7][256];
    for (int c = 0; c < 3; c++) { s[c][threadIdx.x] = mn[c]; s[3 + c][threadIdx.x] = mx[c]; }
    s[6][threadIdx.x] = __int_as_float(cnt);
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            for (int c = 0; c < 3; c++) {
                s[c][threadIdx.x] = fminf(s[c][threadIdx.x], s[c][threadIdx.x + w]);
                s[3 + c][threadIdx.x] = fmaxf(s[3 + c][threadIdx.x], s[3 + c][threadIdx.x + w]);
            }
            s[6][threadIdx.x] = __int_as_float(__float_as_int(s[6][threadIdx.x]) +
                                               __float_as_int(s[6][threadIdx.x + w]));
        }
        __syncthreads();
    }
    if (threadIdx.x < 7) partial[blockIdx.x * 7 + threadIdx.x] = s[threadIdx.x][0];
}

struct VoxelParams {
    float inv[3];
    int minb[3];
    uint32_t mul1, mul2;
};

__global__ __launch_bounds__(256) void k_voxel_keys(const float4* __restrict__ p, int n, VoxelParams v,
                                                    uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 q = p[i];
    uint64_t k = ~0ull;
    if (finite3(q.x, q.y, q.z)) {
        const int i0 = (int)(floorf(q.x * v.inv[0]) - (float)v.minb[0]);
        const int i1 = (int)(floorf(q.y * v.inv[1]) - (float)v.minb[1]);
        const int i2 = (int)(floorf(q.z * v.inv[2]) - (float)v.minb[2]);
        const uint32_t idx = (uint32_t)i0 + (uint32_t)i1 * v.mul1 + (uint32_t)i2 * v.mul2;
        k = ((uint64_t)idx << 32) | (uint32_t)i;
    }
    keys[i] = k;
}

__global__ __launch_bounds__(256) void k_voxel_heads(const uint64_t* __restrict__ keys, int n,
                                                     int* __restrict__ head) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    head[i] = k != ~0ull && (i == 0 || (keys[i - 1] >> 32) != (k >> 32)) ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_voxel_centroid(const float4* __restrict__ p,
                                                        const uint64_t* __restrict__ keys, int n,
                                                        const int* __restrict__ head,
                                                        const int* __restrict__ pos,
                                                        float4* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !head[i]) return;
    const uint32_t idx = (uint32_t)(keys[i] >> 32);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sr = 0.0f, sg = 0.0f, sb = 0.0f, sa = 0.0f;
    int j = i;
    for (; j < n; j++) {
        const uint64_t k = keys[j];
        if (k == ~0ull || (uint32_t)(k >> 32) != idx) break;
        const float4 q = p[(uint32_t)k];
        const uint32_t c = __float_as_uint(q.w);
        sx += q.x;
        sy += q.y;
        sz += q.z;
        sr += (float)((c >> 16) & 255u);
        sg += (float)((c >> 8) & 255u);
        sb += (float)(c & 255u);
        sa += (float)(c >> 24);
    }
    const float nn = (float)(j - i);
    float4 o;
    o.x = sx / nn;
    o.y = sy / nn;
    o.z = sz / nn;
    o.w = __uint_as_float((uint32_t)(sa / nn) << 24 | (uint32_t)(sr / nn) << 16 |
                          (uint32_t)(sg / nn) << 8 | (uint32_t)(sb / nn));
    out[pos[i]] = o;
}

// ---- exclusive scan of int32 (reduce, scan the block totals, apply) ----------------------------
constexpr int kScanItems = 8, kScanSeg = 256 * kScanItems;

// the block's exclusive prefix of one int per thread (256 threads), and the block total
__device__ __forceinline__ int block_excl_scan(int v, int* total, int* lds /* [4] */) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[w] = x;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int c = lds[i];
        before += i < w ? c : 0;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const int* __restrict__ in, int n, int* __restrict__ partial) {
    __shared__ int lds[4];
    const int base = blockIdx.x * kScanSeg + threadIdx.x * kScanItems;
    int s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) s += base + i < n ? in[base + i] : 0;
    int tot;
    (void)block_excl_scan(s, &tot, lds);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of the nb block totals in place, 256 at a time with a carry
__global__ __launch_bounds__(256) void k_scan_partials(int* __restrict__ partial, int nb) {
    __shared__ int lds[4];
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += 256) {
        const int i = b0 + threadIdx.x;
        const int v = i < nb ? partial[i] : 0;
        int tot;
        const int ex = block_excl_scan(v, &tot, lds);
        if (i < nb) partial[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void k_scan_apply(const int* __restrict__ in, int n, const int* __restrict__ partial,
                                                    int* __restrict__ out) {
    __shared__ int lds[4];
    const int base = blockIdx.x * kScanSeg + threadIdx.x * kScanItems;
    int v[kScanItems], s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        v[i] = base + i < n ? in[base + i] : 0;
        s += v[i];
    }
    int tot;
    int run = partial[blockIdx.x] + block_excl_scan(s, &tot, lds);
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
}

// ---- stable LSD radix sort of (32-bit key, 32-bit value) pairs, 8-bit digits ------------------
constexpr int kRsRounds = 16, kRsTile = 256 * kRsRounds;

// hist[d * nb + b] = keys of tile b with digit d (digit-major: the scan of this array in order is
// every key's bucket start for the stable scatter)
__global__ __launch_bounds__(256) void k_rs_hist(const uint32_t* __restrict__ keys, int n, int shift,
                                                 int* __restrict__ hist, int nb) {
    __shared__ int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRsTile;
    for (int r = 0; r < kRsRounds; r++) {
        const int i = base + r * 256 + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1);
    }
    __syncthreads();
    hist[threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// tile b's keys to their scanned bucket positions in input order: per round of 256 keys, a key's
// rank among the wave's equal digits (8 ballots), the waves before it (their per-digit counts in
// LDS) and the rounds before it (the running bucket starts)
__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    int n, int shift, const int* __restrict__ hist, int nb,
                                                    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
    __shared__ int start[256];
    __shared__ int wcnt[4][256];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    start[t] = hist[t * nb + blockIdx.x];
    const uint64_t lt = (1ull << lane) - 1ull;
    const int base = blockIdx.x * kRsTile;
    for (int r = 0; r < kRsRounds; r++) {
#pragma unroll
        for (int q = 0; q < 4; q++) wcnt[q][t] = 0;
        __syncthreads();
        const int i = base + r * 256 + t;
        const bool valid = i < n;
        const uint32_t k = valid ? keys[i] : 0u;
        const uint32_t v = valid ? vals[i] : 0u;
        const uint32_t d = (k >> shift) & 255u;
        uint64_t m = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bb = __builtin_amdgcn_ballot_w64(valid && ((d >> b) & 1u));
            m &= (d >> b) & 1u ? bb : ~bb;
        }
        const int rank = __popcll(m & lt);
        if (valid && rank == 0) wcnt[w][d] = __popcll(m);
        __syncthreads();
        if (valid) {
            int off = start[d] + rank;
            for (int q = 0; q < w; q++) off += wcnt[q][d];
            keys_out[off] = k;
            vals_out[off] = v;
        }
        __syncthreads();
        start[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    }
}

// the voxel index of a point (prod for the non-finite ones, which sort last) and its index
__global__ __launch_bounds__(256) void k_voxel_split(const uint64_t* __restrict__ keys, int n, uint32_t past,
                                                     uint32_t* __restrict__ k32, uint32_t* __restrict__ v32) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    k32[i] = k == ~0ull ? past : (uint32_t)(k >> 32);
    v32[i] = (uint32_t)i;
}

// back to the 64-bit keys k_voxel_heads / k_voxel_centroid read (voxel << 32 | point, ~0 non-finite)
__global__ __launch_bounds__(256) void k_voxel_join(const uint32_t* __restrict__ k32, const uint32_t* __restrict__ v32,
                                                    int n, uint32_t past, uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = k32[i];
    keys[i] = k == past ? ~0ull : ((uint64_t)k << 32) | v32[i];
}

}  // namespace sdr

namespace {

#define CLOUD_HIP(call)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return sdr::set_error(SDR_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// The voxel grid's scratch: one grow-only device arena a call, leased from a list of idle arenas
// and bump-allocated.  The call reports a count, so it synchronises its stream before it returns
// and its arena goes back to the list idle (the lease synchronises again on an early exit).
// Stream-ordered allocations freed at the end of every call measured 0.75-1.45 ms of host time
// a call on MI355X (the hipFreeAsync calls), more than the grid's kernels take.
struct Arena {
    int dev = 0;
    sdr::Buf buf;
};
std::mutex g_arena_mu;
std::vector<Arena*> g_idle_arenas;

struct ArenaLease {
    hipStream_t st;
    Arena* a = nullptr;
    size_t used = 0;
    explicit ArenaLease(hipStream_t s) : st(s) {}
    // an idle arena of the stream's device with room for `bytes`: SDR_OK or an SDR_* status
    int open(size_t bytes) {
        int dev = 0;
        const hipError_t e = st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev);
        if (e != hipSuccess) return sdr::set_error(SDR_ERR_DEVICE, std::string("device of the stream: ") + hipGetErrorString(e));
        {
            std::lock_guard<std::mutex> lk(g_arena_mu);
            for (size_t i = 0; i < g_idle_arenas.size(); i++) {
                if (g_idle_arenas[i]->dev == dev) {
                    a = g_idle_arenas[i];
                    g_idle_arenas.erase(g_idle_arenas.begin() + i);
                    break;
                }
            }
        }
        if (!a) {
            a = new Arena;
            a->dev = dev;
        }
        return sdr::ensure(a->buf, bytes);  // grows (hipFree + hipMalloc) only past its size
    }
    void* get(size_t bytes) {
        const size_t at = (used + 255) & ~(size_t)255;
        if (!a || at + bytes > a->buf.n) return nullptr;
        used = at + bytes;
        return (char*)a->buf.p + at;
    }
    ~ArenaLease() {
        if (!a) return;
        (void)hipStreamSynchronize(st);  // idle before another call may take it
        std::lock_guard<std::mutex> lk(g_arena_mu);
        g_idle_arenas.push_back(a);
    }
};

}  // namespace

extern "C" {

int sdr_xyz_to_cloud_device(const float* d_xyz, const uint8_t* d_bgr, size_t bgr_stride,
                            size_t bgr_frame_stride, int width, int height, int nframes,
                            void* d_points, void* stream) {
    if (!d_xyz || !d_points) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (width <= 0 || height <= 0 || nframes <= 0) return sdr::set_error(SDR_ERR_ARG, "bad size");
    if (!bgr_stride) bgr_stride = (size_t)width * 3;
    if (!bgr_frame_stride) bgr_frame_stride = bgr_stride * height;
    if (d_bgr && bgr_stride < (size_t)width * 3) return sdr::set_error(SDR_ERR_ARG, "bad BGR stride");
    const size_t n = (size_t)width * height * nframes;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(sdr::k_xyz_to_cloud, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_xyz,
                       d_bgr, width, height, bgr_stride, bgr_frame_stride, n, (float4*)d_points);
    CLOUD_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_voxel_grid_device(const void* d_points, int n, float lx, float ly, float lz, void* d_out,
                          int* out_count, int* passthrough, void* stream) {
    if (!d_points || !d_out || !out_count) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (n < 0) return sdr::set_error(SDR_ERR_ARG, "negative point count");
    if (!(lx > 0.0f) || !(ly > 0.0f) || !(lz > 0.0f)) return sdr::set_error(SDR_ERR_ARG, "leaf size must be > 0");
    hipStream_t st = (hipStream_t)stream;
#ifdef SDR_VOXEL_TIMING  // diagnostic: host-side phase times of one call on stderr
    struct Phases {
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
        char buf[256];
        int len = 0;
        void mark(const char* what) {
            const auto now = std::chrono::steady_clock::now();
            len += std::snprintf(buf + len, sizeof(buf) - len, " %s %.1f", what,
                                 std::chrono::duration<double, std::micro>(now - last).count());
            last = now;
        }
        ~Phases() {
            mark("end");
            std::fprintf(stderr, "voxel_grid us:%s\n", buf);
        }
    } ph;
#define VOXEL_MARK(w) ph.mark(w)
#else
#define VOXEL_MARK(w) (void)0
#endif
    const float4* p = (const float4*)d_points;
    float4* out = (float4*)d_out;
    *out_count = 0;
    if (passthrough) *passthrough = 0;
    if (n == 0) return SDR_OK;
    // the arena holds everything below: the min/max partials, then the keys, the sort's ping-pong
    // (voxel, point) arrays, the heads and positions, the sort's histograms and the scan's totals
    const size_t un = (size_t)n;
    const int nb_rs = (n + sdr::kRsTile - 1) / sdr::kRsTile;
    const int nh = 256 * nb_rs;
    const int nb_scan = (std::max(n, nh) + sdr::kScanSeg - 1) / sdr::kScanSeg;
    const size_t need = sizeof(float) * 7 * sdr::kMinMaxBlocks + un * (8 + 8 + 4 + 4 + 4 * 4) +
                        sizeof(int) * ((size_t)nh + nb_scan) + 11 * 256;
    ArenaLease scratch(st);
    int rc = scratch.open(need);
    if (rc) return rc;
    float* partial = (float*)scratch.get(sizeof(float) * 7 * sdr::kMinMaxBlocks);
    if (!partial) return sdr::set_error(SDR_ERR_NOMEM, "scratch allocation failed");
    const int mmb = std::min(sdr::kMinMaxBlocks, (n + 255) / 256);
    hipLaunchKernelGGL(sdr::k_minmax, dim3(mmb), dim3(256), 0, st, p, n, partial);
    CLOUD_HIP(hipGetLastError());
    std::vector<float> hp((size_t)7 * mmb);
    CLOUD_HIP(hipMemcpyAsync(hp.data(), partial, sizeof(float) * hp.size(), hipMemcpyDeviceToHost, st));
    VOXEL_MARK("mm_launch");
    CLOUD_HIP(hipStreamSynchronize(st));
    VOXEL_MARK("mm_sync");
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    long long nfin = 0;
    for (int b = 0; b < mmb; b++) {
        for (int c = 0; c < 3; c++) {
            mn[c] = std::fmin(mn[c], hp[b * 7 + c]);
            mx[c] = std::fmax(mx[c], hp[b * 7 + 3 + c]);
        }
        int cnt;
        std::memcpy(&cnt, &hp[b * 7 + 6], 4);
        nfin += cnt;
    }
    if (!nfin) return SDR_OK;  // nothing finite: empty output
    const float inv[3] = {1.0f / lx, 1.0f / ly, 1.0f / lz};
    long long d[3];
    for (int c = 0; c < 3; c++) d[c] = (long long)((mx[c] - mn[c]) * inv[c]) + 1;
    const long long prod = (long long)((unsigned long long)d[0] * (unsigned long long)d[1] *
                                       (unsigned long long)d[2]);
    if (prod > 2147483647LL) {
        // PCL: "Leaf size is too small for the input dataset. Integer indices would overflow." --
        // the output is the input cloud unchanged
        CLOUD_HIP(hipMemcpyAsync(out, p, sizeof(float4) * (size_t)n, hipMemcpyDeviceToDevice, st));
        CLOUD_HIP(hipStreamSynchronize(st));
        *out_count = n;
        if (passthrough) *passthrough = 1;
        return SDR_OK;
    }
    sdr::VoxelParams v;
    int div[3];
    for (int c = 0; c < 3; c++) {
        v.inv[c] = inv[c];
        v.minb[c] = (int)std::floor(mn[c] * inv[c]);
        const int maxb = (int)std::floor(mx[c] * inv[c]);
        div[c] = maxb - v.minb[c] + 1;
    }
    v.mul1 = (uint32_t)div[0];
    v.mul2 = (uint32_t)div[0] * (uint32_t)div[1];
    uint64_t* keys = (uint64_t*)scratch.get(sizeof(uint64_t) * n);
    uint64_t* sorted = (uint64_t*)scratch.get(sizeof(uint64_t) * n);
    int* head = (int*)scratch.get(sizeof(int) * n);
    int* pos = (int*)scratch.get(sizeof(int) * n);
    // the sort's ping-pong (voxel, point) arrays and its histograms; the scan's block totals
    uint32_t* kv[4];
    for (auto& q : kv) q = (uint32_t*)scratch.get(sizeof(uint32_t) * n);
    int* hist = (int*)scratch.get(sizeof(int) * nh);
    int* spart = (int*)scratch.get(sizeof(int) * nb_scan);
    if (!keys || !sorted || !head || !pos || !kv[0] || !kv[1] || !kv[2] || !kv[3] || !hist || !spart)
        return sdr::set_error(SDR_ERR_NOMEM, "scratch allocation failed");
    VOXEL_MARK("alloc");
    const dim3 grid((n + 255) / 256);
    auto scan = [&](const int* in, int m, int* o) {
        const int nb = (m + sdr::kScanSeg - 1) / sdr::kScanSeg;
        hipLaunchKernelGGL(sdr::k_scan_reduce, dim3(nb), dim3(256), 0, st, in, m, spart);
        hipLaunchKernelGGL(sdr::k_scan_partials, dim3(1), dim3(256), 0, st, spart, nb);
        hipLaunchKernelGGL(sdr::k_scan_apply, dim3(nb), dim3(256), 0, st, in, m, spart, o);
    };
    hipLaunchKernelGGL(sdr::k_voxel_keys, grid, dim3(256), 0, st, p, n, v, keys);
    // voxel indices are below div0 * div1 * div2 (each div at most one above PCL's d, whose product
    // passed the overflow check); `past` = that bound marks the non-finite points, which sort last
    const unsigned long long divprod = (unsigned long long)div[0] * (unsigned long long)div[1] * (unsigned long long)div[2];
    const uint32_t past = divprod < 0xFFFFFFFFull ? (uint32_t)divprod : 0xFFFFFFFFu;
    int bits = 1;
    while (bits < 32 && (past >> bits) != 0) bits++;
    hipLaunchKernelGGL(sdr::k_voxel_split, grid, dim3(256), 0, st, keys, n, past, kv[0], kv[1]);
    int cur = 0;
    for (int shift = 0; shift < bits; shift += 8) {
        hipLaunchKernelGGL(sdr::k_rs_hist, dim3(nb_rs), dim3(256), 0, st, kv[cur], n, shift, hist, nb_rs);
        scan(hist, nh, hist);
        hipLaunchKernelGGL(sdr::k_rs_scatter, dim3(nb_rs), dim3(256), 0, st, kv[cur], kv[cur + 1], n, shift, hist,
                           nb_rs, kv[2 - cur], kv[3 - cur]);
        cur = 2 - cur;
    }
    hipLaunchKernelGGL(sdr::k_voxel_join, grid, dim3(256), 0, st, kv[cur], kv[cur + 1], n, past, sorted);
    hipLaunchKernelGGL(sdr::k_voxel_heads, grid, dim3(256), 0, st, sorted, n, head);
    scan(head, n, pos);
    hipLaunchKernelGGL(sdr::k_voxel_centroid, grid, dim3(256), 0, st, p, sorted, n, head, pos, out);
    CLOUD_HIP(hipGetLastError());
    VOXEL_MARK("launches");
    int last_pos = 0, last_head = 0;
    CLOUD_HIP(hipMemcpyAsync(&last_pos, pos + n - 1, 4, hipMemcpyDeviceToHost, st));
    CLOUD_HIP(hipMemcpyAsync(&last_head, head + n - 1, 4, hipMemcpyDeviceToHost, st));
    VOXEL_MARK("copies");
    CLOUD_HIP(hipStreamSynchronize(st));
    VOXEL_MARK("sync");
    *out_count = last_pos + last_head;
    return SDR_OK;
}

int sdr_pcd_header(int width, int height, char* buf, size_t cap) {
    // PCDWriter::generateHeader for PointXYZRGB (rgb written as TYPE U) + writeBinary's DATA line
    char tmp[512];
    const int len = std::snprintf(
        tmp, sizeof(tmp),
        "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\nSIZE 4 4 4 4\n"
        "TYPE F F F U\nCOUNT 1 1 1 1\nWIDTH %d\nHEIGHT %d\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS %lld\n"
        "DATA binary\n",
        width, height, (long long)width * height);
    if (len < 0) return sdr::set_error(SDR_ERR_ARG, "header formatting failed");
    if (buf) {
        if (cap < (size_t)len + 1) return sdr::set_error(SDR_ERR_ARG, "header buffer too small");
        std::memcpy(buf, tmp, (size_t)len + 1);
    }
    return len;
}

int sdr_write_pcd_binary(const char* path, const void* points, int width, int height) {
    if (!path || (!points && width * height > 0)) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (width < 0 || height < 0) return sdr::set_error(SDR_ERR_ARG, "bad size");
    char hdr[512];
    const int len = sdr_pcd_header(width, height, hdr, sizeof(hdr));
    if (len < 0) return len;
    FILE* f = std::fopen(path, "wb");
    if (!f) return sdr::set_error(SDR_ERR_ARG, std::string("cannot open ") + path);
    const size_t nbytes = (size_t)width * height * 16;
    const bool ok = std::fwrite(hdr, 1, (size_t)len, f) == (size_t)len &&
                    (nbytes == 0 || std::fwrite(points, 1, nbytes, f) == nbytes);
    if (std::fclose(f) != 0 || !ok) return sdr::set_error(SDR_ERR_DEVICE, std::string("write failed: ") + path);
    return SDR_OK;
}

}  // extern "C"
