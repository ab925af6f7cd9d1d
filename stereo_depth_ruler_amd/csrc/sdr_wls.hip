// sdr_wls.hip -- the class path's post-filter on the GPU:
//   cv::ximgproc::createDisparityWLSFilter(matcher)    stereo_vision/src/stereo_disparity.cpp:11-13
//   wls_filter->filter(disp_left, left_small, filtered, disp_right)               :31
//   wls_filter->getConfidenceMap()                                                :36
// restating opencv_contrib 4.6 ximgproc disparity_filters.cpp + fgs_filter.cpp as the oracle
// does (oracle/wls_oracle.c, the checker; parity against OpenCV itself is unpinned there).
//
// Kernels (all float work with contraction off and IEEE division, so every rounding matches the
// oracle's operation order bit for bit; the FGS weight table is computed once on the host with
// the same expf the oracle uses):
//   k_wls_disc     depth-discontinuity map of the RIGHT view over its ROI: 1 - roll_off * var
//                  of a (2r+1)^2 box, BORDER_REFLECT_101 inside the ROI, sums in int64/double
//   k_wls_conf     left discontinuity (inline) + discontinuity-aware LR check -> confidence
//                  x255 (full map for getConfidenceMap) and the two FGS inputs conf*d, conf,
//                  compacted to the ROI
//   k_fgs_pcr      one FGS pass (rows or columns), the default solver (SDR_FGS_PCR): every line's
//                  tridiagonal system solved by parallel cyclic reduction in LDS, a 256-thread
//                  workgroup per line (or per G short lines), both right-hand sides at once, the
//                  diagonal carried as the row sum (oracle/wls_oracle.c fgs_line_pcr: every term
//                  non-negative, ~200x closer to the exact solution than the sequential sweep);
//                  rows and columns are both read in place from the row-major images
//   k_fgs_sweep    one FGS pass with the sequential solver (SDR_FGS_THOMAS, ximgproc's own
//                  elimination order, bit-exact with oracle/wls_oracle.c fgs_line): lane = line
//                  over k-major data, PF samples loaded ahead in registers; one lane per line
//                  leaves the chip nearly idle (6-9 waves at 640x360: ~112 us per pass)
//   k_transpose2   LDS-tiled transposes between the sweep's column-major copies and the row-major
//                  images; k_fgs_weights builds the weights once per frame
//   k_wls_final    FGS(conf*d) / FGS(conf) -> saturate_cast<short>, 16*(min_disp-1) outside ROI
#include "../../include/sdr/sdr.h"
#include "sdr_device.hpp"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#pragma clang fp contract(off)

namespace sdr {

constexpr int kFgsLevels = 65026;  // 255^2 + 1 squared differences of two 8-bit gray levels

// the sequential solver's k-major arrays keep their sample rows 16-byte aligned: line counts and
// line lengths rounded up to 4 (frames fgs_pad4(w) * fgs_pad4(h) samples apart)
__host__ __device__ __forceinline__ int fgs_pad4(int x) { return (x + 3) & ~3; }

__device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

// 1 - roll_off * (boxmean(d^2) - boxmean(d)^2), clamped at 0, at ROI pixel (i, j) of map d
// (ComputeDepthDisc: convertTo(CV_32F), multiply, boxFilter(CV_32F) x2 with double row sums)
__device__ __forceinline__ float disc_at(const int16_t* __restrict__ d, int W, int rx, int ry,
                                         int rw, int rh, int i, int j, int radius, double scale,
                                         float roll_off) {
    long long s = 0, s2 = 0;
    for (int a = -radius; a <= radius; a++) {
        const int ii = reflect101(i + a, rh);
        const int16_t* row = d + (size_t)(ry + ii) * W + rx;
        for (int b = -radius; b <= radius; b++) {
            const long long v = row[reflect101(j + b, rw)];
            s += v;
            s2 += v * v;
        }
    }
    const float mean = (float)((double)s * scale);
    const float msq = (float)((double)s2 * scale);
    const float var = msq - mean * mean;
    const float c = 1.0f - roll_off * var;
    return c > 0.0f ? c : 0.0f;
}

struct WlsGeom {
    int W, H;
    int rx, ry, rw, rh;      // left ROI
    int rrx;                 // right ROI x (same y, w, h)
    int radius;
    double scale;            // 1 / (2r+1)^2
    float roll_off;
    int lrc_thresh;
    int fill;                // 16 * (min_disp - 1)
};

// The filter's outputs (the class path's epilogue: fout = out / 16, xyz = reprojectImageTo3D(fout,
// Q), both nullable), written by whichever kernel holds a pixel's final value: k_wls_final, or,
// with SDR_FGS_PCR, k_wls_prep (pixels outside the ROI) and the last FGS column pass (the ROI).
struct WlsOut {
    int16_t* out;
    float* fout;
    float* xyz;
    Q16 Q;
};

// saturate_cast<short>(FGS(conf*d) / FGS(conf)) (cv::divide of floats: 0 for a zero divisor;
// cvRound = cvtss2si: NaN / |v| >= 2^31 give INT_MIN, which saturates to -32768)
__device__ __forceinline__ int16_t wls_value(float a, float c) {
    const float v = c != 0.0f ? a / c : 0.0f;
    float q = rintf(v);
    q = fminf(fmaxf(q, -32768.0f), 32767.0f);
    return fabsf(v) < 2147483648.0f ? (int16_t)(int)q : (int16_t)-32768;
}

// pixel (x, y) of frame f: the int16 value and the epilogue
__device__ __forceinline__ void wls_emit(const WlsOut& o, const WlsGeom& g, int f, int x, int y, int16_t r) {
    const size_t p = (size_t)f * g.W * g.H + (size_t)y * g.W + x;
    o.out[p] = r;
    if (o.fout) {
        const float df = (float)r * 0.0625f;
        o.fout[p] = df;
        if (o.xyz) reproject_px(o.Q, x, y, (double)df, 0.0, 0, o.xyz + 3 * p);
    }
}

__global__ __launch_bounds__(256) void k_wls_disc(const int16_t* __restrict__ dr, WlsGeom g,
                                                  float* __restrict__ rdisc) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (j >= g.rw || i >= g.rh) return;
    const size_t fo = (size_t)blockIdx.z * g.W * g.H;
    rdisc[fo + (size_t)(g.ry + i) * g.W + g.rrx + j] =
        disc_at(dr + fo, g.W, g.rrx, g.ry, g.rw, g.rh, i, j, g.radius, g.scale, g.roll_off);
}

// ComputeDiscontinuityAwareLRC + confidence_map = 255 * map; A = conf * d, B = conf (ROI-compact)
__global__ __launch_bounds__(256) void k_wls_conf(const int16_t* __restrict__ dl,
                                                  const int16_t* __restrict__ dr,
                                                  const float* __restrict__ rdisc, WlsGeom g,
                                                  float* __restrict__ conf_full,
                                                  float* __restrict__ A, float* __restrict__ B) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const size_t fo = (size_t)blockIdx.z * g.W * g.H;
    const size_t o = fo + (size_t)y * g.W + x;
    const int j = x - g.rx, i = y - g.ry;
    const bool in_roi = j >= 0 && j < g.rw && i >= 0 && i < g.rh;
    float c = 1.0f;
    int v = 0;
    if (in_roi) {
        c = disc_at(dl + fo, g.W, g.rx, g.ry, g.rw, g.rh, i, j, g.radius, g.scale, g.roll_off);
        v = dl[o];
        const int ridx = x - (v >> 4);
        if (ridx >= g.rrx && ridx < g.rrx + g.rw) {
            const size_t ro = fo + (size_t)y * g.W + ridx;
            if (abs(v + (int)dr[ro]) < g.lrc_thresh) {
                const float rc = rdisc[ro];
                c = c < rc ? c : rc;
            } else {
                c = 0.0f;
            }
        }
    }
    const float conf = 255.0f * c;
    if (conf_full) conf_full[o] = conf;
    if (in_roi) {
        const size_t co = (size_t)blockIdx.z * g.rw * g.rh + (size_t)i * g.rw + j;
        A[co] = conf * (float)v;
        B[co] = conf;
    }
}

// FGS line solve, per line of n samples with weights C[k] = lut[(g[k] - g[k+1])^2] (0 at the
// last sample):  (1 - lam*(C[k-1] + C[k])) u_k + lam*C[k-1] u_{k-1} + lam*C[k] u_{k+1} = f_k
// (C = -w <= 0), Thomas forward elimination then back substitution, in the oracle's order
// (oracle/wls_oracle.c fgs_line, ximgproc's fgs_filter.cpp sweep):
//   k=0:  den = 1 - lam*C0;  t0 = lam*C0 / den;  u0 = u0 / den
//   k>0:  a = lam*C[k-1];  c = lam*C[k];  den = (1 - c) - a*(1 + t[k-1]);
//         t[k] = c / den;  u_k = (u_k - a*u_{k-1}) / den
//   back: u_k = u_k - t[k]*u_{k+1}
// The elimination coefficients (den, t) depend on the guide's weights and lambda only, not on the
// right-hand sides: one launch of coefficient jobs computes them for every pass of a filter first
// (the t recurrence, ~13 dependent operations a sample with its IEEE division, and 1/den beside
// it), and the passes then run only the right-hand sides' recurrence, with the division x / den
// done from the correctly rounded reciprocal r = 1/den:
//   q0 = x*r,  rem = -fma(q0, den, -x) (exact),  q = fma(rem, r, q0)
// which is the correctly rounded quotient (Markstein's theorem: r within half an ulp of 1/den and
// q0 within an ulp of x/den; den >= 1 here) as long as nothing underflows: for 0 < |q0| < 2^-96 a
// chunk runs again with real divisions; scripts/markstein_check.c finds no difference at or above
// that threshold in 2e9 random pairs (den up to 2^60).  Five dependent operations a sample.
//
// A pass of F frames x nl lines runs as a chain on one wave per workgroup (lane = line, LPB = 16,
// 32 or 64 lines a workgroup), which touches nothing but LDS, with three helper waves:
//   wave 0    the solver: the recurrence of its LPB lines sample by sample, each sample's operands
//             read from the LDS ring kThPF samples ahead (ds_read latency off the chain), each
//             result written to an LDS row for the writer
//   waves 1-2 loaders: LDS-DMA (global_load_lds_dwordx4, 1 KiB a wave-instruction) of the next
//             chunks (CH = 1024 / LPB samples x LPB lines of every operand stream) into a ring of
//             kThNB buffers, up to kThNB - 2 chunks in flight
//   wave 3    the writer: every global store of the pass -- the forward values (k-major, in place)
//             and the results (line-major: the next pass's k-major layout, the transpose between
//             passes done by reading the rows transposed; or k-major into the two outputs)
// One s_barrier per chunk orders them: chunk c + 2 has landed (loaders' counted vmcnt), the solver
// is done with chunk c - 1's buffer and has written chunk c's rows before the barrier that ends
// iteration c.  Measured at 640x360 (a 560x360 ROI, two right-hand sides): 64 lines a workgroup
// with the solver storing its own results, 96 us a pass; 16 lines, 77 us; 16 lines with the
// stores on the writer wave, 39 us (the solver's stores queued behind the loaders' DMA in the
// CU's memory pipeline: a variant without them ran 45 us at 77).
// Layout: every k-major array (element (line l, sample k) at k * st + l, st = nl rounded up to 4)
// has 16-byte aligned sample rows, which the 16-byte DMA needs; the frames are fs apart.
constexpr int kThNB = 5;          // LDS ring buffers
constexpr int kThPF = 8;          // the solver's LDS lookahead (samples)
constexpr int kThBuf = 1024 * 24; // a chunk (1024 line-samples) of the largest stream set
template <int LPB, int ES> struct ThRows {
    // the solver's back-substitution rows: CH samples x LPB lines, double-buffered; the row stride
    // S (dwords) is = E * LPB / 16 (mod 64), so that the writer's transposed reads (CH samples of
    // 64 / CH lines a wave-instruction) fall on distinct banks
    static constexpr int CH = 1024 / LPB, E = ES / 4;
    static constexpr int S = LPB * E + (64 - (LPB * E) % 64) % 64 + E * LPB / 16;
    static constexpr int bytes = 2 * CH * S * 4;
};
constexpr int kThRows = ThRows<16, 8>::bytes;  // the rows area (the largest use)
constexpr int kThLds = kThNB * kThBuf + kThRows;
static_assert(ThRows<32, 8>::bytes <= kThRows && ThRows<64, 8>::bytes <= kThRows, "rows");
static_assert(kThRows >= 2 * 1024 * 16, "the forward and job rows fit the rows area");
// two flag words (chunk parity) in the rows area's last bytes -- padding of the back substitution's
// last row, clear of the job rows: a job chunk to run with IEEE divisions
constexpr int kThFlags = kThRows - 16;

static_assert(2 * 1024 * 16 <= kThFlags && ThRows<16, 8>::S * 4 - 16 >= 16 * 8, "flags in the rows' padding");
static_assert(kThLds <= 160 * 1024, "one workgroup's LDS");
constexpr int kFgsMaxJobs = 8;         // coefficient jobs in one launch
constexpr size_t kFgsOverread = 4096;  // bytes past a k-major array the loaders may read (the
                                       // last workgroup's lines beyond st, at the last sample)
constexpr double kFgsThomasMaxLambda = 0x1p100;  // pivots below 2^126 (fgs_rcp)
constexpr uint32_t kFgsTinyKey = 0x1EFFFFFFu;  // fgs_tiny_key(q) < this <=> 0 < |q| < 2^-96

// The correctly rounded 1/d for 1 <= d < 2^126: v_rcp_f32 and one Newton step, equal to the IEEE
// quotient 1.0f / d for every mantissa of d at every exponent checked (sdr_fgs_rcp_selftest,
// tests/test_gpu_wls.py; at 2^126 and beyond 1/d is subnormal and it is not) -- 3 operations
// instead of the IEEE division's ~11.  Every pivot is at most 1 + 2 * lambda, hence
// kFgsThomasMaxLambda.
__device__ __forceinline__ float fgs_rcp(float d) {
    const float r0 = __builtin_amdgcn_rcpf(d);
    return __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
}

// 2|q| - 1 as an integer (the sign bit shifted out): below kFgsTinyKey exactly when 0 < |q| < 2^-96
// (+-0 wraps to the largest key); the minimum over a chunk decides the redo
__device__ __forceinline__ uint32_t fgs_tiny_key(float q) { return __builtin_bit_cast(uint32_t, q) * 2u - 1u; }

struct FgsCoefJob {
    const float* Cw;  // the pass's weights, k-major
    float4* coef;     // [F] frames of (a, den, 1/den, t), k-major
    float* tt;        // [F] frames of t, k-major (the back substitution's stream)
    float lam;
    int nl, n;
    int st;           // k-major sample stride (nl rounded up to 4)
    int blocks;
    int lpb;          // k_fgs_lrjob: lines a workgroup (16, 8 or 4)
};

struct FgsThArgs {
    void* U;                // k-major right-hand sides: float, or float2 (two, interleaved); the
                            // forward values are written back in place
    const float4* coef;     // this pass's (a, den, 1/den, t) ...
    const float* tt;        // ... and t
    void* O;                // line-major results (same element type as U; line stride onp), or
                            // null: ...
    float* O0;              // ... k-major results split into two arrays (the last pass; sample
    float* O1;              // stride ost, frames ofs apart)
    int nl, n;
    int st;                 // k-major sample stride of U, coef, tt
    int onp;                // O's line stride (n rounded up to 4: the next pass's st)
    size_t fs;              // frame stride of U, coef, tt, O
    size_t ost, ofs;
    int dbg;                // diagnostic builds (SDR_TH_STAMPS): the k_fgs_lr stamp slot
    int main_blocks;        // blocks of the pass itself; blocks past them run coefficient jobs
    int njobs;
    FgsCoefJob job[kFgsMaxJobs];
};

template <bool TWO> struct FgsRhs;
template <> struct FgsRhs<true> {
    typedef float2 T;
    static __device__ __forceinline__ float x(const T& v) { return v.x; }
    static __device__ __forceinline__ float y(const T& v) { return v.y; }
    static __device__ __forceinline__ T make(float a, float b) { return make_float2(a, b); }
};
template <> struct FgsRhs<false> {
    typedef float T;
    static __device__ __forceinline__ float x(const T& v) { return v; }
    static __device__ __forceinline__ float y(const T&) { return 0.0f; }
    static __device__ __forceinline__ T make(float a, float) { return a; }
};

typedef __attribute__((address_space(3))) void* th_lds_ptr;
typedef __attribute__((address_space(1))) void* th_glb_ptr;

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
template <int N> __device__ __forceinline__ void th_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// s_waitcnt lgkmcnt(0) alone: the solver's LDS rows are written before the barrier
__device__ __forceinline__ void th_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }
// the workgroup barrier without the fence __syncthreads() carries (whose vmcnt(0) would drain the
// loaders' DMA in flight); the empty asm keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void th_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

#ifdef SDR_TH_STAMPS
// diagnostic build only: s_memtime stamps of workgroup (0, 0) of one launch (scripts/th_stamps.py)
__device__ unsigned long long* g_th_stamps;
#define TH_STAMP(role, idx)                                                                       \
    do {                                                                                          \
        if (g_th_stamps && blockIdx.x == 0 && blockIdx.y == 0 && (threadIdx.x & 63) == 0)         \
            g_th_stamps[(role) * 1024 + (idx)] = __builtin_amdgcn_s_memtime();                    \
    } while (0)
constexpr int kThStampRoles = 6;
__device__ unsigned long long g_th_blk[512][3];  // per workgroup of the stamped launch: start, fwd end, end
#define TH_BLK(i)                                                                                  \
    do {                                                                                           \
        if (g_th_stamps && blockIdx.y == 0 && (threadIdx.x & 63) == 0 && blockIdx.x < 512)         \
            g_th_blk[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                                \
    } while (0)
__device__ unsigned int g_th_counts[4];  // pass chunks: reciprocal form, exact from the start, redone
#define TH_COUNT(i)                                                                                \
    do {                                                                                           \
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_th_counts[i], 1u);                               \
    } while (0)
#else
#define TH_STAMP(role, idx) \
    do {                    \
    } while (0)
#define TH_COUNT(i) \
    do {            \
    } while (0)
#define TH_BLK(i) \
    do {          \
    } while (0)
#endif

// A loader wave's share (lw = 0, 1) of one stream's chunk image: CH = 1024 / LPB sample rows of
// LPB lines x ES bytes, ES wave-instructions of 1 KiB, the wave taking every other one.  Slot j
// holds sample k0 + dk * j (clamped into the line: the slots past its end are never read).
template <int LPB, int ES>
__device__ __forceinline__ void th_issue(const char* g, size_t st, int l0, int k0, int dk, int last, char* img,
                                         int lw, int lane) {
    constexpr int SB = LPB * ES;  // bytes of a slot
    static_assert(ES % 2 == 0 && SB % 16 == 0, "two loader waves, whole pieces");
#pragma unroll
    for (int q = 0; q < ES / 2; q++) {
        const int ii = 2 * q + lw;  // wave-uniform
        const int off = ii * 1024 + lane * 16;
        const int j = off / SB, b = off - j * SB;
        const int k = min(max(k0 + dk * j, 0), last);
        const char* src = g + ((size_t)k * st + l0) * ES + b;
        __builtin_amdgcn_global_load_lds((th_glb_ptr)src, (th_lds_ptr)(img + ii * 1024), 16, 0, 0);
    }
}

// waits until at most m of the wave's younger chunks (IW instructions each) are in flight
template <int IW> __device__ __forceinline__ void th_wait_chunks(int m) {
    static_assert(kThNB == 5, "m <= kThNB - 3");
    if (m >= 2) th_vmcnt<2 * IW>();
    else if (m == 1) th_vmcnt<IW>();
    else th_vmcnt<0>();
}

// A loader wave over one phase of nch chunks (chunk c = samples k0 + dk * (c * CH + j)): chunks
// 0 .. kThNB-2 ahead, then per iteration c chunk c + kThNB - 1 into the buffer chunk c - 1 left,
// and chunk c + 2 landed before the barrier; 1 + extra + nch barriers, as every wave of the phase.
// (not inlined: with the loaders' DMA in the kernel body the compiler's wait analysis, merging
// paths, put a vmcnt(0) before LDS writes of the other waves' code -- every row of a job)
template <int LPB, int ES0, int ES1>
__device__ __noinline__ void th_load_phase(const char* g0, const char* g1, size_t st, int l0, int k0, int dk,
                                              int last, int nch, char* lds, int lw, int lane, int extra = 0) {
    constexpr int CH = 1024 / LPB, IW = (ES0 + ES1) / 2;
    auto issue = [&](int c) __attribute__((always_inline)) {
        char* buf = lds + (c % kThNB) * kThBuf;
        th_issue<LPB, ES0>(g0, st, l0, k0 + dk * c * CH, dk, last, buf, lw, lane);
        if constexpr (ES1 > 0) th_issue<LPB, ES1>(g1, st, l0, k0 + dk * c * CH, dk, last, buf + 1024 * ES0, lw, lane);
    };
    const int pre = min(kThNB - 1, nch);
    for (int c = 0; c < pre; c++) issue(c);
    th_wait_chunks<IW>(pre - 2);
    th_barrier();
    for (int i = 0; i < extra; i++) th_barrier();  // (a job's flag barrier)
    for (int c = 0; c < nch; c++) {
        if (c + kThNB - 1 < nch) issue(c + kThNB - 1);
        if (lw == 0) TH_STAMP(2, (dk < 0 ? 512 : 0) + c);
        th_wait_chunks<IW>(min(c + kThNB - 1, nch - 1) - (c + 2));
        if (lw == 0) TH_STAMP(3, (dk < 0 ? 512 : 0) + c);
        th_barrier();
    }
}

// The writer wave: the solver's rows of chunk c (double-buffered by chunk parity) go to memory
// during iteration c + 1, the last chunk's after the phase's final barrier.
//   fwd:  row j = sample c * CH + j of the forward values, k-major in place (a row = the block's
//         LPB lines, contiguous); all in memory (vmcnt(0)) before the barrier that ends the phase,
//         since the back substitution's loaders read them
//   back: row j = sample kb - j, kb = last - 1 - c * CH, in the padded ThRows layout: line-major
//         into O (a wave-instruction: CH consecutive samples of 64 / CH lines) or k-major split
//         into O0 / O1 (the last pass)
//   job:  row j = (a, den, 1/den, t) of sample c * CH + j -> coef and tt, k-major
template <bool TWO, int LPB>
__device__ __forceinline__ void th_write_fwd_phase(void* U, size_t st, size_t fofs, int l0, int nl, int last, int nch,
                                                   const char* orow, int lane) {
    typedef typename FgsRhs<TWO>::T V;
    constexpr int ES = TWO ? 8 : 4, CH = 1024 / LPB;
    const int line = lane % LPB;
    const bool lv = l0 + line < nl;
    V* u = (V*)U + fofs + l0 + line;
    auto put = [&](int c) __attribute__((always_inline)) {
        const char* rows = orow + (c & 1) * 1024 * ES;
#pragma unroll 4
        for (int it = 0; it < 16; it++) {
            const int jj = it * (64 / LPB) + lane / LPB;
            const int k = c * CH + jj;
            if (lv && k <= last) u[(size_t)k * st] = *(const V*)(rows + (jj * LPB + line) * ES);
        }
    };
    th_barrier();
    for (int c = 0; c < nch; c++) {
        if (c > 0) put(c - 1);
        TH_STAMP(4, c);
        th_barrier();
    }
    if (nch > 0) put(nch - 1);
    th_vmcnt<0>();
}

template <bool TWO, int LPB>
__device__ __forceinline__ void th_write_back_phase(const FgsThArgs& a, size_t fofs, int l0, int last, int nch,
                                                    const char* orow, int lane) {
    typedef typename FgsRhs<TWO>::T V;
    constexpr int ES = TWO ? 8 : 4;
    typedef ThRows<LPB, ES> RW;
    constexpr int CH = RW::CH;
    auto put = [&](int c) __attribute__((always_inline)) {
        const char* rows = orow + (c & 1) * CH * RW::S * 4;
        const int kb = last - 1 - c * CH;
        if (a.O) {
            const int cnt = min(CH, kb + 1), kmin = kb - cnt + 1;
            const int s = lane % CH;
#pragma unroll 4
            for (int it = 0; it < 16; it++) {
                const int line = it * (64 / CH) + lane / CH;
                if (s < cnt && l0 + line < a.nl) {
                    const int k = kmin + s;
                    const V v = *(const V*)(rows + (kb - k) * RW::S * 4 + line * ES);
                    ((V*)a.O)[fofs + (size_t)(l0 + line) * a.onp + k] = v;
                }
            }
        } else {
            const int line = lane % LPB;
            const size_t fo = (size_t)blockIdx.y * a.ofs + l0 + line;
#pragma unroll 4
            for (int it = 0; it < 16; it++) {
                const int jj = it * (64 / LPB) + lane / LPB;
                const int k = kb - jj;
                if (k >= 0 && l0 + line < a.nl) {
                    const V v = *(const V*)(rows + jj * RW::S * 4 + line * ES);
                    a.O0[fo + (size_t)k * a.ost] = FgsRhs<TWO>::x(v);
                    if constexpr (TWO) a.O1[fo + (size_t)k * a.ost] = FgsRhs<TWO>::y(v);
                }
            }
        }
    };
    th_barrier();
    for (int c = 0; c < nch; c++) {
        if (c > 0) put(c - 1);
        th_barrier();
    }
    if (nch > 0) put(nch - 1);
}

// A coefficient job.  Its pivots' reciprocal is fgs_rcp and t = cc / den comes from it
// (Markstein) -- exact unless cc / den can fall below ~2^-96, which happens only when cc = lam * C
// is tiny (the weights of gray-level steps of ~80 and more at sigma 1.1).  The writer flags each
// chunk holding such a weight on any of the workgroup's lines (kThFlags in LDS, one word per
// chunk parity; chunk c + 1's during iteration c, chunk 0's between two prologue barriers) and the
// solver runs a flagged chunk with IEEE divisions, a clean one with no per-sample test or branch
// (a branch a sample cost more than the divisions it saved: 63 us a 560-sample job launch on a
// noise guide, 48 on a scene).

template <int LPB>
__device__ __forceinline__ void th_write_job_phase(const FgsCoefJob& J, size_t fofs, int l0, int nch, const char* lds,
                                                   char* orow, int lane) {
    constexpr int CH = 1024 / LPB;
    const int line = lane % LPB, last = J.n - 1;
    const bool lv = l0 + line < J.nl;
    float4* co = J.coef + fofs + l0 + line;
    float* tt = J.tt + fofs + l0 + line;
    const size_t st = (size_t)J.st;
    const float lam = J.lam, tiny = 0x1p-96f * (1.0f + 2.0f * lam);
    auto put = [&](int c) __attribute__((always_inline)) {
        const char* rows = orow + (c & 1) * 1024 * 16;
#pragma unroll 4
        for (int it = 0; it < 16; it++) {
            const int jj = it * (64 / LPB) + lane / LPB;
            const int k = c * CH + jj;
            if (lv && k <= last) {
                const float4 v = *(const float4*)(rows + (jj * LPB + line) * 16);
                co[(size_t)k * st] = v;
                tt[(size_t)k * st] = v.w;
            }
        }
    };
    // chunk c's weights (1024 floats, 16 a lane): any tiny lam * C on a real line and sample
    auto flag = [&](int c) __attribute__((always_inline)) {
        const float* cw = (const float*)(lds + (c % kThNB) * kThBuf);
        bool t = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int e0 = (q * 64 + lane) * 4;  // element j * LPB + l
            const float4 v = *(const float4*)(cw + e0);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float x = lam * (&v.x)[e];
                const int el = e0 + e, j = el / LPB, l = el % LPB;
                t = t || (fabsf(x) < tiny && x != 0.0f && c * CH + j <= last && l0 + l < J.nl);
            }
        }
        if (lane == 0) *(int*)(orow + kThFlags + (c & 1) * 4) = __builtin_amdgcn_ballot_w64(t) != 0;
    };
    th_barrier();
    if (nch > 0) flag(0);
    th_lgkm0();
    th_barrier();
    for (int c = 0; c < nch; c++) {
        if (c > 0) put(c - 1);
        if (c + 1 < nch) flag(c + 1);
        th_lgkm0();
        th_barrier();
    }
    if (nch > 0) put(nch - 1);
}

// a coefficient job's LPB lines on the solver wave: the t recurrence; (a, den, 1/den, t) per
// sample into the writer's rows
template <int LPB>
__device__ __forceinline__ void th_job_solver(const FgsCoefJob& J, int l0, int lane, const char* lds, char* orow) {
    constexpr int CH = 1024 / LPB;
    const int ln = lane & (LPB - 1);
    const int last = J.n - 1, nch = (J.n + CH - 1) / CH;
    const float lam = J.lam;
    float rc[kThPF];
    th_barrier();
    th_barrier();  // (chunk 0's flag)
#pragma unroll
    for (int j = 0; j < kThPF; j++) rc[j] = *(const float*)(lds + (j * LPB + ln) * 4);
    float cprev = 0.0f, tprev = 0.0f;
    for (int c = 0; c < nch; c++) {
        const char* cur = lds + (c % kThNB) * kThBuf;
        const char* nxt = lds + ((c + 1) % kThNB) * kThBuf;
        const int kc = c * CH;
        char* w = orow + (c & 1) * 1024 * 16 + ln * 16;
        TH_STAMP(0, c);
        // a chunk with a tiny weight divides (IEEE), a clean one takes the reciprocal form
        auto body = [&](auto guard, auto exact) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < CH; j++) {
                if (j % 16 == 0) TH_STAMP(5, c * 8 + j / 16);
                const float cw = rc[j % kThPF];
                const int jn = j + kThPF;
                rc[j % kThPF] = jn < CH ? *(const float*)(cur + (jn * LPB + ln) * 4)
                                        : *(const float*)(nxt + ((jn - CH) * LPB + ln) * 4);
                if (!decltype(guard)::value || kc + j <= last) {
                    const float aa = lam * cprev;
                    const float cc = lam * cw;
                    const float den = (1.0f - cc) - aa * (1.0f + tprev);
                    const float r = fgs_rcp(den);
                    if constexpr (decltype(exact)::value) {
                        tprev = cc / den;
                    } else {
                        const float q0 = cc * r;
                        tprev = __builtin_fmaf(-__builtin_fmaf(q0, den, -cc), r, q0);  // cc / den
                    }
                    *(float4*)(w + j * LPB * 16) = make_float4(aa, den, r, tprev);
                    cprev = cw;
                }
            }
        };
        const bool full = kc + CH - 1 <= last;
        if (*(const volatile int*)(orow + kThFlags + (c & 1) * 4)) {
            if (full) body(std::false_type{}, std::true_type{});
            else body(std::true_type{}, std::true_type{});
        } else {
            if (full) body(std::false_type{}, std::false_type{});
            else body(std::true_type{}, std::false_type{});
        }
        TH_STAMP(1, c);
        th_lgkm0();
        th_barrier();
    }
}

// The solver wave of one pass: forward elimination (streams U and (a, den, 1/den, t)), then the
// back substitution (streams U -- the forward values -- and t); every result into the writer's
// LDS rows.
template <bool TWO, int LPB>
__device__ __forceinline__ void th_pass_solver(const FgsThArgs& a, size_t fofs, int l0, int lane, const char* lds,
                                               char* orow) {
    typedef FgsRhs<TWO> R;
    typedef typename R::T V;
    constexpr int ESU = TWO ? 8 : 4;
    constexpr int CH = 1024 / LPB;
    constexpr int S1 = 1024 * ESU;  // stream 1's offset in a chunk buffer
    typedef ThRows<LPB, ESU> RW;
    const int ln = lane & (LPB - 1);
    const int l = l0 + ln;
    const bool valid = lane < LPB && l < a.nl;
    const int n = a.n, last = n - 1;
    const int nch = (n + CH - 1) / CH;
    auto rdu = [&](const char* buf, int j) __attribute__((always_inline)) {
        return *(const V*)(buf + (j * LPB + ln) * ESU);
    };
    auto rdq = [&](const char* buf, int j) __attribute__((always_inline)) {
        return *(const float4*)(buf + S1 + (j * LPB + ln) * 16);
    };
    // ---- forward elimination ----
    TH_BLK(0);
    V ru[kThPF];
    float4 rq[kThPF];
    auto rd = [&](const char* buf, int j, int r) __attribute__((always_inline)) {
        ru[r] = rdu(buf, j);
        rq[r] = rdq(buf, j);
    };
    th_barrier();
#pragma unroll
    for (int j = 0; j < kThPF; j++) rd(lds, j, j);
    float p0 = 0.0f, p1 = 0.0f;
    for (int c = 0; c < nch; c++) {
        const char* cur = lds + (c % kThNB) * kThBuf;
        const char* nxt = lds + ((c + 1) % kThNB) * kThBuf;
        const int kc = c * CH;
        char* wu = orow + (c & 1) * 1024 * ESU + ln * ESU;  // this chunk's rows
        TH_STAMP(0, c);
        const float ps0 = p0, ps1 = p1;
        uint32_t key = 0xffffffffu;
        // exact: IEEE divisions (the right-hand sides decayed into the range the reciprocal form
        // does not cover: long runs of zero confidence); otherwise the reciprocal form with the
        // tiny-quotient key
        auto body = [&](auto guard, auto exact) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < CH; j++) {
                if (j % 16 == 0) TH_STAMP(5, c * 8 + j / 16);
                const int r = j % kThPF;
                const V xu = ru[r];
                const float4 xq = rq[r];  // a, den, 1/den, t
                const int jn = j + kThPF;
                if (jn < CH) rd(cur, jn, r);
                else rd(nxt, jn - CH, r);
                if (!decltype(guard)::value || kc + j <= last) {
                    const float x0 = R::x(xu) - xq.x * p0;
                    const float x1 = TWO ? R::y(xu) - xq.x * p1 : 0.0f;
                    if constexpr (decltype(exact)::value) {
                        p0 = x0 / xq.y;
                        if constexpr (TWO) p1 = x1 / xq.y;
                    } else {
                        const float q00 = x0 * xq.z;
                        p0 = __builtin_fmaf(-__builtin_fmaf(q00, xq.y, -x0), xq.z, q00);
                        key = min(key, fgs_tiny_key(q00));
                        if constexpr (TWO) {
                            const float q01 = x1 * xq.z;
                            p1 = __builtin_fmaf(-__builtin_fmaf(q01, xq.y, -x1), xq.z, q01);
                            key = min(key, fgs_tiny_key(q01));
                        }
                    }
                    *(V*)(wu + j * LPB * ESU) = R::make(p0, p1);
                }
            }
        };
        const bool full = kc + CH - 1 <= last;
        // a chunk starting from values already small (|p| < 2^-64) is likely to decay through the
        // uncovered range: it divides from the start
        const uint32_t small = 0x3EFFFFFFu;  // fgs_tiny_key(q) < small <=> 0 < |q| < 2^-64
        if (__builtin_amdgcn_ballot_w64(valid && (fgs_tiny_key(p0) < small || (TWO && fgs_tiny_key(p1) < small)))) {
            TH_COUNT(1);
            if (full) body(std::false_type{}, std::true_type{});
            else body(std::true_type{}, std::true_type{});
        } else {
            if (full) body(std::false_type{}, std::false_type{});
            else body(std::true_type{}, std::false_type{});
            // a chunk with a quotient the reciprocal form does not cover runs again from its start
            // with real divisions, its rows overwriting the first run's (the chunk's buffer is
            // intact until the barrier; the operand ring restarts at its first slots)
            TH_COUNT(0);
            if (__builtin_amdgcn_ballot_w64(valid && key < kFgsTinyKey)) {
                TH_COUNT(2);
                p0 = ps0;
                p1 = ps1;
#pragma unroll
                for (int j = 0; j < kThPF; j++) rd(cur, j, j);
                if (full) body(std::false_type{}, std::true_type{});
                else body(std::true_type{}, std::true_type{});
            }
        }
        TH_STAMP(1, c);
        th_lgkm0();
        th_barrier();
    }
    // (the writer has the forward values in memory before this barrier)
    TH_BLK(1);
    th_barrier();
    // ---- back substitution: u_k -= t[k] * u_{k+1}, k = n-2 .. 0 (the last sample keeps p) ----
    if (valid) {
        if (a.O) ((V*)a.O)[fofs + (size_t)l * a.onp + last] = R::make(p0, p1);
        else {
            a.O0[(size_t)blockIdx.y * a.ofs + (size_t)last * a.ost + l] = p0;
            if constexpr (TWO) a.O1[(size_t)blockIdx.y * a.ofs + (size_t)last * a.ost + l] = p1;
        }
    }
    const int nchb = (last + CH - 1) / CH;
    float q0 = p0, q1 = p1;
    V bu[kThPF];
    float bt[kThPF];
    auto rdb = [&](const char* buf, int j, int r) __attribute__((always_inline)) {
        bu[r] = rdu(buf, j);
        bt[r] = *(const float*)(buf + S1 + (j * LPB + ln) * 4);
    };
    th_barrier();
#pragma unroll
    for (int j = 0; j < kThPF; j++) rdb(lds, j, j);
    for (int c = 0; c < nchb; c++) {
        const char* cur = lds + (c % kThNB) * kThBuf;
        const char* nxt = lds + ((c + 1) % kThNB) * kThBuf;
        char* rows = orow + (c & 1) * CH * RW::S * 4 + ln * ESU;
        const int kb = last - 1 - c * CH;
        TH_STAMP(0, 512 + c);
        auto body = [&](auto guard) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const int r = j % kThPF;
                const V xu = bu[r];
                const float xt = bt[r];
                const int jn = j + kThPF;
                if (jn < CH) rdb(cur, jn, r);
                else rdb(nxt, jn - CH, r);
                if (!decltype(guard)::value || kb - j >= 0) {
                    q0 = R::x(xu) - xt * q0;
                    if constexpr (TWO) q1 = R::y(xu) - xt * q1;
                    *(V*)(rows + j * RW::S * 4) = R::make(q0, q1);
                }
            }
        };
        if (kb - CH + 1 >= 0) body(std::false_type{});
        else body(std::true_type{});
        TH_STAMP(1, 512 + c);
        th_lgkm0();
        th_barrier();
    }
    TH_BLK(2);
}

// One FGS pass (all lines of F frames) in ximgproc's order from its jobs' coefficients; blocks
// past main_blocks run coefficient jobs (a.job) instead (a launch of jobs alone: main_blocks = 0).
// 256 threads: solver, two loaders, writer.
template <bool TWO, int LPB>
__global__ __launch_bounds__(256) void k_fgs_th(FgsThArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[kThLds];
    char* orow = lds + kThNB * kThBuf;
    constexpr int CH = 1024 / LPB;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    const size_t fofs = (size_t)blockIdx.y * a.fs;
    const int blk = blockIdx.x;
    if (blk >= a.main_blocks) {
        int jb = blk - a.main_blocks, j = 0;
        while (j < a.njobs && jb >= a.job[j].blocks) jb -= a.job[j++].blocks;
        if (j >= a.njobs) return;  // uniform over the workgroup
        const FgsCoefJob& J = a.job[j];
        const int l0 = jb * LPB, nch = (J.n + CH - 1) / CH;
        if (wave == 0) th_job_solver<LPB>(J, l0, lane, lds, orow);
        else if (wave <= 2)
            th_load_phase<LPB, 4, 0>((const char*)(J.Cw + fofs), nullptr, J.st, l0, 0, 1, J.n - 1, nch, lds,
                                     wave - 1, lane, 1);
        else th_write_job_phase<LPB>(J, fofs, l0, nch, lds, orow, lane);
        return;
    }
    constexpr int ESU = TWO ? 8 : 4;
    const int l0 = blk * LPB, n = a.n, last = n - 1;
    const int nch = (n + CH - 1) / CH, nchb = (last + CH - 1) / CH;
    const char* gu = (const char*)a.U + fofs * ESU;
    if (wave == 0) {
        th_pass_solver<TWO, LPB>(a, fofs, l0, lane, lds, orow);
    } else if (wave <= 2) {
        const int lw = wave - 1;
        th_load_phase<LPB, ESU, 16>(gu, (const char*)(a.coef + fofs), a.st, l0, 0, 1, last, nch, lds, lw, lane);
        th_barrier();
        th_load_phase<LPB, ESU, 4>(gu, (const char*)(a.tt + fofs), a.st, l0, last - 1, -1, last, nchb, lds, lw, lane);
    } else {
        th_write_fwd_phase<TWO, LPB>(a.U, a.st, fofs, l0, a.nl, last, nch, orow, lane);
        th_barrier();
        th_write_back_phase<TWO, LPB>(a, fofs, l0, last, nchb, orow, lane);
    }
}

// ---- k_fgs_lr: the sequential pass with its lines resident in LDS (round 6) ----------------
// The same recurrences, operations and roundings as k_fgs_th (ximgproc's order, bit-exact), for
// both right-hand sides at once, rebuilt around what bounds a one-wave chain: every instruction
// the chain's wave issues is on the critical path (a dependent f32 op takes ~4.9 cycles, the
// issue of the next about 4: nothing hides behind the chain), so the pass time is the solver
// wave's instruction count per sample times the line length (scripts/probe/fgs_rows.hip).
//  * one solver wave PER IMAGE (waves 0 and 1, on two SIMDs): scalar chains, 5 dependent ops a
//    forward sample and 2 a back sample (the packed form issues at 8 cycles an op: no gain);
//  * lane = (row, line): L <= 16 lines on the 16 lanes of each 16-lane row, and the four rows hold
//    four consecutive samples each of a 16-sample group, so ONE LDS instruction reads or writes
//    4 samples x L lines; the chain value walks the rows 0 -> 1 -> 3 -> 2 (one v_permlane16/32_swap
//    per row change, every 4 samples), every row computing every step (the issue cost is the
//    wave's whatever the rows), each row keeping its own steps' results (selected per lane at the
//    group's end: no exec masks);
//  * the whole line stays in LDS: the loader waves (2 and 3) DMA the pass's input U and its
//    coefficients (a, den, 1/den, t) once, a chunk of 1024 line-samples at a time, up to
//    kLrAhead chunks ahead; the forward values overwrite U in place and the back substitution
//    reads them from there (no global round trip between the two phases, no buffer reuse), its
//    results overwrite them again and the same two waves store them to global memory a chunk
//    behind the solvers;
//  * the reciprocal-form division with the tiny-quotient key per 16-sample group; a group whose
//    key trips runs again from its start with IEEE divisions (its operands are still in
//    registers), and a group starting from an already small value (|p| < 2^-64) divides from the
//    start (the same rule as k_fgs_th's chunks, per 16 samples instead of per chunk).
// LDS: [U: kLrChunks x 8 KiB][coef: kLrChunks x 16 KiB], sample k of line l at (k * L + l): a line
// of up to kLrChunks * 1024 / L samples (L = 16: 384, 8: 768, 4: 1536, 2: 3072).  Longer lines
// take k_fgs_th.
constexpr int kLrChunks = 6;
constexpr int kLrU = kLrChunks * 8192, kLrLds = kLrChunks * 24576;
constexpr int kLrAhead = 4;  // chunks in flight (th_wait_chunks waits for at most 2 beyond)
static_assert(kLrAhead - 2 <= kThNB - 3, "th_wait_chunks' range");

// the chain value from one lane row to the next in the walk 0 -> 1 -> 3 -> 2 -> 0: the swap of p
// with itself keeps the source row's value where it was AND copies it into the next row, so the
// result is both the step's kept value (for the source row) and the next row's chain input
__device__ __forceinline__ float lr_row(int step, float p) {
    const int b = __builtin_bit_cast(int, p);
    if (step == 0) return __builtin_bit_cast(float, (int)__builtin_amdgcn_permlane16_swap(b, b, false, false)[0]);
    if (step == 1) return __builtin_bit_cast(float, (int)__builtin_amdgcn_permlane32_swap(b, b, false, false)[0]);
    if (step == 2) return __builtin_bit_cast(float, (int)__builtin_amdgcn_permlane16_swap(b, b, false, false)[1]);
    return __builtin_bit_cast(float, (int)__builtin_amdgcn_permlane32_swap(b, b, false, false)[1]);
}

// a lane's own row's value among the walk's four steps (rows 0, 1, 3, 2 take steps 0, 1, 2, 3)
template <typename T>
__device__ __forceinline__ T lr_own(const T (&v)[4], bool s0, bool s1, bool s2) {
    return s0 ? v[0] : s1 ? v[1] : s2 ? v[2] : v[3];
}

struct LrFwdOps {
    float4 q[4];  // (a, den, 1/den, t) of the lane's 4 samples
    float x[4];   // the right-hand side
};
struct LrBackOps {
    float t[4];
    float x[4];  // the forward values
};

template <int L>
struct LrLane {
    int l, step;     // line within the workgroup, the walk step of the lane's row
    bool s0, s1, s2;  // step == 0, 1, 2
    bool valid;       // a real line (l < L and inside the pass)
    int img4;         // 4 * image (the float2 half)
};

// forward group: samples k0 .. k0 + 15 (k0 = 16 g); lane row of walk step s holds k0 + 4 s + e.
// The reciprocal form keeps per walk step the tiny-quotient key of its row's steps (kk[s]: each
// row's own is selected after the group).
template <bool EXACT, bool GUARD>
__device__ __forceinline__ void lr_fwd_body(float& p, const LrFwdOps& o, int k0, int n, float (&res)[4][4],
                                            uint32_t (&kk)[4]) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
        if constexpr (!EXACT) kk[s] = 0xffffffffu;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            if (!GUARD || k0 + 4 * s + e < n) {
                const float x = o.x[e] - o.q[e].x * p;
                if constexpr (EXACT) {
                    p = x / o.q[e].y;
                } else {
                    const float q0 = x * o.q[e].z;
                    p = __builtin_fmaf(-__builtin_fmaf(q0, o.q[e].y, -x), o.q[e].z, q0);
                    kk[s] = min(kk[s], fgs_tiny_key(q0));
                }
            }
            if (e < 3) res[s][e] = p;
        }
        p = lr_row(s, p);  // keeps the row's value and hands it to the next row
        res[s][3] = p;
    }
}

// The group with the reciprocal form, or with IEEE divisions when it starts from an already small
// value (0 < |p| < 2^-64: a decaying run of zero right-hand sides) or when a quotient came out
// 0 < |q0| < 2^-96 (outside what the reciprocal form covers, scripts/markstein_check.c): then
// again from the group's start value.  k_fgs_th's rules, per 16 samples.
template <int L, bool GUARD>
__device__ __forceinline__ void lr_fwd_group(float& p, const LrFwdOps& o, const LrLane<L>& ln, int k0, int n,
                                             char* uw) {
    float res[4][4];
    uint32_t kk[4];
    const float ps = p;  // (valid in row 0, where the walk starts)
    const uint32_t small = 0x3EFFFFFFu;  // fgs_tiny_key(p) < small <=> 0 < |p| < 2^-64
    bool exact = __builtin_amdgcn_ballot_w64(ln.valid & ln.s0 & (fgs_tiny_key(p) < small)) != 0;
    if (!exact) {
        lr_fwd_body<false, GUARD>(p, o, k0, n, res, kk);
        exact = __builtin_amdgcn_ballot_w64(ln.valid & (lr_own(kk, ln.s0, ln.s1, ln.s2) < kFgsTinyKey)) != 0;
        if (exact) p = ps;
    }
    if (exact) lr_fwd_body<true, GUARD>(p, o, k0, n, res, kk);
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const float v[4] = {res[0][e], res[1][e], res[2][e], res[3][e]};
        if (!GUARD || k0 + 4 * ln.step + e < n) *(float*)(uw + e * L * 8) = lr_own(v, ln.s0, ln.s1, ln.s2);
    }
}

// back group: samples k1 .. k1 - 15 (k1 = n - 1 - 16 gb); lane row of walk step s holds
// k1 - 4 s - e; the line's last sample keeps its forward value
template <int L, bool GUARD>
__device__ __forceinline__ void lr_back_group(float& p, const LrBackOps& o, const LrLane<L>& ln, int k1, int n,
                                              char* uw) {
    float res[4][4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int k = k1 - 4 * s - e;
            if (!GUARD || k >= 0) {
                if (GUARD && k == n - 1) p = o.x[e];
                else p = o.x[e] - o.t[e] * p;
            }
            if (e < 3) res[s][e] = p;
        }
        p = lr_row(s, p);
        res[s][3] = p;
    }
    // the lane's samples k1 - 4 s - e sit at uw - e * L * 8 (uw: its first, the highest)
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const float v[4] = {res[0][e], res[1][e], res[2][e], res[3][e]};
        if (!GUARD || k1 - 4 * ln.step - e >= 0) *(float*)(uw - e * L * 8) = lr_own(v, ln.s0, ln.s1, ln.s2);
    }
}

#ifdef SDR_TH_STAMPS
// diagnostic build only: per workgroup of the first 512 of each of 16 launch slots (scripts/lr_stamps.py):
// 0 entry, 1 first chunk landed, 2 forward done, 3 back done (solver 0), 4 writer done, 5 solver exit,
// 6 entry s_memrealtime (100 MHz)
__device__ unsigned long long g_lr_blk[16][512][8];
#define LR_STAMP(cond, slot, i)                                                                      \
    do {                                                                                             \
        if ((cond) && (slot) >= 0 && (threadIdx.x & 63) == 0 && blockIdx.x < 512 && blockIdx.y == 0) { \
            g_lr_blk[(slot) & 15][blockIdx.x][i] = __builtin_amdgcn_s_memtime();                     \
            if ((i) == 0) g_lr_blk[(slot) & 15][blockIdx.x][6] = __builtin_amdgcn_s_memrealtime();    \
            if ((i) == 5) g_lr_blk[(slot) & 15][blockIdx.x][7] = __builtin_amdgcn_s_memrealtime();    \
        }                                                                                            \
    } while (0)
#else
#define LR_STAMP(cond, slot, i) \
    do {                        \
    } while (0)
#endif

#ifdef SDR_TH_STAMPS
// diagnostic build only: k_fgs_lrjob's per-workgroup stamps of the last launch (frame 0, the first
// 512 workgroups; scripts/lj_stamps.py): 0 entry, 1 chunk 0 prepared (prep), 2 solver past its
// first barrier, 3 solver done, 4 writer 0 done, 5 prep done, 6 / 7 s_memrealtime at 0 / 3
__device__ unsigned long long g_lj_blk[512][8];
#define LJ_STAMP(cond, i)                                                                            \
    do {                                                                                             \
        if ((cond) && (threadIdx.x & 63) == 0 && blockIdx.x < 512 && blockIdx.y == 0) {              \
            g_lj_blk[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                                  \
            if ((i) == 0) g_lj_blk[blockIdx.x][6] = __builtin_amdgcn_s_memrealtime();                 \
            if ((i) == 3) g_lj_blk[blockIdx.x][7] = __builtin_amdgcn_s_memrealtime();                 \
        }                                                                                            \
    } while (0)
#else
#define LJ_STAMP(cond, i) \
    do {                  \
    } while (0)
#endif

// The solver wave of image `img` (0: A / U.x, 1: B / U.y).  The whole groups of a chunk run in
// unrolled blocks of up to 8 with the next group's operands loaded during the current one into a
// second, static register set (a loop-carried pair made the compiler copy the loads and wait for
// each right away); every load is unconditional, clamped inside the chunk images (a conditional
// load made it wait for all of them).  The partial groups -- the line's last forward group, the
// back groups holding its last and its first samples -- take the guarded form.
template <int L>
__device__ __forceinline__ void lr_solver(int n, int nch, int img, int lane, bool lv, char* lds, int dbg) {
    constexpr int CH = 1024 / L;  // samples a chunk
    constexpr int G = CH / 16;    // groups a chunk
    constexpr int UB = G < 8 ? G : 8;  // groups an unrolled block
    LrLane<L> ln;
    ln.l = lane & 15;
    const int row = lane >> 4;
    ln.step = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
    ln.s0 = ln.step == 0;
    ln.s1 = ln.step == 1;
    ln.s2 = ln.step == 2;
    ln.valid = lv && ln.l < L;
    const int l = ln.l < L ? ln.l : L - 1;  // (lanes past L repeat line L - 1: the same values)
    ln.img4 = img * 4;
    char* U = lds + img * 4;
    const char* Cq = lds + kLrU;
    const int kmax = nch * CH - 1;  // the last sample slot of the chunk images
    auto uaddr = [&](int k) __attribute__((always_inline)) { return U + (k * L + l) * 8; };
    auto ld_fwd = [&](int g, LrFwdOps& o) __attribute__((always_inline)) {
        const int k = min(16 * g + 4 * ln.step, kmax - 3);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            o.q[e] = *(const float4*)(Cq + ((k + e) * L + l) * 16);
            o.x[e] = *(const float*)uaddr(k + e);
        }
    };
    const int ng = (n + 15) / 16, ngf = n / 16;  // groups of the line, whole ones
    // ---- forward elimination: barrier c = chunks <= c + 1 landed ----
    float p = 0.0f;
    th_barrier();
    LR_STAMP(img == 0, dbg, 1);
    for (int c = 0; c < nch; c++) {
        if (c > 0) th_barrier();
        for (int b0 = c * G; b0 < min(c * G + G, ngf); b0 += UB) {
            LrFwdOps ops[UB];  // (one set per unrolled group: static indices, no copies)
            ld_fwd(b0, ops[0]);
#pragma unroll
            for (int gg = 0; gg < UB; gg++) {
                const int g = b0 + gg;
                if (gg + 1 < UB) ld_fwd(g + 1, ops[gg + 1 < UB ? gg + 1 : gg]);
                if (g < ngf) lr_fwd_group<L, false>(p, ops[gg], ln, 16 * g, n, uaddr(16 * g + 4 * ln.step));
            }
        }
        if (ngf < ng && ngf >= c * G && ngf < c * G + G) {  // the partial last group is in this chunk
            LrFwdOps A;
            const int k = 16 * ngf + 4 * ln.step;  // (each sample clamped on its own: the mapping holds)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                A.q[e] = *(const float4*)(Cq + (min(k + e, kmax) * L + l) * 16);
                A.x[e] = *(const float*)uaddr(min(k + e, kmax));
            }
            lr_fwd_group<L, true>(p, A, ln, 16 * ngf, n, uaddr(min(16 * ngf + 4 * ln.step, kmax)));
        }
    }
    LR_STAMP(img == 0, dbg, 2);
    // ---- back substitution: barrier cb = chunk cb's results in LDS for the writers ----
    // back group gb: samples k1 .. k1 - 15, k1 = n - 1 - 16 gb: gb = 0 holds the last sample,
    // gb = ngf the first ones when n % 16 != 0 (guarded); the others are whole
    auto ld_back = [&](int gb, LrBackOps& o) __attribute__((always_inline)) {
        const int k = max(n - 1 - 16 * gb - 4 * ln.step, 3);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            o.t[e] = *(const float*)(Cq + ((k - e) * L + l) * 16 + 12);
            o.x[e] = *(const float*)uaddr(k - e);
        }
    };
    auto back_guarded = [&](int gb, float& q) __attribute__((always_inline)) {
        LrBackOps A;
        const int k1 = n - 1 - 16 * gb;
        const int k = k1 - 4 * ln.step;  // (each sample clamped on its own: the mapping holds)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            A.t[e] = *(const float*)(Cq + (max(k - e, 0) * L + l) * 16 + 12);
            A.x[e] = *(const float*)uaddr(max(k - e, 0));
        }
        lr_back_group<L, true>(q, A, ln, k1, n, uaddr(max(k1 - 4 * ln.step, 0)));
    };
    float q = 0.0f;
    for (int cb = 0; cb < nch; cb++) {
        const int lo = max(cb * G, 1), hi = min(cb * G + G, ngf);  // whole back groups: 1 .. ngf - 1
        if (cb == 0) back_guarded(0, q);
        for (int b0 = lo; b0 < hi; b0 += UB) {
            LrBackOps ops[UB];
            ld_back(b0, ops[0]);
#pragma unroll
            for (int gg = 0; gg < UB; gg++) {
                const int gb = b0 + gg;
                if (gg + 1 < UB) ld_back(gb + 1, ops[gg + 1 < UB ? gg + 1 : gg]);
                if (gb < hi) {
                    const int k1 = n - 1 - 16 * gb;
                    lr_back_group<L, false>(q, ops[gg], ln, k1, n, uaddr(k1 - 4 * ln.step));
                }
            }
        }
        if (ng > ngf && ngf >= cb * G && ngf < cb * G + G && ngf >= 1) back_guarded(ngf, q);
        th_lgkm0();
        th_barrier();
    }
    LR_STAMP(img == 0, dbg, 3);
}

// The loader waves (lw = 0, 1): the pass's U (float2) and coefficient chunks, up to kLrAhead in
// flight; before barrier c, chunks <= c + 1 have landed.  Then, as writers, the results of back
// chunk cb after barrier cb: line-major float2 into a.O (the next pass's input), or k-major split
// into a.O0 / a.O1 (the last pass).
template <int L>
__device__ __forceinline__ void lr_loader_writer(const FgsThArgs& a, size_t fofs, int l0, int nch, int lw, int lane,
                                                 char* lds) {
    constexpr int CH = 1024 / L, IW = (8 + 16) / 2;
    const int n = a.n, last = n - 1;
    const char* gu = (const char*)((const float2*)a.U + fofs);
    const char* gc = (const char*)(a.coef + fofs);
    auto issue = [&](int c) __attribute__((always_inline)) {
        th_issue<L, 8>(gu, a.st, l0, c * CH, 1, last, lds + c * 8192, lw, lane);
        th_issue<L, 16>(gc, a.st, l0, c * CH, 1, last, lds + kLrU + c * 16384, lw, lane);
    };
    int issued = 0;
#ifdef SDR_LR_PRELOAD  // diagnostic: every chunk landed before the solvers start
    for (; issued < nch; issued++) {
        issue(issued);
        th_vmcnt<0>();
    }
    for (int c = 0; c < nch; c++) th_barrier();
#else
    for (; issued < min(kLrAhead, nch); issued++) issue(issued);
    for (int c = 0; c < nch; c++) {
        th_wait_chunks<IW>(issued - min(c + 2, issued));
        th_barrier();
        if (issued < nch) issue(issued++);
    }
#endif
    // ---- writers ----
    const float2* R = (const float2*)lds;
    for (int cb = 0; cb < nch; cb++) {
        th_barrier();
        const int khi = n - cb * CH, klo = max(khi - CH, 0);  // samples [klo, khi)
        if (a.O) {
            // line-major: a wave-instruction = 64 consecutive samples of one line
            for (int l = lw; l < L; l += 2) {
                if (l0 + l >= a.nl) break;
                float2* o = (float2*)a.O + fofs + (size_t)(l0 + l) * a.onp;
                for (int k = klo + lane; k < khi; k += 64) o[k] = R[k * L + l];
            }
        } else {
            // k-major split: a wave-instruction = 64 / L samples x L lines
            const size_t fo = (size_t)blockIdx.y * a.ofs + l0;
            const int l = lane % L;
            for (int k = klo + lw * (64 / L) + lane / L; k < khi; k += 2 * (64 / L)) {
                if (l0 + l < a.nl) {
                    const float2 v = R[k * L + l];
                    a.O0[fo + (size_t)k * a.ost + l] = v.x;
                    a.O1[fo + (size_t)k * a.ost + l] = v.y;
                }
            }
        }
    }
}

// One FGS pass of two right-hand sides (a.U float2), L lines a workgroup, every line resident.
template <int L>
__global__ __launch_bounds__(256) void k_fgs_lr(FgsThArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[kLrLds];
    constexpr int CH = 1024 / L;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    const size_t fofs = (size_t)blockIdx.y * a.fs;
    const int l0 = blockIdx.x * L;
    const int nch = (a.n + CH - 1) / CH;
    LR_STAMP(wave == 0, a.dbg, 0);
#ifdef SDR_LR_ONE_SOLVER  // diagnostic: the second solver only keeps the barrier count (its image is not solved)
    if (wave == 1) {
        for (int c = 0; c < 2 * nch; c++) th_barrier();
    } else
#endif
    if (wave < 2) lr_solver<L>(a.n, nch, wave, lane, l0 + (lane & 15) < a.nl, lds, a.dbg);
    else lr_loader_writer<L>(a, fofs, l0, nch, wave - 2, lane, lds);
    LR_STAMP(wave == 2, a.dbg, 4);
    LR_STAMP(wave == 0, a.dbg, 5);
}

// ---- k_fgs_lrjob: the coefficient jobs the k_fgs_lr way (round 6) --------------------------
// th_job_solver's recurrence, operations and roundings (bit-exact): per sample k of a line
//   aa = lam * C[k-1] (C[-1] = 0),  cc = lam * C[k],  den = (1 - cc) - aa * (1 + t),
//   r = fgs_rcp(den),  t = cc / den (from r by Markstein, or IEEE in a group holding a tiny cc)
// with t carried from sample to sample: a chain of 9 dependent operations.  On one wave every
// instruction it issues is on that chain (k_fgs_lr's finding), so the work is split so that the
// chain's wave issues little else:
//   wave 0     the solver: lane = (row, line) as in k_fgs_lr -- 4 consecutive samples x L lines
//              an LDS instruction, the chain walking the rows by permlane swaps -- reading each
//              sample's (aa, cc, 1 - cc) and writing (den, 1/den, t) with its row's stores
//              (exec-masked per walk step, no selects; the writers add aa);
//   wave 1     the prep wave: the line's weights DMA'd at the start (resident, kLrChunks chunks),
//              then per chunk (aa, cc, 1 - cc) into LDS and a flag bit per 16-sample group holding a
//              tiny cc (one word a chunk, read once by the solver) (0 < |cc| < 2^-96 (1 + 2 lam), where the reciprocal form may round apart
//              from the division), a chunk ahead of the solver;
//   waves 2, 3 the writers: chunk c's rows to coef and tt, a chunk behind the solver.
// Iteration i (a barrier each, nch + 2 of them): prep chunk i, solve chunk i - 1, write chunk i - 2.
// LDS: [weights: kLrChunks x 4 KiB][prep: kLrChunks x 16 KiB][rows: 2 x 16 KiB][chunk flags].
constexpr int kLjW = kLrChunks * 4096, kLjP = kLrChunks * 16384, kLjO = 2 * 16384;
constexpr int kLjLds = kLjW + kLjP + kLjO + kLrChunks * 4;  // + a flag word a chunk (bit: group)
static_assert(1024 / 4 / 16 <= 32, "a chunk's groups fit a flag word");
static_assert(kLjLds <= 160 * 1024, "one workgroup's LDS");

// one walk step after another: the step-s row's 4 samples are the chain's, its stores the only
// ones that land (the other rows compute from their own operands and are masked off)
template <int L, bool EXACT, bool GUARD>
__device__ __forceinline__ void lj_body(float& t, const float4 (&q)[4], int step, int k0, int n, float4* orow) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
        float3 res[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            if (!GUARD || k0 + 4 * s + e < n) {
                const float aa = q[e].x, cc = q[e].y;
#ifdef SDR_LJ_NOCHAIN  // diagnostic: one op a sample instead of the chain (results wrong)
                t = t + cc;
                res[e] = make_float3(aa, cc, t);
                continue;
#endif
                const float den = q[e].z - aa * (1.0f + t);
                const float r = fgs_rcp(den);
                if constexpr (EXACT) {
                    t = cc / den;
                } else {
                    const float q0 = cc * r;
                    t = __builtin_fmaf(-__builtin_fmaf(q0, den, -cc), r, q0);  // cc / den
                }
                res[e] = make_float3(den, r, t);
            }
        }
#ifndef SDR_LJ_NOSTORE  // diagnostic: the solver stores nothing (results wrong)
        if (step == s) {
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (!GUARD || k0 + 4 * s + e < n) *(float3*)(orow + e * L) = res[e];
        }
#else
        if (t == 12345.0f) *(float3*)orow = res[0];
#endif
        t = lr_row(s, t);
    }
}

template <int L>
__device__ __forceinline__ void lj_solver(int n, int nch, int lane, char* lds) {
    constexpr int CH = 1024 / L, G = CH / 16;
    constexpr int UB = G < 8 ? G : 8;  // groups an unrolled block (within a chunk)
    const int row = lane >> 4, lq = lane & 15;
    const int l = lq < L ? lq : L - 1;  // (lanes past L repeat line L - 1: the same values, the same slots)
    const int step = row == 0 ? 0 : row == 1 ? 1 : row == 3 ? 2 : 3;
    const float4* P = (const float4*)(lds + kLjW);
    float4* O = (float4*)(lds + kLjW + kLjP);
    const uint32_t* flags = (const uint32_t*)(lds + kLjW + kLjP + kLjO);
    const int ng = (n + 15) / 16, ngf = n / 16;
    struct Ops {
        float4 q[4];
    };
    // a group's operands (every slot of a chunk holds a value: the prep wave covers all)
    auto ld = [&](int g, Ops& o) __attribute__((always_inline)) {
        const int k = 16 * g + 4 * step;
#pragma unroll
        for (int e = 0; e < 4; e++) o.q[e] = P[(k + e) * L + l];
    };
    uint32_t cflags = 0;  // the chunk's group flags (bit g - c * G), wave-uniform
    auto group = [&](float& t, const Ops& o, int g, int c, auto guard) __attribute__((always_inline)) {
        constexpr bool GU = decltype(guard)::value;
        float4* orow = O + (c & 1) * 1024 + (16 * g - c * CH + 4 * step) * L + l;
        if ((cflags >> (g - c * G)) & 1u) lj_body<L, true, GU>(t, o.q, step, 16 * g, n, orow);
        else lj_body<L, false, GU>(t, o.q, step, 16 * g, n, orow);
    };
    float t = 0.0f;
    th_barrier();  // iteration 0: chunk 0 prepared
    LJ_STAMP(true, 2);
    for (int c = 0; c < nch; c++) {
        cflags = __builtin_amdgcn_readfirstlane(flags[c]);
        for (int b0 = c * G; b0 < min(c * G + G, ngf); b0 += UB) {
            Ops ops[UB];  // (one set per unrolled group: static indices, no copies)
            ld(b0, ops[0]);
#pragma unroll
            for (int gg = 0; gg < UB; gg++) {
                const int g = b0 + gg;
                if (gg + 1 < UB) ld(g + 1, ops[gg + 1 < UB ? gg + 1 : gg]);
                if (g < ngf) group(t, ops[gg], g, c, std::false_type{});
            }
        }
        if (ngf < ng && ngf >= c * G && ngf < c * G + G) {  // the line's partial last group
            Ops o;
            ld(ngf, o);
            group(t, o, ngf, c, std::true_type{});
        }
        th_lgkm0();
        th_barrier();
    }
    LJ_STAMP(true, 3);
    th_barrier();  // iteration nch + 1: the writers' last chunk
}

// s_waitcnt for the prep wave's DMA: chunk i landed when at most `younger` chunks (4
// wave-instructions each) are in flight after it
__device__ __forceinline__ void lj_wait(int younger) {
    static_assert(kLrChunks <= 6, "vmcnt cases");
    switch (younger) {
        case 0: th_vmcnt<0>(); break;
        case 1: th_vmcnt<4>(); break;
        case 2: th_vmcnt<8>(); break;
        case 3: th_vmcnt<12>(); break;
        case 4: th_vmcnt<16>(); break;
        default: th_vmcnt<20>(); break;
    }
}

template <int L>
__device__ __forceinline__ void lj_prep(const FgsCoefJob& J, size_t fofs, int l0, int nch, int lane, char* lds) {
    constexpr int CH = 1024 / L;
    const int last = J.n - 1;
    const float lam = J.lam, tiny = 0x1p-96f * (1.0f + 2.0f * lam);
    const float* W = (const float*)lds;
    float4* P = (float4*)(lds + kLjW);
    uint32_t* flags = (uint32_t*)(lds + kLjW + kLjP + kLjO);
    if (lane < kLrChunks) flags[lane] = 0;
    const char* gw = (const char*)(J.Cw + fofs);
    for (int c = 0; c < nch; c++) {
        th_issue<L, 4>(gw, J.st, l0, c * CH, 1, last, lds + c * 4096, 0, lane);
        th_issue<L, 4>(gw, J.st, l0, c * CH, 1, last, lds + c * 4096, 1, lane);
    }
    for (int i = 0; i < nch + 2; i++) {
        if (i < nch) {
            lj_wait(nch - 1 - i);
#pragma unroll 4
            for (int it = 0; it < 16; it++) {
                const int j = i * 1024 + it * 64 + lane;  // = k * L + l
                const int k = j / L, l = j % L;
                const float cw = W[j];
                const float cp = k > 0 ? W[j - L] : 0.0f;
                const float aa = lam * cp, cc = lam * cw;
                P[j] = make_float4(aa, cc, 1.0f - cc, 0.0f);
                if (fabsf(cc) < tiny && cc != 0.0f && k <= last && l0 + l < J.nl)
                    atomicOr(&flags[i], 1u << (k / 16 - i * (CH / 16)));
            }
            if (i == 0) LJ_STAMP(true, 1);
        }
        th_lgkm0();
        th_barrier();
    }
    LJ_STAMP(true, 5);
}

template <int L>
__device__ __forceinline__ void lj_writer(const FgsCoefJob& J, size_t fofs, int l0, int nch, int lw, int lane,
                                          const char* lds) {
    constexpr int CH = 1024 / L;
    const int last = J.n - 1;
    const float4* O = (const float4*)(lds + kLjW + kLjP);
    const float* W = (const float*)lds;
    for (int i = 0; i < nch + 2; i++) {
        const int c = i - 2;
        if (c >= 0) {
            const float4* Oc = O + (c & 1) * 1024;
#pragma unroll 4
            for (int it = 0; it < 8; it++) {
                const int j = (2 * it + lw) * 64 + lane;  // = (k - c * CH) * L + l
                const int k = c * CH + j / L, l = j % L;
                if (k <= last && l0 + l < J.nl) {
                    // the solver's (den, 1/den, t); aa = lam * C[k-1] again from the weights
                    const float4 v = Oc[j];
                    const float aa = J.lam * (k > 0 ? W[c * 1024 + j - L] : 0.0f);
                    const size_t o = fofs + (size_t)k * J.st + l0 + l;
                    J.coef[o] = make_float4(aa, v.x, v.y, v.z);
                    J.tt[o] = v.z;
                }
            }
        }
        th_barrier();
    }
    LJ_STAMP(lw == 0, 4);
}

template <int L>
__device__ __forceinline__ void lj_block(const FgsCoefJob& J, size_t fofs, int jb, int wave, int lane, char* lds) {
    constexpr int CH = 1024 / L;
    const int l0 = jb * L, nch = (J.n + CH - 1) / CH;
    if (wave == 0) lj_solver<L>(J.n, nch, lane, lds);
    else if (wave == 1) lj_prep<L>(J, fofs, l0, nch, lane, lds);
    else lj_writer<L>(J, fofs, l0, nch, wave - 2, lane, lds);
}

// The coefficient jobs of a launch (a.job, blocks of job.lpb lines each; blockIdx.y = frame).
__global__ __launch_bounds__(256) void k_fgs_lrjob(FgsThArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[kLjLds];
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    const size_t fofs = (size_t)blockIdx.y * a.fs;
    int jb = blockIdx.x, j = 0;
    while (j < a.njobs && jb >= a.job[j].blocks) jb -= a.job[j++].blocks;
    if (j >= a.njobs) return;  // uniform over the workgroup
    const FgsCoefJob& J = a.job[j];
    LJ_STAMP(wave == 0, 0);
    switch (J.lpb) {
        case 16: lj_block<16>(J, fofs, jb, wave, lane, lds); break;
        case 8: lj_block<8>(J, fofs, jb, wave, lane, lds); break;
        default: lj_block<4>(J, fofs, jb, wave, lane, lds); break;
    }
}

// R0 (and R1) row-major [h][w] -> the first row pass's input: transposed [w][hp] (hp = h rounded
// up to 4, frames fgs_pad4(w) * hp apart), the two images interleaved (float2) when R1 is given;
// 64x64 LDS tiles
__global__ __launch_bounds__(256) void k_fgs_pack(const float* __restrict__ r0, const float* __restrict__ r1,
                                                  float* __restrict__ dst, int h, int w) {
    __shared__ float tile[2][64][65];
    const int c0 = blockIdx.x * 64, rw0 = blockIdx.y * 64;
    const size_t fo = (size_t)blockIdx.z * h * w;
    const int hp = fgs_pad4(h);
    const size_t fd = (size_t)blockIdx.z * fgs_pad4(w) * hp;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int rr = rw0 + r, cc = c0 + tx;
        if (rr < h && cc < w) {
            tile[0][r][tx] = r0[fo + (size_t)rr * w + cc];
            if (r1) tile[1][r][tx] = r1[fo + (size_t)rr * w + cc];
        }
    }
    __syncthreads();
    for (int c = ty; c < 64; c += 4) {
        const int cc = c0 + c, rr = rw0 + tx;
        if (rr < h && cc < w) {
            const size_t o = fd + (size_t)cc * hp + rr;
            if (r1) ((float2*)dst)[o] = make_float2(tile[0][tx][c], tile[1][tx][c]);
            else dst[o] = tile[0][tx][c];
        }
    }
}

// FGS line solves by parallel cyclic reduction (the default solver), in the operation order of
// oracle/wls_oracle.c fgs_line_pcr.  A workgroup of T threads (blockDim.x, a multiple of 64, up
// to 1024) owns G lines of n samples of one frame (G = 1 for long lines); equation e = g*n + k of
// the block lives in registers of thread e mod T (slot e / T), so a thread keeps its equations'
// (a, c, e, b, d0, d1) across the log2(n) stages and only publishes what its neighbours read:
//   X[e] = {row sum, 1/b, d0, d1} (one 16-byte LDS word), A[e] = a, Cc[e] = c
// Stage s reads X and A of e - s, X and Cc of e + s (zeros past the line's ends), then every
// equation is rewritten at once.  The published values are double-buffered by stage parity, so
// a stage costs one barrier: a thread can only overwrite a buffer two stages later, after the
// barrier every reader of it has passed.  The chip holds few lines (360 rows or 280 column pairs
// at 640x360), so the block takes as many threads as equations (EPT = 1 up to 1024 samples):
// several waves per SIMD hide the LDS and division latencies of the stage chain.  The images are
// read and written in place in their row-major layout: for rows (lines = rows) a block's loads
// are whole rows, for columns (lines = columns) G adjacent columns per row; loads and stores go
// through LDS with consecutive threads on consecutive addresses.  Weights Cw: same layout as the
// images (Ch for rows, Cv for columns, 0 on each line's last sample).
constexpr int kPcrMaxN = 4096;  // samples per block (G * n): 4 equations per thread of 1024

// DB: the stage buffers double-buffered (48 B of LDS per sample, one barrier per stage), or single
// (24 B per sample, two barriers per stage) for blocks whose 48 B per sample exceed the
// workgroup's LDS (160 KiB on gfx950: past 3413 samples)
// FIN (the last column pass, both right-hand sides): instead of storing the solved A, B back, the
// block writes the filter's outputs for its ROI pixels (wls_value / wls_emit; gw = the geometry)
template <int EPT, bool TWO, bool DB = true, bool FIN = false>
__global__ __launch_bounds__(1024) void k_fgs_pcr(float* U0, float* U1, const float* __restrict__ Cw,
                                                  int w, int h, size_t fstride, int rows, int G,
                                                  float lam, WlsGeom gw = {}, WlsOut wo = {}) {
    extern __shared__ float4 pcr_smem[];
    constexpr int NB = DB ? 2 : 1;
    const int T = blockDim.x;
    const int n = rows ? w : h;
    const int nlines = rows ? h : w;
    const int N = G * n;
    // NB stage buffers: X [NB][N] {row sum, 1/b, d0, d1}, then A [NB][N] (a; the weights during
    // the load), Cc [NB][N] (c)
    float4* X = pcr_smem;
    float* A = (float*)(X + NB * N);
    float* Cc = A + NB * N;
    const int tid = threadIdx.x;
    // consecutive line groups share an XCD: the column pass's G-column blocks of one row band
    // read and write parts of the same cache lines, which then meet in one L2
    const int gx = gridDim.x;
    const int lb = xcd_block(blockIdx.x + gx * blockIdx.y, gx * gridDim.y);
    const int l0 = (lb % gx) * G;
    const size_t fo = (size_t)(lb / gx) * fstride;
    auto addr = [&](int idx, int& g, int& k) -> size_t {
        if (rows) {
            g = idx / n;
            k = idx - g * n;
            return (size_t)(l0 + g) * w + k;
        }
        k = idx / G;
        g = idx - k * G;
        return (size_t)k * w + l0 + g;
    };
    // ---- coalesced load into LDS: weight -> A[e], rhs -> X[e].z/.w ----
    for (int idx = tid; idx < N; idx += T) {
        int g, k;
        const size_t off = addr(idx, g, k);
        const int e = g * n + k;
        float cw = 0.0f, r0 = 0.0f, r1 = 0.0f;
        if (l0 + g < nlines) {
            cw = Cw[fo + off];
            r0 = U0[fo + off];
            if constexpr (TWO) r1 = U1[fo + off];
        }
        A[e] = cw;
        X[e] = make_float4(0.0f, 0.0f, r0, r1);
    }
    __syncthreads();
    float a[EPT], c[EPT], rs[EPT], b[EPT], d0[EPT], d1[EPT];
    int kk[EPT];
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int e = tid + j * T;
        kk[j] = 0;
        a[j] = c[j] = 0.0f;
        rs[j] = b[j] = 1.0f;
        d0[j] = d1[j] = 0.0f;
        if (e < N) {
            const int k = e - (e / n) * n;
            kk[j] = k;
            c[j] = lam * A[e];
            a[j] = k > 0 ? lam * A[e - 1] : 0.0f;
            rs[j] = 1.0f;
            b[j] = (1.0f - a[j]) - c[j];
            d0[j] = X[e].z;
            d1[j] = X[e].w;
        }
    }
    __syncthreads();
    int buf = 0;
    for (int s = 1; s < n; s <<= 1, buf ^= DB ? N : 0) {
        float4* Xb = X + buf;
        float* Ab = A + buf;
        float* Cb = Cc + buf;
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int e = tid + j * T;
            if (e < N) {
                Xb[e] = make_float4(rs[j], 1.0f / b[j], d0[j], d1[j]);
                Ab[e] = a[j];
                Cb[e] = c[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            // branch-free: all four reads in flight at once, missing neighbours selected to zero
            // (threads past N compute on a clamped equation and never publish)
            const int e = min(tid + j * T, N - 1);
            {
                const bool hm = kk[j] >= s, hp = kk[j] + s < n;
                const int em = hm ? e - s : e, ep = hp ? e + s : e;
                float4 xm = Xb[em], xp = Xb[ep];
                float am = Ab[em], cp = Cb[ep];
                const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (!hm) {
                    xm = z4;
                    am = 0.0f;
                }
                if (!hp) {
                    xp = z4;
                    cp = 0.0f;
                }
                const float k1 = a[j] * xm.y;
                const float k2 = c[j] * xp.y;
                const float na = -(am * k1);
                const float nc = -(cp * k2);
                const float ne = (rs[j] - xm.x * k1) - xp.x * k2;
                b[j] = (ne - na) - nc;
                a[j] = na;
                c[j] = nc;
                rs[j] = ne;
                d0[j] = (d0[j] - xm.z * k1) - xp.z * k2;
                if constexpr (TWO) d1[j] = (d1[j] - xm.w * k1) - xp.w * k2;
            }
        }
        if constexpr (!DB) __syncthreads();  // every read of the one buffer done before the next writes
    }
    // ---- decoupled: u = d / b, staged in LDS (buffer `buf`, untouched since two stages back) for
    // the coalesced store ----
    float4* Xo = X + buf;
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int e = tid + j * T;
        if (e < N) Xo[e] = make_float4(0.0f, 0.0f, d0[j] / b[j], TWO ? d1[j] / b[j] : 0.0f);
    }
    __syncthreads();
    for (int idx = tid; idx < N; idx += T) {
        int g, k;
        const size_t off = addr(idx, g, k);
        if (l0 + g >= nlines) continue;
        const float4 x = Xo[g * n + k];
        if constexpr (FIN) {
            // columns pass: line l0 + g is ROI column j, sample k its ROI row i
            wls_emit(wo, gw, lb / gx, gw.rx + l0 + g, gw.ry + k, wls_value(x.z, x.w));
        } else {
            U0[fo + off] = x.z;
            if constexpr (TWO) U1[fo + off] = x.w;
        }
    }
}

// FGS weights of one guide (per frame): Ch (weight between (i, j) and (i, j+1): column-major at
// j*h + i for the sequential sweep, row-major at i*w + j for k_fgs_pcr) and Cv (row-major:
// (i, j)-(i+1, j) at i*w + j)
__global__ __launch_bounds__(256) void k_fgs_weights(const uint8_t* __restrict__ guide, size_t gstride,
                                                     size_t gfstride, const float* __restrict__ lut,
                                                     int w, int h, int ch_rowmajor, float* __restrict__ ChT,
                                                     float* __restrict__ Cv) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (j >= w || i >= h) return;
    const uint8_t* g = guide + (size_t)blockIdx.z * gfstride + (size_t)i * gstride + j;
    // the sequential solver's layouts: Ch at j*hp + i, Cv at i*wp + j (fgs_pad4)
    const int wp = ch_rowmajor ? w : fgs_pad4(w), hp = ch_rowmajor ? h : fgs_pad4(h);
    const size_t fo = (size_t)blockIdx.z * wp * hp;
    const int v = g[0];
    float ch = 0.0f, cv = 0.0f;
    if (j + 1 < w) {
        const int d = v - g[1];
        ch = lut[d * d];
    }
    if (i + 1 < h) {
        const int d = v - g[gstride];
        cv = lut[d * d];
    }
    ChT[fo + (ch_rowmajor ? (size_t)i * w + j : (size_t)j * hp + i)] = ch;
    Cv[fo + (size_t)i * wp + j] = cv;
}

// dst[f][c][r] = src[f][r][c] for two arrays (rows x cols per frame), 64x64 LDS tiles
__global__ __launch_bounds__(256) void k_transpose2(const float* __restrict__ s0,
                                                    const float* __restrict__ s1, float* __restrict__ d0,
                                                    float* __restrict__ d1, int rows, int cols) {
    __shared__ float tile[2][64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
    const size_t fo = (size_t)blockIdx.z * rows * cols;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int rr = r0 + r, cc = c0 + tx;
        if (rr < rows && cc < cols) {
            tile[0][r][tx] = s0[fo + (size_t)rr * cols + cc];
            if (s1) tile[1][r][tx] = s1[fo + (size_t)rr * cols + cc];
        }
    }
    __syncthreads();
    for (int c = ty; c < 64; c += 4) {
        const int cc = c0 + c, rr = r0 + tx;
        if (rr < rows && cc < cols) {
            d0[fo + (size_t)cc * rows + rr] = tile[0][tx][c];
            if (s1) d1[fo + (size_t)cc * rows + rr] = tile[1][tx][c];
        }
    }
}

// The whole filter front end of one ROI row in one workgroup (grid: rows x frames), replacing
// k_wls_disc + k_wls_conf + k_fgs_weights:
//   1. vertical (2r+1)-row sums of d and d^2 of both maps over the row's window (BORDER_REFLECT_101
//      inside the ROI), one column per thread, into LDS (int32 / int64: exact integers)
//   2. horizontal sums of those -> the depth-discontinuity value of every ROI column of both maps
//      (the same integers as disc_at's 2-D loop, so the same floats) into LDS
//   3. the discontinuity-aware LR check of the row (its partner column x - (d >> 4) is in the same
//      row, so the row's right map is all it needs): full-size confidence x255, A = conf * d,
//      B = conf (ROI-compact)
//   4. the row's FGS weights from the guide (Ch row-major for k_fgs_pcr or column-major for the
//      sequential sweep, Cv row-major), computed in step 1's column loop
// Rows outside the ROI only get the confidence map's 255.  Dynamic LDS: 32 B per ROI column
// (int64 + int32 column sums and a float discontinuity value, per map).
template <int RMAX>
__global__ __launch_bounds__(256) void k_wls_prep(const int16_t* __restrict__ dl, const int16_t* __restrict__ dr,
                                                  WlsGeom g, const uint8_t* __restrict__ guide,
                                                  size_t gstride, size_t gfstride,
                                                  const float* __restrict__ lut, int ch_rowmajor,
                                                  float* __restrict__ conf_full, float* __restrict__ A,
                                                  float* __restrict__ B, float* __restrict__ ChW,
                                                  float* __restrict__ Cv, int border, WlsOut wo) {
    extern __shared__ int64_t wls_smem[];
    const int y = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, T = blockDim.x;
    const size_t fo = (size_t)f * g.W * g.H;
    const int i = y - g.ry;
    // border: this row's outputs outside the ROI (16 * (min_disp - 1)) are final now (the last FGS
    // pass writes the ROI's)
    if (border)
        for (int x = tid; x < g.W; x += T)
            if (i < 0 || i >= g.rh || x < g.rx || x >= g.rx + g.rw) wls_emit(wo, g, f, x, y, (int16_t)g.fill);
    if (i < 0 || i >= g.rh) {
        if (conf_full)
            for (int x = tid; x < g.W; x += T) conf_full[fo + (size_t)y * g.W + x] = 255.0f;
        return;
    }
    const int rw = g.rw, r = g.radius;
    int64_t* V2 = wls_smem;                // [2][rw] column sums of d^2 (left, right)
    int* V = (int*)(V2 + 2 * rw);          // [2][rw] column sums of d
    float* disc = (float*)(V + 2 * rw);    // [2][rw] discontinuity values
    const int16_t* L = dl + fo;
    const int16_t* R = dr + fo;
    // the window's rows (wave-uniform: one image row per workgroup), then all 2(2r+1) loads of a
    // column at once: RMAX taps unrolled, those past the radius loading a duplicate row and masked
    // (a runtime-length tap loop issued its loads one iteration at a time)
    size_t rowo[2 * RMAX + 1];
#pragma unroll
    for (int t = 0; t <= 2 * RMAX; t++)
        rowo[t] = (size_t)(g.ry + reflect101(i + min(max(t - RMAX, -r), r), g.rh)) * g.W;
    // the row's FGS weights from the guide (k_fgs_weights' formulas; the sequential solver's
    // layouts: Ch at j*hp + i, Cv at i*wp + j, fgs_pad4), computed in the first phase's column loop
    // so that their loads share its round trips
    const uint8_t* gr = guide + (size_t)f * gfstride + (size_t)(g.ry + i) * gstride + g.rx;
    const int wp = ch_rowmajor ? rw : fgs_pad4(rw), hp = ch_rowmajor ? g.rh : fgs_pad4(g.rh);
    const size_t wfo = (size_t)f * wp * hp;
    const int gs = i + 1 < g.rh ? (int)gstride : 0;
    for (int j = tid; j < rw; j += T) {
        int vl[2 * RMAX + 1], vr[2 * RMAX + 1];
        const int gv = gr[j], gh = gr[min(j + 1, rw - 1)], gd = gr[gs + j];
#pragma unroll
        for (int t = 0; t <= 2 * RMAX; t++) {
            vl[t] = L[rowo[t] + g.rx + j];
            vr[t] = R[rowo[t] + g.rrx + j];
        }
        {
            // (unconditional lookups from clamped neighbours, then the edges' zeros)
            const int dh = gv - gh, dv = gv - gd;
            const float ch = lut[dh * dh], cv = lut[dv * dv];
            ChW[wfo + (ch_rowmajor ? (size_t)i * rw + j : (size_t)j * hp + i)] = j + 1 < rw ? ch : 0.0f;
            Cv[wfo + (size_t)i * wp + j] = gs ? cv : 0.0f;
        }
        int s0 = 0, s1 = 0;
        int64_t q0 = 0, q1 = 0;
#pragma unroll
        for (int t = 0; t <= 2 * RMAX; t++) {
            const int a = t - RMAX;
            const int ml = a >= -r && a <= r ? vl[t] : 0, mr = a >= -r && a <= r ? vr[t] : 0;
            s0 += ml;
            q0 += (int64_t)ml * ml;
            s1 += mr;
            q1 += (int64_t)mr * mr;
        }
        V[j] = s0;
        V[rw + j] = s1;
        V2[j] = q0;
        V2[rw + j] = q1;
    }
    __syncthreads();
    // BORDER_REFLECT_101 of a column index one reflection deep (rw > RMAX; narrower ROIs loop)
    const bool shallow = rw > RMAX;
    auto refl = [&](int p) { return shallow ? (p < 0 ? -p : p >= rw ? 2 * rw - 2 - p : p) : reflect101(p, rw); };
    for (int j = tid; j < rw; j += T) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            long long s = 0, s2 = 0;
#pragma unroll
            for (int t = 0; t <= 2 * RMAX; t++) {
                const int b = t - RMAX;
                if (b < -r || b > r) continue;  // uniform
                const int jj = refl(j + b);
                s += V[m * rw + jj];
                s2 += V2[m * rw + jj];
            }
            const float mean = (float)((double)s * g.scale);
            const float msq = (float)((double)s2 * g.scale);
            const float var = msq - mean * mean;
            const float c = 1.0f - g.roll_off * var;
            disc[m * rw + j] = c > 0.0f ? c : 0.0f;
        }
    }
    __syncthreads();
    const size_t cf = (size_t)f * rw * g.rh + (size_t)i * rw;
    for (int x = tid; x < g.W; x += T) {
        const size_t o = (size_t)y * g.W + x;
        const int j = x - g.rx;
        const bool in_roi = j >= 0 && j < rw;
        float c = 1.0f;
        int v = 0;
        if (in_roi) {
            c = disc[j];
            v = L[o];
            const int ridx = x - (v >> 4);
            if (ridx >= g.rrx && ridx < g.rrx + rw) {
                if (abs(v + (int)R[(size_t)y * g.W + ridx]) < g.lrc_thresh) {
                    const float rc = disc[rw + ridx - g.rrx];
                    c = c < rc ? c : rc;
                } else {
                    c = 0.0f;
                }
            }
        }
        const float conf = 255.0f * c;
        if (conf_full) conf_full[fo + o] = conf;
        if (in_roi) {
            if (ch_rowmajor) {
                A[cf + j] = conf * (float)v;
                B[cf + j] = conf;
            } else {
                // the sequential solver's first pass reads them transposed ([column][row]), the two
                // right-hand sides interleaved (A is its pass buffer, B unused)
                ((float2*)A)[(size_t)f * fgs_pad4(rw) * fgs_pad4(g.rh) + (size_t)j * fgs_pad4(g.rh) + i] =
                    make_float2(conf * (float)v, conf);
            }
        }
    }

}

// saturate_cast<short>(float): round half to even, saturate; 0 where FGS(conf) == 0 (cv::divide
// of floats returns 0 for a zero divisor)
// Optional epilogue of the class path (stereo_disparity.cpp:34, :76-80), fused: fout = out / 16
// (convertTo(CV_32F, 1/16)) and xyz = reprojectImageTo3D(fout, Q) (computeDepth,
// handleMissing = false).
__global__ __launch_bounds__(256) void k_wls_final(const float* __restrict__ A,
                                                   const float* __restrict__ B, WlsGeom g, WlsOut wo) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.W || y >= g.H) return;
    const int j = x - g.rx, i = y - g.ry;
    int16_t r = (int16_t)g.fill;
    if (j >= 0 && j < g.rw && i >= 0 && i < g.rh) {
        const size_t co = (size_t)blockIdx.z * g.rw * g.rh + (size_t)i * g.rw + j;
        r = wls_value(A[co], B[co]);
    }
    wls_emit(wo, g, blockIdx.z, x, y, r);
}

// FastGlobalSmootherFilter::filter on nimg (1 or 2) row-major w x h images per frame (R0, R1, in
// place), F frames sharing per-frame guides.  Scratch, in frames of fsp = fgs_pad4(w) *
// fgs_pad4(h) samples (SDR_FGS_PCR uses ChT and Cv only, w * h a frame):
struct FgsScratch {
    float *A, *B;    // the sequential solver's two pass layouts (2 floats a sample), F frames each
    float *ChT, *Cv; // the weights, F frames each
    float* coef;     // the sequential solver's coefficients of each of the 2 * iters passes:
                     // [F * fsp] float4 (a, den, 1/den, t) then [F * fsp] t (5 * F * fsp floats)
};

#ifdef SDR_TH_STAMPS
static unsigned long long* th_stamp_buf = nullptr;
#endif

template <int LPB>
static void launch_fgs_th_lpb(const dim3& grid, const FgsThArgs& a, bool two, hipStream_t st) {
    if (two) hipLaunchKernelGGL((k_fgs_th<true, LPB>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_fgs_th<false, LPB>), grid, dim3(256), 0, st, a);
}

// One k_fgs_th launch: the pass (a.nl lines; none when !pass) or its jobs, with the fewest lines
// a workgroup (LPB) whose workgroups still all fit on the chip at once (one a CU: the LDS ring),
// so that every chain runs on a CU's memory pipeline shared with as few lines as possible.
static void launch_fgs_th(FgsThArgs a, bool pass, bool two, int F, hipStream_t st) {
    const int cus = device_cus();
    int lpb = 64;
#ifdef SDR_TH_FORCE_LPB
    for (int c : {SDR_TH_FORCE_LPB}) {
#else
    for (int c : {16, 32, 64}) {
#endif
        int blocks = pass ? (a.nl + c - 1) / c : 0;
        for (int j = 0; j < a.njobs; j++) blocks += (a.job[j].nl + c - 1) / c;
        if ((long long)blocks * F <= cus) {
            lpb = c;
            break;
        }
    }
    a.main_blocks = pass ? (a.nl + lpb - 1) / lpb : 0;
    int blocks = a.main_blocks;
    for (int j = 0; j < a.njobs; j++) blocks += a.job[j].blocks = (a.job[j].nl + lpb - 1) / lpb;
    const dim3 grid(blocks, F);
#ifdef SDR_TH_STAMPS
    {
        static int launches = 0;
        static unsigned long long* buf = nullptr;
        static const int want = getenv("SDR_TH_STAMP_LAUNCH") ? atoi(getenv("SDR_TH_STAMP_LAUNCH")) : -1;
        if (!buf) (void)hipMalloc((void**)&buf, kThStampRoles * 1024 * 8);
        unsigned long long* v = launches++ == want ? buf : nullptr;
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_th_stamps), &v, sizeof(v), 0, hipMemcpyHostToDevice, st);
        th_stamp_buf = buf;
    }
#endif
    if (lpb == 16) launch_fgs_th_lpb<16>(grid, a, two, st);
    else if (lpb == 32) launch_fgs_th_lpb<32>(grid, a, two, st);
    else launch_fgs_th_lpb<64>(grid, a, two, st);
}

// One k_fgs_lr launch when the pass's lines fit in LDS (two right-hand sides, n <= 6 * 1024 / L
// for some L of 16, 8, 4, 2 lines a workgroup: the largest that fits); false: take k_fgs_th.
static bool launch_fgs_lr(FgsThArgs a, bool two, int F, hipStream_t st) {
    static const bool off = getenv("SDR_FGS_LR") && atoi(getenv("SDR_FGS_LR")) == 0;  // A/B knob
    if (!two || off) return false;
#ifdef SDR_TH_STAMPS
    static int slot = 0;
    a.dbg = slot++ & 15;
#else
    a.dbg = -1;
#endif
    // at most 8 lines a workgroup by default (profiles/r6_fgs_lr_maxl.txt, C4): the 360-sample
    // column passes on 16 lines ran ~15 % slower a sample than the row passes on 8 (the four rows'
    // reads of 16 distinct lines conflict in LDS); capped at 8, one stream 0.4195 -> 0.413 ms with
    // 6 frames in flight unchanged within noise; at 4, one stream 0.4123 ms but 6 frames in flight
    // 4128 -> 3948 fps (a workgroup of ~147 KiB LDS per CU, 4x as many)
    static const int maxl = getenv("SDR_FGS_LR_MAXL") ? atoi(getenv("SDR_FGS_LR_MAXL")) : 8;  // A/B knob
    for (int L : {16, 8, 4, 2}) {
        if (L > maxl || a.n > kLrChunks * 1024 / L) continue;
        const dim3 grid((a.nl + L - 1) / L, F);
        if (L == 16) hipLaunchKernelGGL(k_fgs_lr<16>, grid, dim3(256), 0, st, a);
        else if (L == 8) hipLaunchKernelGGL(k_fgs_lr<8>, grid, dim3(256), 0, st, a);
        else if (L == 4) hipLaunchKernelGGL(k_fgs_lr<4>, grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_fgs_lr<2>, grid, dim3(256), 0, st, a);
        return true;
    }
    return false;
}

// One k_fgs_lrjob launch for the jobs of c when every job's lines fit in LDS (n <= 6 * 1024 / L
// for L of 16, 8, 4 lines a workgroup: the largest that fits, per job); false: take k_fgs_th.
static bool launch_fgs_lrjob(FgsThArgs c, int F, hipStream_t st) {
    static const bool off = getenv("SDR_FGS_LRJOB") && atoi(getenv("SDR_FGS_LRJOB")) == 0;  // A/B knob
    if (off || c.njobs <= 0) return false;
    int blocks = 0;
    for (int j = 0; j < c.njobs; j++) {
        FgsCoefJob& J = c.job[j];
        J.lpb = 0;
        for (int L : {16, 8, 4})  // (2 lines: the weights' 8-byte rows are not whole DMA pieces)
            if (J.n <= kLrChunks * 1024 / L) {
                J.lpb = L;
                break;
            }
        if (!J.lpb) return false;
        J.blocks = (J.nl + J.lpb - 1) / J.lpb;
        blocks += J.blocks;
    }
    c.main_blocks = 0;
    hipLaunchKernelGGL(k_fgs_lrjob, dim3(blocks, F), dim3(256), 0, st, c);
    return true;
}

// k_fgs_pcr instance for G*n samples per block: one equation per thread up to 1024 samples
// (T = the samples rounded up to whole waves), 2 or 4 per thread of 1024 beyond
template <bool TWO, bool FIN = false>
static int launch_pcr(float* U0, float* U1, const float* Cw, int w, int h, int F, int rows,
                      float lam, hipStream_t st, const WlsGeom& gw = {}, const WlsOut& wo = {}) {
    const int n = rows ? w : h, nlines = rows ? h : w;
    if (n > kPcrMaxN) return -1;
    // short lines: G per block so that a block holds up to 1024 samples
    const int G = std::max(1, std::min(nlines, 1024 / n));
    const int N = G * n;
    // (one equation per thread: 2 or 4 per thread at 640x360 measured 12.8 -> 15.0 / 16.8 us a pass)
    const int ept = N <= 1024 ? 1 : N <= 2048 ? 2 : 4;
    const int T = std::min(1024, ((N + ept - 1) / ept + 63) / 64 * 64);
    const dim3 grid((nlines + G - 1) / G, F), blk(T);
    const size_t fs = (size_t)w * h;
    // the workgroup's LDS (160 KiB on gfx950) holds double-buffered stages up to 3413 samples
    static thread_local int max_lds = 0;
    if (!max_lds) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
            max_lds <= 0)
            max_lds = 64 * 1024;
    }
    const bool db = (size_t)N * 48 <= (size_t)max_lds;
    if (!db && (size_t)N * 24 > (size_t)max_lds) return -1;
    if (!db) {
        hipLaunchKernelGGL((k_fgs_pcr<4, TWO, false, FIN>), grid, blk, (size_t)N * 24, st, U0, U1, Cw, w, h, fs,
                           rows, G, lam, gw, wo);
        return 0;
    }
    const size_t lds = (size_t)N * 48;
    if (ept == 1)
        hipLaunchKernelGGL((k_fgs_pcr<1, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    else if (ept == 2)
        hipLaunchKernelGGL((k_fgs_pcr<2, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    else
        hipLaunchKernelGGL((k_fgs_pcr<4, TWO, true, FIN>), grid, blk, lds, st, U0, U1, Cw, w, h, fs, rows, G, lam, gw, wo);
    return 0;
}

// FastGlobalSmootherFilter::filter on R0 (and R1 when non-null: a second right-hand side of the
// same systems), row-major w x h per frame, F frames with per-frame guides, in place.
//   SDR_FGS_THOMAS: weights (ChT column-major = the row pass's k-major, Cv row-major = the column
//                   pass's), the right-hand sides transposed into s.A (in_transposed: the caller
//                   already wrote them there), one launch of coefficient jobs (every pass's
//                   (a, den, 1/den, t)), then the passes of k_fgs_th alternating between the two
//                   layouts (row pass: s.A -> s.B, column pass: s.B -> s.A; the last column pass
//                   into R0 / R1): 2 * iters + 1 launches
//   SDR_FGS_PCR:    weights (Ch, Cv row-major), then per iteration k_fgs_pcr over the rows and
//                   over the columns of the images themselves (2 launches per iteration)
static int launch_fgs(const uint8_t* guide, size_t gstride, size_t gfstride, const float* lut,
                      float* R0, float* R1, int w, int h, int F, double lambda, double att,
                      int iters, int solver, const FgsScratch& s, hipStream_t st,
                      bool weights_ready = false, sdr_sgbm* timer = nullptr,
                      const WlsGeom* fin_g = nullptr, const WlsOut* fin_o = nullptr,
                      bool in_transposed = false) {
    const size_t fs = (size_t)w * h;
    const bool pcr = solver == SDR_FGS_PCR;
    if (!weights_ready)
        hipLaunchKernelGGL(k_fgs_weights, dim3((w + 63) / 64, (h + 3) / 4, F), dim3(256), 0, st, guide,
                           gstride, gfstride, lut, w, h, pcr ? 1 : 0, s.ChT, s.Cv);
    float lam = (float)lambda;
    const float fa = (float)att;
    if (!pcr) {
        if (iters <= 0) return 0;
        const bool two = R1 != nullptr;
        if (!in_transposed)
            hipLaunchKernelGGL(k_fgs_pack, dim3((w + 63) / 64, (h + 63) / 64, F), dim3(256), 0, st, R0, R1, s.A, h, w);
        const int npass = 2 * iters;
        // pass p: iteration p / 2, rows (even p: lines = rows, k = column) or columns (odd p);
        // k-major arrays with sample rows of fgs_pad4(lines)
        const int wp = fgs_pad4(w), hp = fgs_pad4(h);
        const size_t fsp = (size_t)wp * hp;
        std::vector<float> lams(iters);
        for (int it = 0; it < iters; it++, lam = lam * fa) lams[it] = lam;  // lambda *= attenuation
        auto pass_args = [&](int p) {
            FgsThArgs a{};
            const bool rows = (p & 1) == 0;
            a.nl = rows ? h : w;
            a.n = rows ? w : h;
            a.st = rows ? hp : wp;
            a.onp = rows ? wp : hp;
            a.fs = fsp;
            a.ost = (size_t)w;
            a.ofs = fs;
            // rows: transposed (s.A) -> row-major (s.B); columns: row-major (s.B) -> transposed (s.A),
            // the last pass split back into R0 / R1
            a.U = rows ? s.A : s.B;
            const bool last = p == npass - 1;
            a.O = last ? nullptr : rows ? s.B : s.A;
            a.O0 = last ? R0 : nullptr;
            a.O1 = last ? R1 : nullptr;
            // the pass's coefficient block: float4 (a, den, 1/den, t), then t alone
            float* cb = s.coef + (size_t)p * 5 * F * fsp;
            a.coef = (const float4*)cb;
            a.tt = cb + 4 * F * fsp;
            return a;
        };
        // the coefficient jobs of every pass (kFgsMaxJobs a launch), then the passes
        for (int p0 = 0; p0 < npass; p0 += kFgsMaxJobs) {
            FgsThArgs c{};
            c.fs = fsp;
            for (int p = p0; p < npass && c.njobs < kFgsMaxJobs; p++) {
                const FgsThArgs q = pass_args(p);
                const bool rows = (p & 1) == 0;
                FgsCoefJob& j = c.job[c.njobs++];
                j.Cw = rows ? s.ChT : s.Cv;
                j.coef = (float4*)q.coef;
                j.tt = (float*)q.tt;
                j.lam = lams[p / 2];
                j.nl = q.nl;
                j.n = q.n;
                j.st = q.st;
            }
            KScope kt(timer, SDR_KERNEL_FGS_COEF);
            if (!launch_fgs_lrjob(c, F, st)) launch_fgs_th(c, false, two, F, st);
        }
        for (int p = 0; p < npass; p++) {
            KScope kt(timer, SDR_KERNEL_FGS);
            const FgsThArgs a = pass_args(p);
            if (!launch_fgs_lr(a, two, F, st)) launch_fgs_th(a, true, two, F, st);
        }
        return 0;
    }
    for (int it = 0; it < iters; it++) {
        int e1, e2;
        {
            KScope kt(timer, SDR_KERNEL_FGS);
            e1 = R1 ? launch_pcr<true>(R0, R1, s.ChT, w, h, F, 1, lam, st)
                    : launch_pcr<false>(R0, R1, s.ChT, w, h, F, 1, lam, st);
        }
        {
            KScope kt(timer, SDR_KERNEL_FGS);
            // the last column pass writes the filter's outputs itself (fin_g / fin_o)
            if (fin_g && R1 && it == iters - 1)
                e2 = launch_pcr<true, true>(R0, R1, s.Cv, w, h, F, 0, lam, st, *fin_g, *fin_o);
            else
                e2 = R1 ? launch_pcr<true>(R0, R1, s.Cv, w, h, F, 0, lam, st)
                        : launch_pcr<false>(R0, R1, s.Cv, w, h, F, 0, lam, st);
        }
        if (e1 || e2) return -1;
        lam = lam * fa;  // FastGlobalSmootherFilterImpl::filter: lambda *= lambda_attenuation
    }
    return 0;
}

// ComputeLUT_ParBody: LUT[i] = -exp(-sqrt((float)i) / sigmaColor), float math on the host
static void fgs_lut_host(double sigma, std::vector<float>* lut) {
    lut->resize(kFgsLevels);
    const float s = (float)sigma;
    for (int i = 0; i < kFgsLevels; i++) (*lut)[i] = -expf(-sqrtf((float)i) / s);
}

}  // namespace sdr

// ===========================================================================================
// C ABI (include/sdr/sdr.h)
// ===========================================================================================
struct sdr_wls {
    sdr_wls_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    sdr::Buf rdisc, conf, A, B, Ac, Bc, ChT, Cv, lut, out, hbuf, coef;
    double lut_sigma = -1.0;
};

namespace {

#define WLS_HIP(call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return sdr::set_error(SDR_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// The sequential solver's exact division needs every pass's pivots in [1, 2^126): each pass's
// lambda (lambda * attenuation^k, in launch_fgs's float arithmetic) in [0, kFgsThomasMaxLambda]
// (an attenuation above 1 or below 0 used to pass with only the first checked)
bool thomas_lambdas_ok(double lambda, double att, int iters) {
    float lam = (float)lambda;
    const float fa = (float)att;
    for (int it = 0; it < iters; it++, lam = lam * fa)
        if (!(lam >= 0.0f) || !((double)lam <= sdr::kFgsThomasMaxLambda)) return false;
    return true;
}
constexpr const char* kThomasLambdaMsg =
    "SDR_FGS_THOMAS needs every pass's lambda * attenuation^k in [0, 2^100] (its pivots stay in [1, 2^126))";

int check_wls_params(const sdr_wls_params& p) {
    if (!(p.lambda >= 0.0) || !(p.sigma_color >= 0.0) || p.num_iter < 1)
        return sdr::set_error(SDR_ERR_ARG, "FGS needs lambda >= 0, sigma_color >= 0, num_iter >= 1");
    if (p.fgs_solver == SDR_FGS_THOMAS && !thomas_lambdas_ok(p.lambda, p.lambda_attenuation, p.num_iter))
        return sdr::set_error(SDR_ERR_ARG, kThomasLambdaMsg);
    if (p.fgs_solver != SDR_FGS_PCR && p.fgs_solver != SDR_FGS_THOMAS)
        return sdr::set_error(SDR_ERR_ARG, "fgs_solver must be SDR_FGS_PCR or SDR_FGS_THOMAS");
    if (p.depth_discontinuity_radius < 0 || p.left_offset < 0 || p.right_offset < 0 ||
        p.top_offset < 0 || p.bottom_offset < 0)
        return sdr::set_error(SDR_ERR_ARG, "negative WLS radius or offset");
    return SDR_OK;
}

int upload_lut(sdr_wls* h, double sigma, const float** out) {
    int rc;
    if ((rc = sdr::ensure(h->lut, sizeof(float) * sdr::kFgsLevels))) return rc;
    if (h->lut_sigma != sigma) {
        std::vector<float> lut;
        sdr::fgs_lut_host(sigma, &lut);
        WLS_HIP(hipMemcpy(h->lut.p, lut.data(), sizeof(float) * lut.size(), hipMemcpyHostToDevice));
        h->lut_sigma = sigma;
    }
    *out = (const float*)h->lut.p;
    return SDR_OK;
}

}  // namespace

extern "C" {

void sdr_wls_params_for_sgbm(sdr_sgbm_params* m, sdr_wls_params* p) {
    if (!m || !p) return;
    // createDisparityWLSFilter(Ptr<StereoMatcher>) [ximgproc disparity_filters.cpp]:
    // setDisp12MaxDiff(1000000), setSpeckleWindowSize(0), and for SGBM setUniquenessRatio(0);
    // offsets (max(0, minD+numD), max(0, -minD), 0, 0); radius ceil(0.5 * blockSize)
    m->disp12MaxDiff = 1000000;
    m->speckleWindowSize = 0;
    m->uniquenessRatio = 0;
    const int l = m->minDisparity + m->numDisparities;
    p->lambda = 8000.0;
    p->sigma_color = 1.5;
    p->lrc_thresh = 24;
    p->depth_discontinuity_radius = (int)std::ceil(0.5 * m->blockSize);
    p->roll_off = 0.001f;
    p->lambda_attenuation = 0.25;
    p->num_iter = 3;
    p->left_offset = l > 0 ? l : 0;
    p->right_offset = m->minDisparity < 0 ? -m->minDisparity : 0;
    p->top_offset = 0;
    p->bottom_offset = 0;
    p->min_disp = m->minDisparity;
    p->fgs_solver = SDR_FGS_THOMAS;  // ximgproc's own elimination order (sdr.h)
}

int sdr_wls_create(const sdr_wls_params* p, int device, sdr_wls** out) {
    if (!p || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    int rc = check_wls_params(*p);
    if (rc) return rc;
    WLS_HIP(hipSetDevice(device));
    sdr_wls* h = new sdr_wls();
    h->p = *p;
    h->device = device;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return sdr::set_error(SDR_ERR_DEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    *out = h;
    return SDR_OK;
}

int sdr_wls_destroy(sdr_wls* h) {
    if (!h) return SDR_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (sdr::Buf* b : {&h->rdisc, &h->conf, &h->A, &h->B, &h->Ac, &h->Bc, &h->ChT, &h->Cv,
                        &h->lut, &h->out, &h->hbuf, &h->coef})
        if (b->p) (void)hipFree(b->p);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return SDR_OK;
}

int sdr_wls_set_params(sdr_wls* h, const sdr_wls_params* p) {
    if (!h || !p) return sdr::set_error(SDR_ERR_ARG, "null argument");
    int rc = check_wls_params(*p);
    if (rc) return rc;
    h->p = *p;
    return SDR_OK;
}

int sdr_wls_get_params(const sdr_wls* h, sdr_wls_params* p) {
    if (!h || !p) return sdr::set_error(SDR_ERR_ARG, "null argument");
    *p = h->p;
    return SDR_OK;
}

int sdr_wls_set_stream(sdr_wls* h, void* stream) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = (hipStream_t)stream;  // NULL = the HIP null (legacy default) stream
    return SDR_OK;
}

int sdr_wls_reset_stream(sdr_wls* h) {
    if (!h) return sdr::set_error(SDR_ERR_ARG, "null handle");
    h->stream = h->own_stream;
    return SDR_OK;
}

void* sdr_wls_get_stream(const sdr_wls* h) { return h ? (void*)h->stream : nullptr; }

int sdr_wls_get_roi(const sdr_wls* h, int W, int H, int roi[4]) {
    if (!h || !roi) return sdr::set_error(SDR_ERR_ARG, "null argument");
    roi[0] = h->p.left_offset;
    roi[1] = h->p.top_offset;
    roi[2] = W - h->p.left_offset - h->p.right_offset;
    roi[3] = H - h->p.top_offset - h->p.bottom_offset;
    return SDR_OK;
}

}  // extern "C"

// DisparityWLSFilter::filter on device with the class path's optional fused epilogue (fout =
// out / 16, xyz = reprojectImageTo3D(fout, Q)); sdr_wls_filter_device is this with neither.
// ROIs up to kPcrMaxN columns take the fused front end (k_wls_prep: discontinuity maps, LR check,
// confidence, FGS weights in one launch); wider ones the per-pixel k_wls_disc / k_wls_conf /
// k_fgs_weights kernels.
int sdr::wls_filter_enqueue(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide,
                            int W, int H, size_t gstride, size_t gfstride, int F, int16_t* out,
                            float* conf, float* fout, const double* Q, float* xyz, sdr_sgbm* timer) {
    if (!h || !dl || !dr || !guide || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || F <= 0 || gstride < (size_t)W || (F > 1 && gfstride < gstride * H))
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    if (xyz && (!fout || !Q)) return sdr::set_error(SDR_ERR_ARG, "the fused reprojection needs fout and Q");
    WLS_HIP(hipSetDevice(h->device));
    hipStream_t st = h->stream;
    const sdr_wls_params& p = h->p;
    sdr::WlsGeom g{};
    g.W = W;
    g.H = H;
    g.rx = p.left_offset;
    g.ry = p.top_offset;
    g.rw = W - p.left_offset - p.right_offset;
    g.rh = H - p.top_offset - p.bottom_offset;
    g.rrx = W - (g.rx + g.rw);
    g.radius = p.depth_discontinuity_radius;
    const int k = 2 * g.radius + 1;
    g.scale = 1.0 / (double)(k * k);
    g.roll_off = p.roll_off;
    g.lrc_thresh = p.lrc_thresh;
    g.fill = 16 * (p.min_disp - 1);
    const size_t px = (size_t)W * H;
    const bool roi = g.rw > 0 && g.rh > 0;
    if (roi && p.fgs_solver == SDR_FGS_PCR && (g.rw > sdr::kPcrMaxN || g.rh > sdr::kPcrMaxN))
        return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                            "(use SDR_FGS_THOMAS for larger ROIs)");
    const bool fused = roi && g.rw <= sdr::kPcrMaxN && g.radius <= 9;
    const size_t cpx = roi ? (size_t)g.rw * g.rh : 0;
    int rc;
    const float* lut = nullptr;
    if (!fused && (rc = sdr::ensure(h->rdisc, F * px * 4))) return rc;
    // the sequential solver's k-major arrays: sample rows padded to 4 lines (fgs_pad4), and room
    // for its loaders' reads past the last row (kFgsOverread)
    const size_t cpp = roi ? (size_t)sdr::fgs_pad4(g.rw) * sdr::fgs_pad4(g.rh) : 0;
    const size_t ov = sdr::kFgsOverread;
    for (sdr::Buf* b : {&h->A, &h->B})
        if ((rc = sdr::ensure(*b, F * cpx * 4 + 4))) return rc;
    for (sdr::Buf* b : {&h->ChT, &h->Cv})
        if ((rc = sdr::ensure(*b, F * cpp * 4 + ov))) return rc;
    if (p.fgs_solver == SDR_FGS_THOMAS) {
        // the two pass layouts (both right-hand sides interleaved) and every pass's elimination
        // coefficients (float4 (a, den, 1/den, t) and t: 20 bytes a sample and pass)
        for (sdr::Buf* b : {&h->Ac, &h->Bc})
            if ((rc = sdr::ensure(*b, F * cpp * 8 + ov))) return rc;
        if ((rc = sdr::ensure(h->coef, (size_t)std::max(2 * p.num_iter, 0) * F * cpp * 20 + ov))) return rc;
    }
    if ((rc = upload_lut(h, p.sigma_color, &lut))) return rc;
    float* A = (float*)h->A.p;
    float* B = (float*)h->B.p;
    const dim3 blk(256);
    const bool rowmajor = p.fgs_solver == SDR_FGS_PCR;
    // the sequential solver's first pass (rows) reads the right-hand sides transposed: the fused
    // front end writes them there directly
    float* Ain = rowmajor ? A : (float*)h->Ac.p;
    float* Bin = rowmajor ? B : nullptr;
    const dim3 grid((W + 63) / 64, (H + 3) / 4, F);
    sdr::WlsOut wo{out, fout, xyz, {}};
    if (Q)
        for (int t = 0; t < 16; t++) wo.Q.q[t] = Q[t];
    // with the default solver the outputs need no pass of their own: k_wls_prep writes the pixels
    // outside the ROI and the last FGS column pass the ROI's (k_wls_final otherwise)
    const bool fin_fused = fused && roi && p.fgs_solver == SDR_FGS_PCR;
    if (fused) {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_PREP);
        // the window radius is ceil(blockSize / 2) <= 9 for every valid SGBM block; wider ones
        // (setDepthDiscontinuityRadius) take the per-pixel kernels below
        if (g.radius <= 4)
            hipLaunchKernelGGL(sdr::k_wls_prep<4>, dim3(H, F), blk, (size_t)g.rw * 32, st, dl, dr, g, guide,
                               gstride, gfstride, lut, rowmajor ? 1 : 0, conf, Ain, Bin, (float*)h->ChT.p,
                               (float*)h->Cv.p, fin_fused ? 1 : 0, wo);
        else
            hipLaunchKernelGGL(sdr::k_wls_prep<9>, dim3(H, F), blk, (size_t)g.rw * 32, st, dl, dr, g, guide,
                               gstride, gfstride, lut, rowmajor ? 1 : 0, conf, Ain, Bin, (float*)h->ChT.p,
                               (float*)h->Cv.p, fin_fused ? 1 : 0, wo);
    } else {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_PREP);
        if (roi)
            hipLaunchKernelGGL(sdr::k_wls_disc, dim3((g.rw + 63) / 64, (g.rh + 3) / 4, F), blk, 0, st,
                               dr, g, (float*)h->rdisc.p);
        hipLaunchKernelGGL(sdr::k_wls_conf, grid, blk, 0, st, dl, dr, (const float*)h->rdisc.p, g,
                           conf, A, B);
    }
    if (roi) {
        const uint8_t* g0 = guide + (size_t)g.ry * gstride + g.rx;
        const sdr::FgsScratch fs{(float*)h->Ac.p, (float*)h->Bc.p, (float*)h->ChT.p,
                                 (float*)h->Cv.p, (float*)h->coef.p};
        if (sdr::launch_fgs(g0, gstride, gfstride, lut, A, B, g.rw, g.rh, F, p.lambda,
                            p.lambda_attenuation, p.num_iter, p.fgs_solver, fs, st, fused, timer,
                            fin_fused ? &g : nullptr, fin_fused ? &wo : nullptr, fused && !rowmajor))
            return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                                "(use SDR_FGS_THOMAS for larger ROIs)");
        if (fin_fused) {
            WLS_HIP(hipGetLastError());
            return SDR_OK;
        }
    }
    {
        sdr::KScope kt(timer, SDR_KERNEL_WLS_FINAL);
        hipLaunchKernelGGL(sdr::k_wls_final, grid, blk, 0, st, A, B, g, wo);
    }
    WLS_HIP(hipGetLastError());
    return SDR_OK;
}

extern "C" {

int sdr_wls_filter_device(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide,
                          int W, int H, size_t gstride, size_t gfstride, int F, int16_t* out,
                          float* conf) {
    return sdr::wls_filter_enqueue(h, dl, dr, guide, W, H, gstride, gfstride, F, out, conf, nullptr,
                                   nullptr, nullptr);
}

int sdr_wls_filter(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide, int W,
                   int H, size_t gstride, int16_t* out, float* conf) {
    if (!h || !dl || !dr || !guide || !out) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || gstride < (size_t)W) return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    WLS_HIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    // device staging: dl, dr, guide, out (int16), conf (float)
    int rc;
    if ((rc = sdr::ensure(h->hbuf, px * (2 + 2 + 1 + 2 + 4) + 64))) return rc;
    uint8_t* base = (uint8_t*)h->hbuf.p;
    float* dconf = (float*)base;
    int16_t* ddl = (int16_t*)(base + px * 4);
    int16_t* ddr = ddl + px;
    int16_t* dout = ddr + px;
    uint8_t* dg = (uint8_t*)(dout + px);
    hipStream_t st = h->stream;
    WLS_HIP(hipMemcpyAsync(ddl, dl, px * 2, hipMemcpyHostToDevice, st));
    WLS_HIP(hipMemcpyAsync(ddr, dr, px * 2, hipMemcpyHostToDevice, st));
    WLS_HIP(hipMemcpy2DAsync(dg, W, guide, gstride, W, H, hipMemcpyHostToDevice, st));
    if ((rc = sdr_wls_filter_device(h, ddl, ddr, dg, W, H, W, px, 1, dout, conf ? dconf : nullptr)))
        return rc;
    WLS_HIP(hipMemcpyAsync(out, dout, px * 2, hipMemcpyDeviceToHost, st));
    if (conf) WLS_HIP(hipMemcpyAsync(conf, dconf, px * 4, hipMemcpyDeviceToHost, st));
    WLS_HIP(hipStreamSynchronize(st));
    return SDR_OK;
}

// sdr_fgs_rcp_selftest: fgs_rcp against the IEEE division for all 2^23 mantissas of d in
// [2^e, 2^(e+1))
namespace sdr {
__global__ __launch_bounds__(256) void k_fgs_rcp_check(int e, unsigned int* bad) {
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    const float d = __builtin_bit_cast(float, (uint32_t)(127 + e) << 23 | m);
    const volatile float one = 1.0f;
    if (__builtin_bit_cast(uint32_t, fgs_rcp(d)) != __builtin_bit_cast(uint32_t, one / d)) atomicAdd(bad, 1u);
}
}  // namespace sdr

int sdr_fgs_rcp_selftest(int e, unsigned int* mismatches) {
    if (!mismatches || e < 0 || e > 126) return sdr::set_error(SDR_ERR_ARG, "e must be in [0, 126]");
    unsigned int* d = nullptr;
    WLS_HIP(hipMalloc((void**)&d, 4));
    hipError_t err = hipMemset(d, 0, 4);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(sdr::k_fgs_rcp_check, dim3((1u << 23) / 256), dim3(256), 0, 0, e, d);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipMemcpy(mismatches, d, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    WLS_HIP(err);
    return SDR_OK;
}

#ifdef SDR_TH_STAMPS
// diagnostic build only: the stamps of the launch SDR_TH_STAMP_LAUNCH names ([5][1024] u64)
int sdr_th_blocks(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sdr::g_th_blk), 512 * 3 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int sdr_lr_blocks(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sdr::g_lr_blk), 16 * 512 * 8 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int sdr_lj_blocks(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sdr::g_lj_blk), 512 * 8 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int sdr_th_counts(unsigned int* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sdr::g_th_counts), 16, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int sdr_th_stamps(unsigned long long* host) {
    if (!sdr::th_stamp_buf) return -1;
    return hipMemcpy(host, sdr::th_stamp_buf, sdr::kThStampRoles * 1024 * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

int sdr_fgs_filter_device(const uint8_t* d_guide, size_t gstride, int w, int h, double lambda,
                          double sigma, double att, int iters, float* d_img, int nimg,
                          int solver, void* stream) {
    if (!d_guide || !d_img) return sdr::set_error(SDR_ERR_ARG, "null argument");
    if (w <= 0 || h <= 0 || nimg <= 0 || gstride < (size_t)w)
        return sdr::set_error(SDR_ERR_ARG, "bad size/stride");
    if (!(lambda >= 0.0) || !(sigma >= 0.0) || iters < 1)
        return sdr::set_error(SDR_ERR_ARG, "FGS needs lambda >= 0, sigma_color >= 0, num_iter >= 1");
    if (solver == SDR_FGS_THOMAS && !thomas_lambdas_ok(lambda, att, iters))
        return sdr::set_error(SDR_ERR_ARG, kThomasLambdaMsg);
    if (solver != SDR_FGS_PCR && solver != SDR_FGS_THOMAS)
        return sdr::set_error(SDR_ERR_ARG, "solver must be SDR_FGS_PCR or SDR_FGS_THOMAS");
    if (solver == SDR_FGS_PCR && (w > sdr::kPcrMaxN || h > sdr::kPcrMaxN))
        return sdr::set_error(SDR_ERR_SIZE, "SDR_FGS_PCR solves lines of at most 4096 samples "
                                            "(use SDR_FGS_THOMAS for larger images)");
    hipStream_t st = (hipStream_t)stream;
    std::vector<float> lut;
    sdr::fgs_lut_host(sigma, &lut);
    // stream-ordered scratch: LUT, column-major copies, coefficients, weights
    float* dlut = nullptr;
    float* scr = nullptr;
    const size_t px = (size_t)w * h;
    // (frames of the sequential solver's padded layouts: fgs_pad4(w) * fgs_pad4(h) >= px samples)
    const size_t fp = (size_t)sdr::fgs_pad4(w) * sdr::fgs_pad4(h);
    WLS_HIP(sdr::scratch_alloc((void**)&dlut, sizeof(float) * lut.size(), st));
    // (FgsScratch: the sequential solver's two interleaved pass layouts, the weights, and 5 floats
    // a sample for each of its 2 * iters passes' coefficients; its loaders read up to
    // kFgsOverread bytes past an array)
    const size_t ncoef = solver == SDR_FGS_THOMAS ? (size_t)5 * (2 * iters) : 0;
    WLS_HIP(sdr::scratch_alloc((void**)&scr, sizeof(float) * fp * (6 + ncoef) + sdr::kFgsOverread, st));
    WLS_HIP(hipMemcpyAsync(dlut, lut.data(), sizeof(float) * lut.size(), hipMemcpyHostToDevice, st));
    const sdr::FgsScratch fs{scr, scr + 2 * fp, scr + 4 * fp, scr + 5 * fp, scr + 6 * fp};
    // images are filtered in pairs (two right-hand sides of one system per line)
    for (int i = 0; i < nimg; i += 2) {
        const int m = nimg - i >= 2 ? 2 : 1;
        (void)sdr::launch_fgs(d_guide, gstride, 0, dlut, d_img + i * px, m == 2 ? d_img + (i + 1) * px : nullptr,
                              w, h, 1, lambda, att, iters, solver, fs, st);
    }
    WLS_HIP(hipGetLastError());
    WLS_HIP(sdr::scratch_free(dlut, st));
    WLS_HIP(sdr::scratch_free(scr, st));
    // the host LUT vector dies here: wait for its upload before returning
    WLS_HIP(hipStreamSynchronize(st));
    return SDR_OK;
}

}  // extern "C"
