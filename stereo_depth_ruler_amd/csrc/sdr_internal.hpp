// sdr_internal.hpp -- launchers shared by the kernel files and sdr_engine.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/sdr/sdr.h"
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace sdr {

// partial per-frame minima of the int16 disparity (launch_min_s16 / launch_speckle's out_min):
// [F][kMinSlots] ints, consumed by launch_reproject_s16 (wave-uniform scalar loads).  Block b
// folds into slot b % kMinSlots: 2048 apply blocks make 8 same-address atomics per slot (32
// slots: 64, which serialised to ~13 us of the apply pass)
constexpr int kMinSlots = 256;


// Device buffer that only grows (engine and WLS scratch); ensure() returns an SDR_* status.
struct Buf {
    void* p = nullptr;
    size_t n = 0;
};
int ensure(Buf& b, size_t bytes);
// Stream-ordered scratch of the one-shot device calls that do not synchronise (reprojection
// minima, speckle labels, the FGS filter's coefficients) from a memory pool the library owns, one
// a device, that keeps what it has mapped (release threshold: never; HIP's default pool returns
// freed memory at each synchronize).  The voxel grid, which synchronises, leases a grow-only
// arena instead (sdr_cloud.hip): its ~11 stream-ordered frees a call took 0.75-1.45 ms of host
// time even from this pool.
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t st);
hipError_t scratch_free(void* p, hipStream_t st);
// Records msg as the thread's sdr_last_error() and returns code.
int set_error(int code, const std::string& msg);

// Scanline directions of the path recurrence.
enum Dir : int {
    DIR_E = 0,   // -> (x ascending)        OpenCV dir 0, pass 1
    DIR_W = 1,   // <- (x descending)       OpenCV dir 4 (SGBM/3WAY), dir 0 pass 2 (HH)
    DIR_S = 2,   // top -> bottom           dir 2 pass 1 (3WAY: per stripe)
    DIR_N = 3,   // bottom -> top           dir 2 pass 2 (HH)
    DIR_SE = 4,  // (x-1,y-1) -> (x,y)      dir 1 pass 1
    DIR_SW = 5,  // (x+1,y-1) -> (x,y)      dir 3 pass 1
    DIR_NE = 6,  // (x-1,y+1) -> (x,y)      dir 1 pass 2 (HH)
    DIR_NW = 7,  // (x+1,y+1) -> (x,y)      dir 3 pass 2 (HH)
};

struct Geometry {
    int W, H;           // image size
    int D, minD;        // disparity count / minimum
    int minX1, W1;      // matched column range [minX1, minX1 + W1)
    int SW2, SH2;       // block half sizes
    int P1, P2;
    // paired matchers (the class path's left and right matcher in one launch): frames >= split
    // belong to a second matcher whose parameters differ only in minDisparity (same W1), with the
    // left and right images swapped (right_matcher->compute(R, L)); split > frames: unpaired
    int split;
    int minDb, minX1b;  // the second matcher's minD / minX1
};

// the geometry of frame f (the paired matcher's minD / minX1 for frames >= split)
__host__ __device__ inline Geometry frame_geom(const Geometry& g, int f) {
    Geometry r = g;
    if (f >= g.split) {
        r.minD = g.minDb;
        r.minX1 = g.minX1b;
    }
    return r;
}

// ---- prefilter / cost volume (sdr_cost.hip) ----
struct Planes {
    // per channel c of the input (cn = 1 gray, 3 colour) one operand set:
    uint32_t* L;        // [F][H][W][3cn] 16-bit halves: {sob | sob_lo<<16} {sob_hi | raw<<16} {raw_lo | raw_hi<<16}
    uint64_t* R;        // [F][3cn][H][W] int16 pairs (q(x) | q(x-1) << 16): {sob,sob_lo} {sob_hi,raw} {raw_lo,raw_hi}
    size_t fstrideL, fstrideR;  // elements per frame
    int cn;
};

// MODE_SGBM_3WAY stripe-start rows (A.7): the first SH2 cost rows of stripe s > 0 with the box
// clamped at the stripe's own start row s0, into their own buffer; computed as extra row bands
// of the main k_cost launch (one launch per frame batch)
constexpr int kMaxCostAux = 16;
struct CostAux {
    int16_t* out;  // [F][rows][W1][D], frames out_fstride apart
    int row0, rows, s0, ylim;
};

struct CostArgs {
    Planes pl;
    int16_t* out;            // cost rows
    size_t out_fstride;      // elements per frame
    int out_row0;            // row index of out's first row
    int row_begin, row_end;  // output rows [row_begin, row_end)
    int s0;                  // chain/box start row (box clamp)
    int ylim;                // rows > ylim repeat row ylim (running sum stops updating)
    int hh_bottom;           // MODE_HH: rows y>0 with y+SH2>=H keep the initial P2
    int TY;                  // tile height (output rows)
    int16_t* sink;           // cost_sink_bytes() of scratch: the stores of warm-up rows land here
    int naux;                // stripe-start bands after the main ones (grid.y = bands + naux)
    size_t aux_fstride;      // elements per frame of every aux buffer
    CostAux aux[kMaxCostAux];
};
size_t cost_sink_bytes(const Geometry& g);


// ---- path aggregation (sdr_paths.hip) ----
constexpr int kMaxPathDirs = 24;
constexpr int kMaxPaths = 8;

struct PathDir {
    int dir;
    int nchains;
    int ybeg, yend, write_from;  // DIR_S chain rows (3WAY stripes); others: 0, H, 0
    int aux_row0, aux_rows;      // DIR_S chains read stripe-local cost rows for their first rows
    const int16_t* Caux;         // [F][aux_rows][W1][D] or null
    int16_t* out;                // this direction's slot of the L records: L + dir_index * D
};

// The path costs of the P-1 directions k_paths writes are stored pixel-interleaved,
// L[F][H][W1][P-1][D]: the fused WTA pass then reads one contiguous (P-1)*D record per pixel
// instead of P-1 streams a whole volume apart.
// MODE_SGBM_3WAY: a stripe whose rows all keep their window clamped at the stripe start (the short
// last stripes, where H-1-SH2 < s0 + SH2: every row's window is frozen above s0 + SH2) has cost
// rows that differ from C on its output rows too; OpenCV runs that stripe's horizontal passes on
// its own rows, so the E/W chains of rows [lo, hi) read stripe row y - s0 of aux instead of C
struct RowRedirect {
    int lo, hi, s0;
    const int16_t* aux;  // [F][rows][W1][D], frames PathLaunch::aux_fstride apart
};

struct PathLaunch {
    const int16_t* C;
    size_t cs_fstride;   // elements per frame of C
    size_t l_fstride;    // elements per frame of L
    int l_pix;           // elements per pixel record of L ((P-1) * D)
    size_t aux_fstride;
    int ndirs;
    int prefix[kMaxPathDirs + 1];  // chain prefix sums
    PathDir d[kMaxPathDirs];
    int nredir;
    RowRedirect redir[kMaxCostAux];
};

// Row-synchronous sweeps of batched MODE_HH (sdr_sweep.hip, k_sweep16): the upward directions N,
// NE and NW (up = 1) into one record, or the downward S, SE and SW (up = 0) summed with the E, W
// and up records into S and reduced by the WTA (A.8) in the same step.  A workgroup walks a column
// tile of a frame row by row, one pixel per 16-lane row of a wave; halo waves recompute the
// diagonals' tile-edge columns and reload them from the neighbour tiles through a global ring.
constexpr int kSweepOwn = 10;                     // waves holding the tile's own columns
constexpr int kSweepWaves = kSweepOwn + 2;        // + one halo wave on each side
struct SweepArgs {
    const int16_t* C;
    size_t cs_fstride;     // elements per frame of C
    int16_t* rec;          // up pass: its record slot (L records + slot * D)
    size_t l_fstride;      // elements per frame of the records
    int l_pix;             // elements per pixel record
    uint32_t* edge;        // [nslots][ntiles][2 sides][2 parities][entry_words] the tile edges' path costs
    int* flags;            // [nslots][ntiles][2 sides][npub] rows published (zero before the launch)
    int* err;              // set when a neighbour wait times out (never, with every tile resident)
    int ntiles, nslots;    // frames in flight = nslots (workgroups = nslots * ntiles, all resident)
    int up;
    int spin;              // polls before a wait gives up (kSweepSpin; lower through a debug knob)
    int xcd;               // 1: a frame's consecutive tiles on one XCD (launch_sweep sets it)
};
// the down pass's WTA (A.8): the E, W, up records it reads and the outputs k_south_wta would write
struct SweepWta {
    const int16_t* recs;   // [F][H][W1][3][D]: E, W, up
    int16_t* disp_raw;     // [F][H][W] WTA disparity (matched columns only)
    uint32_t* d2;          // [F][H][W] right-view WTA keys (SouthWtaArgs::d2), nullable
    size_t disp_fstride;
    int uniq, uniq_simd;
};
constexpr int kSweepSpin = 1 << 20;  // polls (~1 us each) before a sweep's wait gives up
// After a batch's sweeps and post-filter: when a wait of this call's sweeps timed out (*err), the
// batch's frames are wrong, so every pixel of disp [F][n] becomes `invalid`, the reprojection's
// frame minima too (mins: [F][kMinSlots], nullable), and the handle's sticky status word is set
// (sdr_sgbm_last_status reports it).  Nothing happens otherwise.
void launch_sweep_verdict(const int* err, int16_t* disp, size_t n, int F, int16_t invalid, int* mins,
                          int* sticky, hipStream_t st);
// a pass's tiling: own columns per wave, tiles per frame, frames in flight (slots; 0: the frame's
// tiles do not fit the resident grid), publishing waves per tile edge, words of one ring entry
struct SweepShape {
    int cols, ntiles, nslots, npub, entry_words;
};
SweepShape sweep_shape(const Geometry& g, int F, bool up);
void launch_sweep(const Geometry& g, const SweepArgs& a, const SweepWta& w, int F, hipStream_t st);

// top-to-bottom direction fused with the WTA (sdr_paths.hip): the other P-1 directions' L in
// sum order with the fused direction at position kSouthIdx
constexpr int kSouthIdx = 2;  // summation order E, W, S, SE, SW, N, NE, NW
// rows of slack before and after the cost volume and the path-cost buffers: the path kernels'
// prefetch runs up to this many rows (or pixels) past either end of a chain instead of being
// clamped
constexpr int kSouthPad = 64;
struct SouthWtaArgs {
    const int16_t* L;             // the P-1 other directions' records, in order, S removed
    int npaths;
    int16_t* disp_raw;   // [F][H][W] WTA disparity (written in the matched columns only)
    // [F][H][W] the right view's WTA keys (A.8's disp2 candidates), null when the LR check cannot
    // fire: each accepted pixel x (matched-range column) folds (minS << 16 | 0xffff - x) into
    // x2 = x + minX1 - bestDisp - minD by atomicMin (the smallest cost wins, ties to the largest
    // x, as OpenCV's descending loop with a strict '>'); k_prefilter fills it with kD2None
    uint32_t* d2;
    size_t disp_fstride;
    int uniq, uniq_simd;
};
void launch_south_wta(const Geometry& g, const PathLaunch& pl, const SouthWtaArgs& a, int F,
                      hipStream_t st);

// A.9, OpenCV's disp12MaxDiff check, at pixel (x, y) of a frame with geometry g: raw is the frame's
// WTA map and d2 its right-view keys (both [H][W]).  Every consumer of the LR-checked map
// computes it on the fly from these two (the median's tiles, the debug stage), so the map itself
// is never written.
constexpr uint32_t kD2None = 0xffffffffu;
__device__ __forceinline__ int lr_at(const Geometry& g, const int16_t* __restrict__ raw,
                                     const uint32_t* __restrict__ d2, int x, int y, int d12) {
    const int invalid = (g.minD - 1) * 16;
    if (x < g.minX1 || x >= g.minX1 + g.W1) return invalid;
    const size_t ro = (size_t)y * g.W;
    const int d1 = raw[ro + x];
    if (d1 == invalid) return d1;
    const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
    const int _x = x - _d, x_ = x - d_;
    if (_x < 0 || _x >= g.W || x_ < 0 || x_ >= g.W) return d1;
    const uint32_t ka = d2[ro + _x], kb = d2[ro + x_];
    const int a2 = ka == kD2None ? invalid : (0xffff - (int)(ka & 0xffff)) + g.minX1 - _x;
    const int b2 = kb == kD2None ? invalid : (0xffff - (int)(kb & 0xffff)) + g.minX1 - x_;
    const bool bad = a2 >= g.minD && abs(a2 - _d) > d12 && b2 >= g.minD && abs(b2 - d_) > d12;
    return bad ? invalid : d1;
}
// the LR-checked map of F frames (frames fstride apart), materialised (debug stage only)
void launch_lr_apply(const Geometry& g, const int16_t* raw, const uint32_t* d2, int16_t* out,
                     size_t fstride, int disp12MaxDiff, int F, hipStream_t st);
// the median's source: A.9 of (raw, d2) per frame (frames fstride apart)
struct LrSrc {
    Geometry g;
    const int16_t* raw;
    const uint32_t* d2;
    size_t fstride;
    int d12;
};

void launch_fill_s16(int16_t* p, int16_t v, size_t n, hipStream_t st);
// d2fill (nullable): [F][H][W] right-view keys set to kD2None on the way
void launch_prefilter(const uint8_t* L, const uint8_t* R, size_t stride, size_t fstride, int W,
                      int H, int F, int ftzero, const Planes& pl, hipStream_t st, int split = 1 << 30,
                      uint32_t* d2fill = nullptr);
bool cost_supported(const Geometry& g);
void launch_cost(const Geometry& g, const CostArgs& a, int F, hipStream_t st);
// blockSize > 11 (SH2 > 5) or D > 256 (sdr_cost_generic.hip): two passes through a scratch volume h1 of
// cost_generic_scratch_bytes (the L-record buffer, idle until the path kernels)
size_t cost_generic_scratch_bytes(const Geometry& g, int F);
void launch_cost_generic(const Geometry& g, const CostArgs& a, int F, uint32_t* h1, hipStream_t st);
void launch_cost_cn3(const Geometry& g, const CostArgs& a, int F, hipStream_t st);  // pl.cn == 3
void launch_paths(const Geometry& g, const PathLaunch& pl, int F, hipStream_t st);
void launch_median3(const int16_t* src, int16_t* dst, int W, int H, int F, hipStream_t st);
// median of the LR-checked map (computed per tile from the WTA map and the right-view keys)
void launch_median3_lr(const LrSrc& lr, int16_t* dst, int F, hipStream_t st);
// median of the WTA map with columns outside [c0, c1) read as fill (LR check skipped)
void launch_median3_cols(const int16_t* src, int16_t* dst, const Geometry& g, int F, hipStream_t st);
void launch_mask_cols(const int16_t* src, int16_t* dst, const Geometry& g, int F, hipStream_t st);
// src may equal dst; out_min (nullable) receives min over each output frame.  lr (nullable): src
// is instead the 3x3 median of the LR-checked map, computed by the first pass (which also
// computes the LR check) and written to median_out (= src) -- A.9 and A.10 fused into the labelling
void launch_speckle(const int16_t* src, int16_t* dst, int W, int H, int F, int newVal, int maxSize,
                    int maxDiff, int* labels, int* sizes, int* out_min, hipStream_t st,
                    const LrSrc* lr = nullptr, int16_t* median_out = nullptr);
void launch_min_s16(const int16_t* img, size_t n_per_frame, size_t fstride, int F, int* out_min,
                    hipStream_t st);
void launch_reproject_s16(const int16_t* disp, int W, int H, size_t dstride, size_t dfstride,
                          const double* Q, int handle_missing, const int* mins, float* xyz,
                          size_t xyz_stride, size_t xyz_fstride, int F, hipStream_t st);
void launch_reproject_f32(const float* disp, int W, int H, size_t dstride, size_t dfstride,
                          const double* Q, int handle_missing, int* minbits_scratch, float* xyz,
                          size_t xyz_stride, size_t xyz_fstride, int F, hipStream_t st);
void launch_disp16_to_f32(const int16_t* d, float* o, size_t n, hipStream_t st);
void launch_bgr2gray(const uint8_t* bgr, int W, int H, size_t bstride, uint8_t* gray,
                     size_t gstride, int F, hipStream_t st);
void launch_area_half(const uint8_t* src, int W, int H, size_t stride, uint8_t* dst,
                      size_t dstride, int F, hipStream_t st);
int selftest_wave_ops(int* failures);
int stream_probe(size_t bytes, int iters, double* gbs);
int stream_probe_ex(size_t bytes, int iters, double* out3);

// Per-kernel HIP-event timing of a matcher handle (timing level 2, sdr_sgbm_kernel_time): an
// event pair of SDR_KERNEL_* kind `kind` on the handle's stream around one launch.  Kernels another
// file launches for the handle (the class path's WLS filter) bracket themselves with a KScope.
bool ktimer_begin(sdr_sgbm* h, int kind);  // false: timing is off (and no end follows)
void ktimer_end(sdr_sgbm* h);
struct KScope {
    sdr_sgbm* h;
    KScope(sdr_sgbm* h_, int kind) : h(h_ && ktimer_begin(h_, kind) ? h_ : nullptr) {}
    ~KScope() {
        if (h) ktimer_end(h);
    }
};

// DisparityWLSFilter::filter on device (sdr_wls.hip) with the class path's fused epilogue:
// fout (nullable) = out / 16, xyz (nullable, needs fout and Q) = reprojectImageTo3D(fout, Q);
// timer (nullable): the matcher handle whose per-kernel timing records the filter's launches
int wls_filter_enqueue(sdr_wls* h, const int16_t* dl, const int16_t* dr, const uint8_t* guide, int W,
                       int H, size_t gstride, size_t gfstride, int F, int16_t* out, float* conf,
                       float* fout, const double* Q, float* xyz, sdr_sgbm* timer = nullptr);

}  // namespace sdr
