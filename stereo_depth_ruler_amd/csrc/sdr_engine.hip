// sdr_engine.hip -- engine handle, scheduling of the stage kernels and the C ABI (include/sdr/sdr.h).
//
// One handle = one HIP stream + device scratch sized for the largest (W, H, D, frames) seen.
// compute_device() enqueues the whole hot path of cv::StereoSGBM::compute on the stream:
//   prefilter -> cost volume (+ 3WAY stripe-start rows) -> path kernels (first writes S, middle
//   ones accumulate, last one fuses WTA/uniqueness/subpixel) -> disp2 + LR check -> median3
//   -> speckle CCL [-> min -> reprojectImageTo3D]
// No host synchronisation, allocation or copy happens inside the enqueue once scratch is sized,
// so the sequence can be captured into a hipGraph by the caller.
#include "../../include/sdr/sdr.h"
#include "sdr_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define SDR_HIP(call)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(SDR_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Eff {
    sdr::Geometry g;
    int mode, uniq, uniq_simd, disp12MaxDiff, ftzero, nstripes, invalid;
    int speckle_ws, speckle_diff, blockSize;
};

// OpenCV's parameter defaulting (stereosgbm.cpp computeDisparitySGBM / SGBM3WayMainLoop ctor).
int make_eff(const sdr_sgbm_params& p, int W, int H, Eff* e) {
    if (p.numDisparities <= 0 || p.numDisparities % 16 != 0)
        return fail(SDR_ERR_NUMDISP, "numDisparities must be positive and divisible by 16");
    if (p.numDisparities > 512) return fail(SDR_ERR_LIMIT, "numDisparities > 512 is not supported");
    if (p.mode != SDR_MODE_SGBM && p.mode != SDR_MODE_HH && p.mode != SDR_MODE_SGBM_3WAY &&
        p.mode != SDR_MODE_HH4)
        return fail(SDR_ERR_MODE, "unknown mode");
    sdr::Geometry& g = e->g;
    g.W = W;
    g.H = H;
    g.D = p.numDisparities;
    g.minD = p.minDisparity;
    int maxD = g.minD + g.D;
    g.minX1 = std::max(maxD, 0);
    g.W1 = W + std::min(g.minD, 0) - g.minX1;
    g.split = 1 << 30;  // unpaired (see sdr::Geometry)
    g.minDb = g.minD;
    g.minX1b = g.minX1;
    if (p.mode == SDR_MODE_SGBM_3WAY) {
        g.SW2 = g.SH2 = p.blockSize > 0 ? p.blockSize / 2 : 1;
    } else {
        int bs = p.blockSize > 0 ? p.blockSize : 5;
        g.SW2 = g.SH2 = bs / 2;
    }
    g.P1 = p.P1 > 0 ? p.P1 : 2;
    g.P2 = std::max(p.P2 > 0 ? p.P2 : 5, g.P1 + 1);
    e->mode = p.mode;
    e->uniq = p.uniquenessRatio >= 0 ? p.uniquenessRatio : 10;
    if (e->uniq >= 100) return fail(SDR_ERR_ARG, "uniquenessRatio must be < 100");
    e->disp12MaxDiff = p.disp12MaxDiff > 0 ? p.disp12MaxDiff : 1;
    e->ftzero = std::max(p.preFilterCap, 15) | 1;  // any size: the clip table wraps mod 256 (k_prefilter)
    e->nstripes = p.nstripes > 0 ? p.nstripes : 4;
    e->uniq_simd = p.uniq_rule == SDR_UNIQ_SIMD ? 1
                 : p.uniq_rule == SDR_UNIQ_SCALAR ? 0
                 : (p.mode == SDR_MODE_SGBM_3WAY ? 1 : 0);
    e->invalid = (g.minD - 1) * 16;
    e->speckle_ws = p.speckleWindowSize;
    e->speckle_diff = 16 * p.speckleRange;
    e->blockSize = p.blockSize;
    // The int16 domain of OpenCV's own arithmetic: C = P2 + block cost and delta = minLp + P2
    // (minLp <= C) must fit a short.  Past it OpenCV's SIMD build wraps (short)delta0 and
    // saturates C while its scalar build computes them in int, so the reference's output is not
    // defined by the algorithm alone; the engine refuses instead of picking one of the two.
    // the largest pixel cost: BT of the prefiltered channel (values in [0, min(2*ftzero, 255)],
    // the uchar clip table) + BT of the raw one >> 2
    const long bmax = (long)(std::min(2 * e->ftzero, 255) + 63) * (2 * g.SW2 + 1) * (2 * g.SH2 + 1);
    if (2L * g.P2 + bmax > 32767)
        return fail(SDR_ERR_LIMIT, "2*P2 + (2*preFilterCap+63)*blockSize^2 exceeds the int16 cost "
                                   "range (OpenCV's SIMD and scalar builds disagree there)");
    return SDR_OK;
}

using sdr::Buf;
using sdr::ensure;

// Frame-size limits of a matched frame (W1 > 0); host-only, shared by the enqueue and
// sdr_sgbm_scratch_bytes.
int check_frame(const Eff& e) {
    const sdr::Geometry& g = e.g;
    if (g.W1 <= 0) return SDR_OK;  // nothing matched: the output is all INVALID
    if (g.W1 <= g.SW2) return fail(SDR_ERR_SIZE, "image too narrow for numDisparities/blockSize");
    if (g.W > 8192) return fail(SDR_ERR_SIZE, "width > 8192 is not supported");
    // k_paths addresses a whole chain through one buffer resource and a 32-bit SGPR offset that
    // stays below 2^31 (num_records): the longest chain span, slack rows included, must fit
    if ((size_t)(g.H + 2 * sdr::kSouthPad) * (size_t)(g.W1 + 1) * g.D * 2 > (size_t)INT32_MAX)
        return fail(SDR_ERR_SIZE, "frame too large: a path chain spans more than 2 GiB of cost volume");
    // k_cost addresses a frame's right-image planes (3 x 8 B per pixel) the same way
    if ((size_t)g.H * g.W * 24 > (size_t)INT32_MAX)
        return fail(SDR_ERR_SIZE, "frame too large: the right image's cost planes span more than 2 GiB");
    if (!sdr::cost_supported(g)) return fail(SDR_ERR_ARG, "unsupported block shape");
    return SDR_OK;
}

// Channel count of the input pair (OpenCV: CV_8UC1 or CV_8UC3; calcPixelCostBT's cn == 3 branch
// sums each channel's Sobel and raw costs, so the int16 domain bound grows with it).
int check_channels(const Eff& e, int cn) {
    if (cn != 1 && cn != 3) return fail(SDR_ERR_TYPE, "images must have 1 or 3 channels");
    if (cn == 1) return SDR_OK;
    const sdr::Geometry& g = e.g;
    const long bmax = (long)cn * (std::min(2 * e.ftzero, 255) + 63) * (2 * g.SW2 + 1) * (2 * g.SH2 + 1);
    if (2L * g.P2 + bmax > 32767)
        return fail(SDR_ERR_LIMIT, "2*P2 + 3*(2*preFilterCap+63)*blockSize^2 exceeds the int16 cost "
                                   "range (OpenCV's SIMD and scalar builds disagree there)");
    if ((size_t)g.H * g.W * 24 * cn > (size_t)INT32_MAX)
        return fail(SDR_ERR_SIZE, "frame too large: the right image's cost planes span more than 2 GiB");
    return SDR_OK;
}

struct Stripe {
    int s0, end, out0, aux_rows, ylim;
};

void stripes_of(const Eff& e, std::vector<Stripe>* out) {
    out->clear();
    const int H = e.g.H;
    const int n = e.nstripes;
    const int sz = (int)std::ceil(H / (double)n);
    const int overlap = (e.blockSize / 2 + 1) + (int)std::ceil(0.1 * sz);
    for (int s = 0; s < n; s++) {
        Stripe st;
        st.out0 = s * sz;
        if (st.out0 >= H) break;
        st.s0 = std::max(std::min(s * sz - overlap, H), 0);
        st.end = std::min((s + 1) * sz, H);
        st.ylim = std::max(H - 1 - e.g.SH2, st.s0);
        if (st.s0 == 0) st.aux_rows = 0;
        else if (st.ylim >= st.s0 + e.g.SH2) st.aux_rows = e.g.SH2;
        else st.aux_rows = st.end - st.s0;
        out->push_back(st);
    }
}

}  // namespace

int sdr::set_error(int code, const std::string& msg) { return fail(code, msg); }

int sdr::ensure(Buf& b, size_t bytes) {
    if (b.n >= bytes && b.p) return SDR_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    if (bytes == 0) return SDR_OK;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        b.p = nullptr;
        const bool cap = e == hipErrorStreamCaptureUnsupported || e == hipErrorStreamCaptureInvalidated;
        return fail(SDR_ERR_NOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e) +
                                       (cap ? " (scratch grows inside a graph capture: make one call of "
                                              "this shape before capturing)" : ""));
    }
    b.n = bytes;
    return SDR_OK;
}

hipError_t sdr::scratch_alloc(void** p, size_t bytes, hipStream_t st) {
    static std::mutex mu;
    static std::map<int, hipMemPool_t> pools;
    int dev = 0;
    hipError_t e = st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    hipMemPool_t pool = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = pools.find(dev);
        if (it == pools.end()) {
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            e = hipMemPoolCreate(&pool, &props);
            if (e != hipSuccess) return e;
            uint64_t keep = UINT64_MAX;
            e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
            if (e != hipSuccess) {
                (void)hipMemPoolDestroy(pool);
                return e;
            }
            pools[dev] = pool;  // lives as long as the process
        } else {
            pool = it->second;
        }
    }
    return hipMallocFromPoolAsync(p, bytes, pool, st);
}

hipError_t sdr::scratch_free(void* p, hipStream_t st) { return hipFreeAsync(p, st); }

namespace {
// Page-locked staging for the host-pointer entry points, kept by its owner across calls (no
// allocation per call).  Copies go through it in row chunks of about kXferChunk bytes: on the way
// in, the CPU copy of chunk i+1 overlaps the DMA of chunk i; on the way out, every chunk's DMA is
// queued behind the compute with an event, and the CPU copies chunk i out while chunk i+1 is
// still on the link.
constexpr size_t kXferChunk = (size_t)1 << 20;  // (256 KB and 4-16 MB chunks measured slower)
// page-locked blocks handed out by sdr_host_alloc: base -> size
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;
// [p, p + bytes) lies inside one sdr_host_alloc block
static bool is_pinned(const void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pinned.upper_bound((uintptr_t)p);
    if (it == g_pinned.begin()) return false;
    --it;
    return (uintptr_t)p + bytes <= it->first + it->second;
}
// 2-D copy, as one linear copy when both sides are dense
static hipError_t copy2d(void* dst, size_t dp, const void* src, size_t sp, size_t rb, int rows,
                         hipMemcpyKind kind, hipStream_t st) {
    if (dp == rb && sp == rb) return hipMemcpyAsync(dst, src, rb * rows, kind, st);
    return hipMemcpy2DAsync(dst, dp, src, sp, rb, rows, kind, st);
}
struct HostXfer {
    char* pin = nullptr;
    size_t cap = 0, used = 0;
    std::vector<hipEvent_t> ev;
    size_t nev = 0;
    struct Out {
        char* dst;
        size_t dpitch, rowbytes;
        const char* src;  // in pin
        int rows;
        size_t ev;        // event index
    };
    std::vector<Out> outs;

    // start a call needing `bytes` of staging
    int begin(size_t bytes) {
        used = 0;
        nev = 0;
        outs.clear();
        if (bytes <= cap) return SDR_OK;
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        cap = 0;
        if (hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault) != hipSuccess) {
            pin = nullptr;
            return fail(SDR_ERR_NOMEM, "hipHostMalloc failed");
        }
        cap = bytes;
        return SDR_OK;
    }
    char* take(size_t bytes) {
        char* p = pin + used;
        used += (bytes + 255) & ~(size_t)255;
        return p;
    }
    int event(size_t* idx) {
        if (nev == ev.size()) {
            hipEvent_t e = nullptr;
            SDR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ev.push_back(e);
        }
        *idx = nev++;
        return SDR_OK;
    }
    // host rows (src, spitch) -> device rows (dst, dpitch), enqueued on st
    int upload(void* dst, size_t dpitch, const void* src, size_t spitch, size_t rowbytes, int rows,
               hipStream_t st) {
        if (is_pinned(src, spitch * (rows - 1) + rowbytes)) {
            SDR_HIP(copy2d(dst, dpitch, src, spitch, rowbytes, rows, hipMemcpyHostToDevice, st));
            return SDR_OK;
        }
        char* stage = take(rowbytes * rows);
        const int step = (int)std::max<size_t>(1, kXferChunk / rowbytes);
        for (int r0 = 0; r0 < rows; r0 += step) {
            const int n = std::min(step, rows - r0);
            char* sp = stage + (size_t)r0 * rowbytes;
            const char* hp = (const char*)src + (size_t)r0 * spitch;
            if (spitch == rowbytes) std::memcpy(sp, hp, rowbytes * n);
            else
                for (int r = 0; r < n; r++) std::memcpy(sp + r * rowbytes, hp + r * spitch, rowbytes);
            SDR_HIP(copy2d((char*)dst + (size_t)r0 * dpitch, dpitch, sp, rowbytes, rowbytes, n,
                           hipMemcpyHostToDevice, st));
        }
        return SDR_OK;
    }
    // device rows (src, spitch) -> host rows (dst, dpitch): DMA chunks queued on st now, the
    // host copies done by drain()
    int download(void* dst, size_t dpitch, const void* src, size_t spitch, size_t rowbytes, int rows,
                 hipStream_t st) {
        if (is_pinned(dst, dpitch * (rows - 1) + rowbytes)) {
            SDR_HIP(copy2d(dst, dpitch, src, spitch, rowbytes, rows, hipMemcpyDeviceToHost, st));
            size_t e = 0;
            int rc = event(&e);
            if (rc) return rc;
            SDR_HIP(hipEventRecord(ev[e], st));
            outs.push_back({nullptr, 0, 0, nullptr, 0, e});  // nothing to copy: wait only
            return SDR_OK;
        }
        char* stage = take(rowbytes * rows);
        const int step = (int)std::max<size_t>(1, kXferChunk / rowbytes);
        for (int r0 = 0; r0 < rows; r0 += step) {
            const int n = std::min(step, rows - r0);
            char* sp = stage + (size_t)r0 * rowbytes;
            SDR_HIP(copy2d(sp, rowbytes, (const char*)src + (size_t)r0 * spitch, spitch, rowbytes, n,
                           hipMemcpyDeviceToHost, st));
            size_t e = 0;
            int rc = event(&e);
            if (rc) return rc;
            SDR_HIP(hipEventRecord(ev[e], st));
            outs.push_back({(char*)dst + (size_t)r0 * dpitch, dpitch, rowbytes, sp, n, e});
        }
        return SDR_OK;
    }
    int drain() {
        for (const Out& o : outs) {
            SDR_HIP(hipEventSynchronize(ev[o.ev]));
            if (!o.dst) continue;
            if (o.dpitch == o.rowbytes) std::memcpy(o.dst, o.src, o.rowbytes * o.rows);
            else
                for (int r = 0; r < o.rows; r++) std::memcpy(o.dst + r * o.dpitch, o.src + r * o.rowbytes, o.rowbytes);
        }
        outs.clear();
        return SDR_OK;
    }
    void release() {
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        cap = 0;
    }
};
size_t stage_bytes(size_t n) { return (n + 255) & ~(size_t)255; }
}  // namespace

struct sdr_sgbm {
    sdr_sgbm_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    Buf planesL, planesR, sink, C, Lr, Caux, draw, dlr, dfin, labels, sizes, mins, hin, hxyz, keys2;
    // MODE_HH row sweeps: [2 passes][slots][tiles][2] counters, the call's error word, the edge
    // rings.  status: the handle's sticky status word on the device (set by a batch whose sweep
    // wait timed out, never cleared by a call; sdr_sgbm_last_status reports and clears it),
    // status_host: its page-locked copy, refreshed after every sweep batch
    Buf sweep, status;
    int* status_host = nullptr;
    int sweep_spin = sdr::kSweepSpin;  // debug knob SDR_DEBUG_SWEEP_SPIN
    HostXfer hx;  // pinned staging of the host-pointer entry points
    Buf cls_bgr, cls_gray, cls_small, cls_dl, cls_wls, cls_f, cls_conf, cls_filt;
    int timing = 0;  // 0 off, 1 stage events, 2 stage + per-kernel events
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // per-kernel event pairs (timing level 2), harvested by sdr_sgbm_kernel_time
    std::vector<hipEvent_t> kev;
    std::vector<int> kkind;
    size_t kused = 0;
    size_t path_slack = 0, path_lslack = 0;  // elements of slack in front of C / Lr (last compute)
    // class path: the right matcher runs on a side stream forked from / joined to this one
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // recorded after the last kernel that touches this handle's scratch; a stream switch makes
    // the new stream wait for it, so one matcher used from two streams never overlaps itself
    hipEvent_t done = nullptr;
    bool pending = false;  // work enqueued on a persistent stream since the last switch, not yet recorded
    // the current stream outlives the handle's use of it: the handle's own stream, or a caller's
    // stream declared persistent (sdr_sgbm_set_stream_ex).  Only such a stream is touched after
    // the call that used it has returned (the lazy retire record at a switch, destroy's sync).
    bool persistent = true;
    // `done` was recorded after the handle's last call on a transient stream, relayed through the
    // handle's own stream so that it refers to no caller stream: the next stream waits on it
    bool relayed = false;
    bool needs_wait = false;  // the current stream has not waited on `done` yet (begin_call)
    // sweep timeouts reported so far (the device word counts them; its copy, status_host, is
    // refreshed after every sweep batch)
    int status_reported = 0;
    // the last compute skipped the no-op LR check (disp12MaxDiff >= D): debug stage 2 is then
    // rebuilt on request from the WTA map with this geometry
    bool lr_skipped = false;
    sdr::Geometry lr_g{};
    int lr_frames = 0, lr_d12 = 0;
    size_t aux_slack = 0;  // elements before the 3WAY stripe-start rows in Caux
};

namespace {
// Events that only order streams on this device (the handle's retire event, the sweep
// serialisation, the class path's fork / join) and the per-kernel timers: a device-scope release.
// The default event's system-scope release writes back and invalidates the caches at every record:
// on the class path's frame that was a ~5 us idle gap between the matchers and the WLS filter, and
// the kernels after it started on cold caches.  (The host-staging events of drain() keep the
// default: the host reads what they order.)
constexpr unsigned kOrderEvent = hipEventDisableTiming | hipEventReleaseToDevice;
constexpr unsigned kTimerEvent = hipEventReleaseToDevice;
// A stream being captured into a graph (hipStreamBeginCapture, torch.cuda.graph).
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}
// The handle's last enqueue, for the next stream that uses its scratch (h->done).
//  * On a persistent stream (the handle's own, or a caller's declared so: torch's pooled streams)
//    the record is lazy: only when the handle moves to another stream does its old stream get the
//    event (after everything queued there so far, the handle's work included), and the new stream
//    wait on it.  An event record is a queue barrier: recorded after every call it left a ~6 us
//    idle gap per class-path frame (rounds 4 and 5).
//  * On a transient caller stream (sdr_sgbm_set_stream; the caller may destroy it as soon as its
//    work is done) the event is recorded at the end of every call, and relayed through the
//    handle's own stream (that stream waits on it, then the event is recorded again there), so
//    neither a later switch nor destroy touches the caller's stream: HIP does not validate a
//    destroyed stream's handle, and an event whose last record was on one crashes a later wait
//    (round 5, gpurun_out/r5b/tests.log).
// Nothing is recorded into or waited on from a graph capture: the capture's replays order
// themselves.
// `done` after everything queued on `from`, re-recorded on the handle's own stream
hipError_t relay(sdr_sgbm* h, hipStream_t from) {
    hipError_t e = hipEventRecord(h->done, from);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->own_stream, h->done, 0);
    if (e == hipSuccess) e = hipEventRecord(h->done, h->own_stream);
    h->relayed = e == hipSuccess;
    return e;
}
hipError_t retire(sdr_sgbm* h) {
    if (h->persistent) {
        h->pending = true;
        return hipSuccess;
    }
    if (!h->done || capturing(h->stream)) return hipSuccess;
    return relay(h, h->stream);
}
// At the start of a call: the handle's stream waits for work the handle queued elsewhere and
// has not been ordered before it yet (the class path's unpaired right matcher, run on a side stream)
hipError_t begin_call(sdr_sgbm* h) {
    if (!h->needs_wait) return hipSuccess;
    h->needs_wait = false;
    if (capturing(h->stream)) return hipSuccess;
    return hipStreamWaitEvent(h->stream, h->done, 0);
}
int use_stream(sdr_sgbm* h, hipStream_t s, bool persistent) {
    // a stream being captured neither queries nor waits on an event recorded outside the capture
    // (both invalidate a global-mode capture); torch.cuda.graph synchronises before it captures,
    // and a caller capturing by hand orders the handle's earlier work before the capture itself
    persistent = persistent || s == h->own_stream;
    if (s == h->stream) {
        // the same stream, now declared transient: record what the persistent form left pending
        // (the stream exists: this call names it)
        hipError_t e = hipSuccess;
        if (h->persistent && !persistent && h->pending) {
            h->persistent = false;
            h->pending = false;
            e = retire(h);
        }
        h->persistent = persistent;
        if (e != hipSuccess)
            return fail(SDR_ERR_DEVICE, std::string("ordering the handle's work on its stream: ") + hipGetErrorString(e));
        return SDR_OK;
    }
    hipError_t e = hipSuccess;
    bool wait = false;
    if (h->pending && h->done && !capturing(h->stream) && !capturing(s)) {
        // h->pending implies a persistent previous stream: it still exists
        e = hipEventRecord(h->done, h->stream);
        wait = true;
    } else if (h->relayed && !capturing(s)) {
        wait = true;  // recorded on the handle's own stream: no caller stream is touched
    }
    if (wait && e == hipSuccess) e = hipStreamWaitEvent(s, h->done, 0);
    // the handle moves to s even when the ordering failed: the error is reported once and the
    // handle stays usable on s
    h->pending = false;
    h->relayed = false;
    h->needs_wait = false;
    h->stream = s;
    h->persistent = persistent;
    if (e != hipSuccess)
        return fail(SDR_ERR_DEVICE, std::string("ordering the handle's previous stream before the new one: ") +
                                        hipGetErrorString(e));
    return SDR_OK;
}
}  // namespace

bool sdr::ktimer_begin(sdr_sgbm* h, int kind) {
    if (h->timing < 2) return false;
    if (h->kused * 2 + 2 > h->kev.size()) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreateWithFlags(&a, kTimerEvent) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&b, kTimerEvent) != hipSuccess) {
            (void)hipEventDestroy(a);
            return false;
        }
        h->kev.push_back(a);
        h->kev.push_back(b);
        h->kkind.push_back(kind);
    }
    h->kkind[h->kused] = kind;
    (void)hipEventRecord(h->kev[2 * h->kused], h->stream);
    return true;
}

void sdr::ktimer_end(sdr_sgbm* h) {
    (void)hipEventRecord(h->kev[2 * h->kused + 1], h->stream);
    h->kused++;
}

namespace {
// RAII event pair around one kernel launch when per-kernel timing is on.
using KTimer = sdr::KScope;
}  // namespace


static int npaths_of(int mode);
// batches from this many frames run MODE_HH's N/NE/NW and SE/SW as row sweeps (k_sweep): a sweep
// walks a frame's rows in order, so it pays one cross-tile hand-over per row per frame and only
// amortises that latency over several frames in flight
constexpr int kSweepMinFrames = 8;

// A sweep's workgroups wait on each other, so its grid must become resident as a whole: other
// kernels only delay that (they finish without waiting on anything), but two sweeps in flight at
// once could each hold part of the chip while waiting for the rest.  Sweeps of every handle and
// stream of a device are therefore chained in submission order through one event per device.
static std::mutex g_sweep_mu;
static std::map<int, hipEvent_t> g_sweep_last;

static size_t scratch_bytes(const Eff& e, int F, std::vector<Stripe>* st, int cn) {
    const sdr::Geometry& g = e.g;
    const size_t cells = (size_t)g.H * std::max(g.W1, 0) * g.D;
    size_t aux = 0;
    if (e.mode == SDR_MODE_SGBM_3WAY) {
        stripes_of(e, st);
        int amax = 0;
        for (auto& s : *st) amax = std::max(amax, s.aux_rows);
        aux = (size_t)st->size() * amax * std::max(g.W1, 0) * g.D * 2;
    }
    const size_t px = (size_t)g.W * g.H;
    return (size_t)F * (3 * px * 4 * cn + 3 * px * 8 * cn + cells * 2 * npaths_of(e.mode) + aux + px * 2 * 3 + px * 4 +
                        px * 4 * 2);
}

static int npaths_of(int mode) {
    return mode == SDR_MODE_HH ? 8 : mode == SDR_MODE_SGBM ? 5 : mode == SDR_MODE_HH4 ? 4 : 3;
}

// Enqueues the full compute for F frames whose inputs are already on the device.
//   prefilter -> cost volume (+ 3WAY stripe-start rows) -> the P-1 directions other than
//   top-to-bottom in one launch, each into its own L buffer -> top-to-bottom chains fused with
//   WTA/uniqueness/subpixel/disp2 -> LR check -> median3 -> speckle
// Per cell this moves 2 (C write) + 4(P-1) (paths: C read + L write) + 2 + 2(P-1) (fused pass:
// C read + the other L reads) = 6P - 2 bytes, 4 fewer than the canonical 2 + 6P of SURVEY.md 8(d).
//   out (nullable): dense [F][H][W] int16 destination for the final map (else internal buffer)
//   out_min (nullable): per-frame minimum of the final map (reprojectImageTo3D handleMissing)
// Paired matchers (the class path): frames [0, F/2) run h's parameters on (L, R), frames
// [F/2, F) the right matcher's `pair` parameters on (R, L) -- right_matcher->compute(R, L) -- in
// the same launches.  Only when the two differ in minDisparity alone and match the same number
// of columns (createRightMatcher + the WLS filter's mutations give exactly that).
static bool can_pair(const Eff& a, const Eff& b) {
    return a.g.W1 == b.g.W1 && a.g.W1 > 0 && a.g.D == b.g.D && a.g.SW2 == b.g.SW2 && a.g.P1 == b.g.P1 &&
           a.g.P2 == b.g.P2 && a.mode == b.mode && a.uniq == b.uniq && a.uniq_simd == b.uniq_simd &&
           a.disp12MaxDiff == b.disp12MaxDiff && a.ftzero == b.ftzero && a.nstripes == b.nstripes &&
           a.speckle_ws == 0 && b.speckle_ws == 0 && a.blockSize == b.blockSize;
}

static int enqueue_compute(sdr_sgbm* h, const uint8_t* L, const uint8_t* R, int W, int H,
                           size_t stride, size_t fstride, int F, int16_t* out, int* out_min,
                           int16_t** final_disp, int cn = 1, const sdr_sgbm_params* pair = nullptr) {
    // a batch of an earlier call whose sweep wait gave up (its frames were written as INVALID):
    // reported here, by the next call, if no sdr_sgbm_last_status has reported it yet.  The
    // host copy is refreshed asynchronously after every sweep batch, so this check never waits
    // (a timeout still in flight is reported by the call after)
    // (a count of timed-out batches: each is reported once, whatever copies are still in flight)
    if (h->status_host && __atomic_load_n(h->status_host, __ATOMIC_ACQUIRE) != h->status_reported) {
        h->status_reported = __atomic_load_n(h->status_host, __ATOMIC_ACQUIRE);
        return fail(SDR_ERR_DEVICE, "an earlier MODE_HH batch's row sweep timed out waiting for a neighbouring "
                                    "tile: that batch's frames were written as INVALID (this call did not run)");
    }
    SDR_HIP(begin_call(h));
    Eff e;
    int rc = make_eff(h->p, W, H, &e);
    if (rc) return rc;
    if ((rc = check_channels(e, cn))) return rc;
    if (pair) {
        Eff eb;
        if ((rc = make_eff(*pair, W, H, &eb))) return rc;
        if (!can_pair(e, eb) || (F & 1)) return fail(SDR_ERR_ARG, "matchers cannot be paired");
        e.g.split = F / 2;
        e.g.minDb = eb.g.minD;
        e.g.minX1b = eb.g.minX1;
    }
    h->lr_skipped = false;
    const sdr::Geometry& g = e.g;
    hipStream_t st = h->stream;
    const size_t px = (size_t)W * H;
    if ((rc = ensure(h->dfin, F * px * 2))) return rc;
    int16_t* dfin = (int16_t*)h->dfin.p;
    int16_t* dst = out ? out : dfin;
    *final_disp = dst;
    if (g.W1 <= 0) {
        sdr::launch_fill_s16(dst, (int16_t)e.invalid, F * px, st);
        if (out_min) sdr::launch_min_s16(dst, px, px, F, out_min, st);
        return SDR_OK;
    }
    if ((rc = check_frame(e))) return rc;

    const size_t cells = (size_t)H * g.W1 * g.D;
    const int P = npaths_of(e.mode);
    // batched MODE_HH: N/NE/NW and S/SE/SW as two row-synchronous sweeps (when every tile of the
    // frames in flight fits the resident grid); the records are then E, W and up -- saturated sums
    // of non-negative path costs, so the grouping is exact -- and the down sweep runs the WTA
    sdr::SweepShape shp[2] = {};  // [0]: down (S, SE, SW + WTA), [1]: up (N, NE, NW)
    // (not inside a graph capture: its replays could overlap another sweep's, which the event
    // chain below orders for directly enqueued sweeps only)
    if (e.mode == SDR_MODE_HH && F >= kSweepMinFrames && g.W1 > 0 && !capturing(h->stream))
        for (int up = 0; up < 2; up++) shp[up] = sdr::sweep_shape(g, F, up != 0);
    const bool sweep = shp[0].nslots > 0 && shp[1].nslots > 0;
    const int nrec = sweep ? 3 : P - 1;  // L records per pixel
    std::vector<Stripe> stripes;
    if (e.mode == SDR_MODE_SGBM_3WAY) stripes_of(e, &stripes);
    if (stripes.size() + 2 > (size_t)sdr::kMaxPathDirs) return fail(SDR_ERR_ARG, "too many 3WAY stripes");
    int amax = 0;
    for (auto& s : stripes) amax = std::max(amax, s.aux_rows);
    const size_t aux_fstride = (size_t)stripes.size() * amax * g.W1 * g.D;

    if ((rc = ensure(h->planesL, F * 3 * px * 4 * cn))) return rc;
    if ((rc = ensure(h->planesR, F * 3 * px * 8 * cn))) return rc;
    if ((rc = ensure(h->sink, sdr::cost_sink_bytes(g)))) return rc;
    // the path kernels' loads overrun a chain's ends by up to kSouthPad rows: slack both sides
    const size_t slack = (size_t)sdr::kSouthPad * g.W1 * g.D;
    const size_t lslack = slack * nrec;
    const size_t lfs = (size_t)nrec * cells;  // L elements per frame, [H][W1][nrec][D]
    // a batch that can take the sweep sizes L for the chains' P - 1 records too, so a graph
    // capture of the same shape (chains only) allocates nothing
    const size_t lrec = e.mode == SDR_MODE_HH && F >= kSweepMinFrames ? (size_t)(P - 1) : (size_t)nrec;
    if ((rc = ensure(h->C, (F * cells + 2 * slack) * 2))) return rc;
    if ((rc = ensure(h->Lr, (F * cells + 2 * slack) * lrec * 2))) return rc;
    if ((rc = ensure(h->keys2, F * px * 4))) return rc;
    // the E/W chains redirected into it (RowRedirect) load up to a lookahead past a row's ends
    const size_t aux_slack = (size_t)sdr::kSouthPad * g.D;
    if ((rc = ensure(h->Caux, (F * aux_fstride + 2 * aux_slack) * 2))) return rc;
    if ((rc = ensure(h->draw, F * px * 2))) return rc;
    if ((rc = ensure(h->dlr, F * px * 2))) return rc;
    if (e.speckle_ws > 0) {
        if ((rc = ensure(h->labels, F * px * 4))) return rc;
        if ((rc = ensure(h->sizes, F * px * 4))) return rc;
    }

    if (h->timing) SDR_HIP(hipEventRecord(h->ev[0], st));
    h->path_slack = slack;
    h->path_lslack = lslack;
    int16_t* C = (int16_t*)h->C.p + slack;
    int16_t* Caux = (int16_t*)h->Caux.p + aux_slack;
    h->aux_slack = aux_slack;
    int16_t* Lr = (int16_t*)h->Lr.p + lslack;  // [F][H][W1][nrec][D]
    // [pass][slots][tiles][2] counters, the error word, then the edge ring (sized for either pass)
    size_t flags_n[2] = {0, 0}, edge_bytes = 0;
    for (int up = 0; up < 2; up++) {
        flags_n[up] = (size_t)shp[up].nslots * shp[up].ntiles * 2 * shp[up].npub;
        edge_bytes = std::max(edge_bytes, (size_t)shp[up].nslots * shp[up].ntiles * 4 * shp[up].entry_words * 4);
    }
    const size_t sweep_flags = (flags_n[0] + flags_n[1]) * sizeof(int);
    if (sweep) {
        if ((rc = ensure(h->sweep, sweep_flags + 256 + edge_bytes))) return rc;
        if (!h->status_host) {
            if ((rc = ensure(h->status, 256))) return rc;
            SDR_HIP(hipMemsetAsync(h->status.p, 0, 256, st));
            if (hipHostMalloc((void**)&h->status_host, sizeof(int), hipHostMallocDefault) != hipSuccess) {
                h->status_host = nullptr;
                return fail(SDR_ERR_NOMEM, "hipHostMalloc failed");
            }
            *h->status_host = 0;
        }
    }
    int16_t* draw = (int16_t*)h->draw.p;

    sdr::Planes pl;
    pl.L = (uint32_t*)h->planesL.p;
    pl.R = (uint64_t*)h->planesR.p;
    pl.fstrideL = pl.fstrideR = 3 * px * cn;
    pl.cn = cn;
    const bool speckle = e.speckle_ws > 0;
    // A.9 can only invalidate a pixel when |disp2 - d| > disp12MaxDiff; both lie in [minD, maxD),
    // so from disp12MaxDiff >= D on (ximgproc's WLS filter sets 1000000 on the class path's left
    // matcher, createRightMatcher on the right one) the check is the identity on the matched
    // columns and INVALID elsewhere: the median reads the WTA map with that column mask instead,
    // and no right-view keys are built
    h->lr_skipped = !speckle && e.disp12MaxDiff >= g.D;
    h->lr_g = g;
    h->lr_frames = F;
    h->lr_d12 = e.disp12MaxDiff;
    uint32_t* d2 = h->lr_skipped ? nullptr : (uint32_t*)h->keys2.p;
    { KTimer kt(h, SDR_KERNEL_PREFILTER); sdr::launch_prefilter(L, R, stride, fstride, W, H, F, e.ftzero, pl, st, g.split, d2); }

    sdr::CostArgs ca{};
    ca.pl = pl;
    ca.out = C;
    ca.out_fstride = cells;
    ca.out_row0 = 0;
    ca.row_begin = 0;
    ca.row_end = H;
    ca.s0 = 0;
    ca.ylim = std::max(H - 1 - g.SH2, 0);
    // the full-DP cost buffers of MODE_HH and MODE_HH4 keep P2 on the rows the running sum never reaches
    ca.hh_bottom = e.mode == SDR_MODE_HH || e.mode == SDR_MODE_HH4;
    ca.TY = 0;  // sized by launch_cost for one full pass of resident blocks
    ca.sink = (int16_t*)h->sink.p;
    // the 3WAY stripe-start rows are extra row bands of the same launch
    ca.naux = 0;
    ca.aux_fstride = aux_fstride;
    for (size_t s = 0; s < stripes.size(); s++) {
        const Stripe& sp = stripes[s];
        if (!sp.aux_rows) continue;
        if (ca.naux == sdr::kMaxCostAux) return fail(SDR_ERR_ARG, "too many 3WAY stripes");
        sdr::CostAux& x = ca.aux[ca.naux++];
        x.out = Caux + s * (size_t)amax * g.W1 * g.D;
        x.row0 = sp.s0;
        x.rows = sp.aux_rows;
        x.s0 = sp.s0;
        x.ylim = sp.ylim;
    }
    {
        KTimer kt(h, SDR_KERNEL_COST);
        // blockSize 13..17 (within the int16 domain) or D > 256: the two-pass cost through the
        // idle L records
        if (g.SH2 > 5 || g.D > 256) sdr::launch_cost_generic(g, ca, F, (uint32_t*)h->Lr.p, st);
        else sdr::launch_cost(g, ca, F, st);
    }
    if (h->timing) SDR_HIP(hipEventRecord(h->ev[1], st));

    // k_paths: every direction except the top-to-bottom one, each into its own L buffer (in the
    // order E, W, [S], SE, SW, N, NE, NW that k_wta_lr's sum uses); k_south_wta: the
    // top-to-bottom chains fused with the WTA, reading the other P-1 buffers
    sdr::PathLaunch pls{}, plS{};
    pls.C = plS.C = C;
    pls.cs_fstride = plS.cs_fstride = cells;
    pls.l_fstride = plS.l_fstride = lfs;
    pls.l_pix = plS.l_pix = nrec * g.D;
    pls.aux_fstride = plS.aux_fstride = aux_fstride;
    int nbuf = 0;
    auto add_dir = [&](sdr::PathLaunch& pl, int dir, int nch, int16_t* out) {
        sdr::PathDir d{};
        d.dir = dir;
        d.nchains = nch;
        d.ybeg = 0;
        d.yend = H;
        d.write_from = 0;
        d.out = out;
        pl.d[pl.ndirs++] = d;
    };
    auto buf = [&]() { return Lr + (size_t)(nbuf++) * g.D; };
    const int nE = H, nS = g.W1, nD = g.W1 + H - 1;
    // longest chains first: the E/W rows (W1 steps) are dispatched before the shorter ones
    add_dir(pls, sdr::DIR_E, nE, buf());
    add_dir(pls, sdr::DIR_W, nE, buf());
    if (e.mode == SDR_MODE_SGBM_3WAY) {
        for (size_t s = 0; s < stripes.size(); s++) {
            const Stripe& sp = stripes[s];
            add_dir(plS, sdr::DIR_S, nS, nullptr);
            sdr::PathDir& d = plS.d[plS.ndirs - 1];
            d.ybeg = sp.s0;
            d.yend = sp.end;
            d.write_from = sp.out0;
            if (sp.aux_rows) {
                d.Caux = Caux + s * (size_t)amax * g.W1 * g.D;
                d.aux_row0 = sp.s0;
                d.aux_rows = sp.aux_rows;
            }
        }
    } else if (e.mode == SDR_MODE_HH4) {
        // computeDisparitySGBM_HH4: the two vertical and the two horizontal directions
        add_dir(plS, sdr::DIR_S, nS, nullptr);
        add_dir(pls, sdr::DIR_N, nS, buf());
    } else if (sweep) {
        // record 2: the up sweep; S, SE and SW run in the down sweep with the WTA
    } else {
        add_dir(plS, sdr::DIR_S, nS, nullptr);
        if (e.mode == SDR_MODE_HH) add_dir(pls, sdr::DIR_N, nS, buf());
        add_dir(pls, sdr::DIR_SE, nD, buf());
        add_dir(pls, sdr::DIR_SW, nD, buf());
        if (e.mode == SDR_MODE_HH) {
            add_dir(pls, sdr::DIR_NE, nD, buf());
            add_dir(pls, sdr::DIR_NW, nD, buf());
        }
    }
    for (size_t s = 0; s < stripes.size(); s++) {
        const Stripe& sp = stripes[s];
        // every row of the stripe comes from its own buffer: its output rows differ from C too
        if (sp.aux_rows == 0 || sp.aux_rows != sp.end - sp.s0 || sp.out0 >= sp.end) continue;
        if (pls.nredir == sdr::kMaxCostAux) return fail(SDR_ERR_ARG, "too many 3WAY stripes");
        sdr::RowRedirect& r = pls.redir[pls.nredir++];
        r.lo = sp.out0;
        r.hi = sp.end;
        r.s0 = sp.s0;
        r.aux = Caux + s * (size_t)amax * g.W1 * g.D;
    }
    for (sdr::PathLaunch* pl : {&pls, &plS}) {
        pl->prefix[0] = 0;
        for (int i = 0; i < pl->ndirs; i++) pl->prefix[i + 1] = pl->prefix[i] + pl->d[i].nchains;
    }
    { KTimer kt(h, SDR_KERNEL_PATHS); sdr::launch_paths(g, pls, F, st); }
    if (sweep) {
        char* sb = (char*)h->sweep.p;
        SDR_HIP(hipMemsetAsync(sb, 0, sweep_flags + sizeof(int), st));
        sdr::SweepArgs sa{};
        sa.C = C;
        sa.cs_fstride = cells;
        sa.l_fstride = lfs;
        sa.l_pix = nrec * g.D;
        sa.flags = (int*)sb;
        sa.err = (int*)(sb + sweep_flags);
        sa.edge = (uint32_t*)(sb + sweep_flags + 256);
        sa.spin = h->sweep_spin;
        sdr::SweepWta sw{};
        sw.recs = Lr;
        sw.disp_raw = draw;
        sw.d2 = d2;
        sw.disp_fstride = px;
        sw.uniq = e.uniq;
        sw.uniq_simd = e.uniq_simd;
        std::lock_guard<std::mutex> lk(g_sweep_mu);
        hipEvent_t& last = g_sweep_last[h->device];
        if (last) SDR_HIP(hipStreamWaitEvent(st, last, 0));
        else SDR_HIP(hipEventCreateWithFlags(&last, kOrderEvent));
        for (int up = 1; up >= 0; up--) {
            sa.up = up;
            sa.ntiles = shp[up].ntiles;
            sa.nslots = shp[up].nslots;
            sa.rec = Lr + (size_t)2 * g.D;
            KTimer kt(h, up ? SDR_KERNEL_SWEEP : SDR_KERNEL_SWEEP_DOWN);
            sdr::launch_sweep(g, sa, sw, F, st);
            sa.flags += flags_n[up];
        }
        SDR_HIP(hipEventRecord(last, st));
    }
    if (h->timing) SDR_HIP(hipEventRecord(h->ev[2], st));

    if (!sweep) {
        sdr::SouthWtaArgs wa{};
        wa.L = Lr;
        wa.npaths = nrec + 1;
        wa.disp_raw = draw;
        wa.d2 = d2;
        wa.disp_fstride = px;
        wa.uniq = e.uniq;
        wa.uniq_simd = e.uniq_simd;
        KTimer kt(h, SDR_KERNEL_WTA_LR);
        sdr::launch_south_wta(g, plS, wa, F, st);
    }
    const sdr::LrSrc lr{g, draw, d2, px, e.disp12MaxDiff};
    if (speckle) {
        // the LR check and the median filter run inside the labelling's first pass (dfin = median
        // of the LR-checked map, computed per tile from draw and d2)
        KTimer kt(h, SDR_KERNEL_SPECKLE);
        sdr::launch_speckle(dfin, dst, W, H, F, e.invalid, e.speckle_ws, e.speckle_diff,
                            (int*)h->labels.p, (int*)h->sizes.p, out_min, st, &lr, dfin);
    } else {
        {
            KTimer kt(h, SDR_KERNEL_MEDIAN);
            if (h->lr_skipped) sdr::launch_median3_cols(draw, dst, g, F, st);
            else sdr::launch_median3_lr(lr, dst, F, st);
        }
        if (out_min) {
            KTimer kt(h, SDR_KERNEL_REPROJECT);
            sdr::launch_min_s16(dst, px, px, F, out_min, st);
        }
    }
    if (sweep) {
        // a timed-out wait made this batch's frames wrong: they become INVALID (and the handle's
        // status says so) before anything downstream reads them
        sdr::launch_sweep_verdict((const int*)((char*)h->sweep.p + sweep_flags), dst, px, F,
                                  (int16_t)e.invalid, out_min, (int*)h->status.p, st);
        SDR_HIP(hipMemcpyAsync(h->status_host, h->status.p, sizeof(int), hipMemcpyDeviceToHost, st));
    }
    if (h->timing) SDR_HIP(hipEventRecord(h->ev[3], st));
    SDR_HIP(retire(h));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

// ===========================================================================================
// C ABI
// ===========================================================================================
extern "C" {

const char* sdr_last_error(void) { return g_last_error.c_str(); }
int sdr_abi_version(void) { return SDR_ABI_VERSION; }

void sdr_sgbm_params_default(sdr_sgbm_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->numDisparities = 16;
    p->blockSize = 3;
    p->mode = SDR_MODE_SGBM;
    p->nstripes = 4;
}

void sdr_right_matcher_params(const sdr_sgbm_params* l, sdr_sgbm_params* r) {
    if (!l || !r) return;
    // ximgproc createRightMatcher: StereoSGBM::create(-(min+num)+1, num, wsize) + setters
    sdr_sgbm_params_default(r);
    r->minDisparity = -(l->minDisparity + l->numDisparities) + 1;
    r->numDisparities = l->numDisparities;
    r->blockSize = l->blockSize;
    r->uniquenessRatio = 0;
    r->P1 = l->P1;
    r->P2 = l->P2;
    r->mode = l->mode;
    r->preFilterCap = l->preFilterCap;
    r->disp12MaxDiff = 1000000;
    r->speckleWindowSize = 0;
    r->speckleRange = l->speckleRange;
    r->nstripes = l->nstripes;
    r->uniq_rule = l->uniq_rule;
}

int sdr_sgbm_create(const sdr_sgbm_params* p, int device, sdr_sgbm** out) {
    if (!p || !out) return fail(SDR_ERR_ARG, "null argument");
    *out = nullptr;
    int ndev = 0;
    SDR_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SDR_ERR_DEVICE, "invalid device index");
    SDR_HIP(hipSetDevice(device));
    sdr_sgbm* h = new sdr_sgbm();
    h->p = *p;
    h->device = device;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail(SDR_ERR_DEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    for (auto& ev : h->ev) (void)hipEventCreateWithFlags(&ev, kTimerEvent);
    (void)hipEventCreateWithFlags(&h->done, kOrderEvent);
    *out = h;
    return SDR_OK;
}

int sdr_sgbm_destroy(sdr_sgbm* h) {
    if (!h) return SDR_OK;
    (void)hipSetDevice(h->device);
    // a transient caller stream is never touched after its call: the relay put its work on own_stream
    if (h->stream && h->persistent) (void)hipStreamSynchronize(h->stream);
    if (h->own_stream && h->own_stream != h->stream) (void)hipStreamSynchronize(h->own_stream);
    if (h->status_host) (void)hipHostFree(h->status_host);
    for (Buf* b : {&h->sweep, &h->status, &h->planesL, &h->planesR, &h->sink, &h->C, &h->Lr, &h->Caux, &h->draw, &h->dlr, &h->dfin, &h->keys2,
                   &h->labels, &h->sizes, &h->mins, &h->hin, &h->hxyz, &h->cls_bgr,
                   &h->cls_gray, &h->cls_small, &h->cls_dl, &h->cls_wls, &h->cls_f,
                   &h->cls_conf, &h->cls_filt})
        if (b->p) (void)hipFree(b->p);
    h->hx.release();
    for (auto ev : h->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto ev : h->kev) (void)hipEventDestroy(ev);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->fork) (void)hipEventDestroy(h->fork);
    if (h->join) (void)hipEventDestroy(h->join);
    if (h->done) (void)hipEventDestroy(h->done);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return SDR_OK;
}

int sdr_sgbm_set_params(sdr_sgbm* h, const sdr_sgbm_params* p) {
    if (!h || !p) return fail(SDR_ERR_ARG, "null argument");
    h->p = *p;
    return SDR_OK;
}

int sdr_sgbm_get_params(const sdr_sgbm* h, sdr_sgbm_params* p) {
    if (!h || !p) return fail(SDR_ERR_ARG, "null argument");
    *p = h->p;
    return SDR_OK;
}

int sdr_sgbm_set_stream(sdr_sgbm* h, void* stream) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    (void)hipSetDevice(h->device);
    // NULL = the HIP null (legacy default) stream, which always exists
    return use_stream(h, (hipStream_t)stream, stream == nullptr);
}

int sdr_sgbm_set_stream_ex(sdr_sgbm* h, void* stream, int flags) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    if (flags & ~SDR_STREAM_PERSISTENT) return fail(SDR_ERR_ARG, "unknown stream flags");
    (void)hipSetDevice(h->device);
    return use_stream(h, (hipStream_t)stream, stream == nullptr || (flags & SDR_STREAM_PERSISTENT));
}

int sdr_sgbm_reset_stream(sdr_sgbm* h) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    (void)hipSetDevice(h->device);
    return use_stream(h, h->own_stream, true);
}

void* sdr_sgbm_get_stream(const sdr_sgbm* h) { return h ? (void*)h->stream : nullptr; }

int sdr_sgbm_enable_timing(sdr_sgbm* h, int enable) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    h->timing = enable < 0 ? 0 : enable;
    h->kused = 0;
    return SDR_OK;
}

int sdr_sgbm_last_timing(const sdr_sgbm* h, float* cost_ms, float* paths_ms, float* post_ms) {
    if (!h || !h->timing) return fail(SDR_ERR_ARG, "timing not enabled");
    SDR_HIP(hipEventSynchronize(h->ev[3]));
    float a = 0, b = 0, c = 0;
    SDR_HIP(hipEventElapsedTime(&a, h->ev[0], h->ev[1]));
    SDR_HIP(hipEventElapsedTime(&b, h->ev[1], h->ev[2]));
    SDR_HIP(hipEventElapsedTime(&c, h->ev[2], h->ev[3]));
    if (cost_ms) *cost_ms = a;
    if (paths_ms) *paths_ms = b;
    if (post_ms) *post_ms = c;
    return SDR_OK;
}

size_t sdr_sgbm_scratch_bytes(const sdr_sgbm_params* p, int width, int height, int nframes) {
    return sdr_sgbm_scratch_bytes_cn(p, width, height, 1, nframes);
}

size_t sdr_sgbm_scratch_bytes_cn(const sdr_sgbm_params* p, int width, int height, int channels,
                                 int nframes) {
    if (!p) return 0;
    Eff e;
    if (make_eff(*p, width, height, &e) || check_channels(e, channels) || check_frame(e)) return 0;
    std::vector<Stripe> st;
    return scratch_bytes(e, std::max(nframes, 1), &st, channels);
}

// Everything enqueue_compute refuses, checked before a host-pointer call stages or uploads
// anything (an error return then leaves no DMA in flight from the staging buffer).
static int precheck(const sdr_sgbm* h, int W, int H, int cn) {
    Eff e;
    int rc = make_eff(h->p, W, H, &e);
    if (rc) return rc;
    if ((rc = check_channels(e, cn))) return rc;
    return e.g.W1 > 0 ? check_frame(e) : SDR_OK;
}

static int check_dims(int W, int H, size_t stride, int F) {
    if (W <= 0 || H <= 0 || F <= 0) return fail(SDR_ERR_ARG, "non-positive size");
    if (stride < (size_t)W) return fail(SDR_ERR_ARG, "stride < width");
    return SDR_OK;
}

int sdr_sgbm_compute_device(sdr_sgbm* h, const uint8_t* dL, const uint8_t* dR, int W, int H,
                            size_t stride, size_t fstride, int F, int16_t* dDisp,
                            size_t disp_stride, size_t disp_fstride) {
    return sdr_sgbm_compute_device_cn(h, dL, dR, W, H, 1, stride, fstride, F, dDisp, disp_stride,
                                      disp_fstride);
}

int sdr_sgbm_compute_device_cn(sdr_sgbm* h, const uint8_t* dL, const uint8_t* dR, int W, int H,
                               int channels, size_t stride, size_t fstride, int F, int16_t* dDisp,
                               size_t disp_stride, size_t disp_fstride) {
    if (!h || !dL || !dR || !dDisp) return fail(SDR_ERR_ARG, "null argument");
    if (channels != 1 && channels != 3) return fail(SDR_ERR_TYPE, "images must have 1 or 3 channels");
    int rc = check_dims(W * channels, H, stride, F);
    if (rc) return rc;
    if (disp_stride < (size_t)W) return fail(SDR_ERR_ARG, "disp_stride < width");
    if (F > 1 && fstride < stride * H) return fail(SDR_ERR_ARG, "frame_stride too small");
    SDR_HIP(hipSetDevice(h->device));
    int16_t* fin = nullptr;
    const size_t px = (size_t)W * H;
    const bool dense = disp_stride == (size_t)W && (F == 1 || disp_fstride == px);
    if ((rc = enqueue_compute(h, dL, dR, W, H, stride, fstride, F, dense ? dDisp : nullptr, nullptr, &fin,
                              channels)))
        return rc;
    if (!dense) {
        for (int f = 0; f < F; f++)
            SDR_HIP(hipMemcpy2DAsync(dDisp + f * disp_fstride, disp_stride * 2, fin + f * px, W * 2,
                                     W * 2, H, hipMemcpyDeviceToDevice, h->stream));
        SDR_HIP(retire(h));
    }
    return SDR_OK;
}

int sdr_sgbm_compute_reproject_device(sdr_sgbm* h, const uint8_t* dL, const uint8_t* dR, int W,
                                      int H, size_t stride, size_t fstride, int F, int16_t* dDisp,
                                      const double Q[16], int handle_missing, float* dXYZ) {
    if (!h || !dL || !dR || !Q || !dXYZ) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, stride, F);
    if (rc) return rc;
    if (F > 1 && fstride < stride * H) return fail(SDR_ERR_ARG, "frame_stride too small");
    SDR_HIP(hipSetDevice(h->device));
    int16_t* fin = nullptr;
    const size_t px = (size_t)W * H;
    if ((rc = ensure(h->mins, (size_t)F * 4 * sdr::kMinSlots))) return rc;
    int* mins = handle_missing ? (int*)h->mins.p : nullptr;
    if ((rc = enqueue_compute(h, dL, dR, W, H, stride, fstride, F, dDisp, mins, &fin))) return rc;
    {
        KTimer kt(h, SDR_KERNEL_REPROJECT);
        sdr::launch_reproject_s16(fin, W, H, W, px, Q, handle_missing, mins, dXYZ, (size_t)W * 3,
                                  px * 3, F, h->stream);
    }
    SDR_HIP(retire(h));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_sgbm_compute(sdr_sgbm* h, const uint8_t* left, const uint8_t* right, int W, int H,
                     int channels, size_t stride, int16_t* disp, size_t disp_stride) {
    if (!h || !left || !right || !disp) return fail(SDR_ERR_ARG, "null argument");
    if (channels != 1 && channels != 3) return fail(SDR_ERR_TYPE, "images must have 1 or 3 channels");
    const int cn = channels;
    int rc = check_dims(W * cn, H, stride, 1);
    if (rc) return rc;
    if (disp_stride < (size_t)W) return fail(SDR_ERR_ARG, "disp_stride < width");
    if ((rc = precheck(h, W, H, cn))) return rc;
    SDR_HIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H, ib = px * cn;
    if ((rc = ensure(h->hin, 2 * ib))) return rc;
    if ((rc = h->hx.begin(2 * stage_bytes(ib) + stage_bytes(px * 2)))) return rc;
    uint8_t* dL = (uint8_t*)h->hin.p;
    uint8_t* dR = dL + ib;
    if ((rc = h->hx.upload(dL, (size_t)W * cn, left, stride, (size_t)W * cn, H, h->stream))) return rc;
    if ((rc = h->hx.upload(dR, (size_t)W * cn, right, stride, (size_t)W * cn, H, h->stream))) return rc;
    int16_t* fin = nullptr;
    if ((rc = enqueue_compute(h, dL, dR, W, H, (size_t)W * cn, ib, 1, nullptr, nullptr, &fin, cn))) {
        (void)hipStreamSynchronize(h->stream);  // the uploads from the staging buffer have landed
        return rc;
    }
    if ((rc = h->hx.download(disp, disp_stride * 2, fin, (size_t)W * 2, (size_t)W * 2, H, h->stream))) return rc;
    return h->hx.drain();
}

int sdr_sgbm_compute_reproject(sdr_sgbm* h, const uint8_t* left, const uint8_t* right, int W, int H,
                               size_t stride, int16_t* disp, size_t disp_stride, const double Q[16],
                               int handle_missing, float* xyz, size_t xyz_stride) {
    if (!h || !left || !right || !Q || !xyz) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, stride, 1);
    if (rc) return rc;
    if (disp && disp_stride < (size_t)W) return fail(SDR_ERR_ARG, "disp_stride < width");
    if (xyz_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "xyz_stride < 3*width");
    if ((rc = precheck(h, W, H, 1))) return rc;
    SDR_HIP(hipSetDevice(h->device));
    const size_t px = (size_t)W * H;
    if ((rc = ensure(h->hin, 2 * px))) return rc;
    if ((rc = ensure(h->hxyz, px * 12))) return rc;
    if ((rc = ensure(h->mins, 4 * sdr::kMinSlots))) return rc;
    if ((rc = h->hx.begin(2 * stage_bytes(px) + stage_bytes(px * 2) + stage_bytes(px * 12)))) return rc;
    uint8_t* dL = (uint8_t*)h->hin.p;
    uint8_t* dR = dL + px;
    float* dX = (float*)h->hxyz.p;
    if ((rc = h->hx.upload(dL, W, left, stride, W, H, h->stream))) return rc;
    if ((rc = h->hx.upload(dR, W, right, stride, W, H, h->stream))) return rc;
    int16_t* fin = nullptr;
    int* mins = handle_missing ? (int*)h->mins.p : nullptr;
    if ((rc = enqueue_compute(h, dL, dR, W, H, W, px, 1, nullptr, mins, &fin))) {
        (void)hipStreamSynchronize(h->stream);  // the uploads from the staging buffer have landed
        return rc;
    }
    // the disparity's copy-out overlaps the reprojection
    if (disp && (rc = h->hx.download(disp, disp_stride * 2, fin, (size_t)W * 2, (size_t)W * 2, H, h->stream)))
        return rc;
    {
        KTimer kt(h, SDR_KERNEL_REPROJECT);
        sdr::launch_reproject_s16(fin, W, H, W, px, Q, handle_missing, mins, dX, (size_t)W * 3, px * 3, 1,
                                  h->stream);
    }
    SDR_HIP(hipGetLastError());
    SDR_HIP(retire(h));
    if ((rc = h->hx.download(xyz, xyz_stride * 4, dX, (size_t)W * 12, (size_t)W * 12, H, h->stream))) return rc;
    return h->hx.drain();
}

int sdr_reproject_device(const float* d_disp, int W, int H, size_t disp_stride, const double Q[16],
                         int handle_missing, float* d_xyz, size_t xyz_stride, int F,
                         void* stream) {
    if (!d_disp || !Q || !d_xyz) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, disp_stride, F);
    if (rc) return rc;
    if (xyz_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "xyz_stride < 3*width");
    int* mins = nullptr;
    if (handle_missing) SDR_HIP(sdr::scratch_alloc((void**)&mins, F * sizeof(int), (hipStream_t)stream));
    sdr::launch_reproject_f32(d_disp, W, H, disp_stride, disp_stride * H, Q, handle_missing, mins,
                              d_xyz, xyz_stride, xyz_stride * H, F, (hipStream_t)stream);
    if (mins) SDR_HIP(sdr::scratch_free(mins, (hipStream_t)stream));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_filter_speckles_device(int16_t* d_img, int W, int H, int F, int newVal, int maxSpeckleSize,
                               int maxDiff, void* stream) {
    if (!d_img) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, (size_t)W, F);
    if (rc) return rc;
    if ((size_t)W * H > (size_t)INT32_MAX) return fail(SDR_ERR_SIZE, "frame too large");
    if (maxSpeckleSize <= 0) return SDR_OK;  // OpenCV: nothing to do
    hipStream_t st = (hipStream_t)stream;
    const size_t n = (size_t)F * W * H;
    int* scratch = nullptr;
    SDR_HIP(sdr::scratch_alloc((void**)&scratch, n * 8, st));
    sdr::launch_speckle(d_img, d_img, W, H, F, newVal, maxSpeckleSize, maxDiff, scratch, scratch + n,
                        nullptr, st);
    SDR_HIP(sdr::scratch_free(scratch, st));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_disp16_reproject_device(const int16_t* d_disp, int W, int H, size_t disp_stride,
                                const double Q[16], int handle_missing, float* d_xyz,
                                size_t xyz_stride, int F, void* stream) {
    if (!d_disp || !Q || !d_xyz) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, disp_stride, F);
    if (rc) return rc;
    if (xyz_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "xyz_stride < 3*width");
    if (handle_missing && disp_stride != (size_t)W)
        return fail(SDR_ERR_ARG, "handle_missing needs a dense disparity (disp_stride == width)");
    int* mins = nullptr;
    hipStream_t st = (hipStream_t)stream;
    if (handle_missing) {
        SDR_HIP(sdr::scratch_alloc((void**)&mins, F * sdr::kMinSlots * sizeof(int), st));
        sdr::launch_min_s16(d_disp, (size_t)W * H, disp_stride * H, F, mins, st);
    }
    sdr::launch_reproject_s16(d_disp, W, H, disp_stride, disp_stride * H, Q, handle_missing, mins,
                              d_xyz, xyz_stride, xyz_stride * H, F, st);
    if (mins) SDR_HIP(sdr::scratch_free(mins, st));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(SDR_ERR_ARG, "null argument");
    *out = nullptr;
    if (!bytes) return fail(SDR_ERR_ARG, "zero size");
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess)
        return fail(SDR_ERR_NOMEM, "hipHostMalloc failed");
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pinned[(uintptr_t)p] = bytes;
    *out = p;
    return SDR_OK;
}

int sdr_host_free(void* p) {
    if (!p) return SDR_OK;
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pinned.find((uintptr_t)p);
        if (it == g_pinned.end()) return fail(SDR_ERR_ARG, "not a block from sdr_host_alloc");
        g_pinned.erase(it);
    }
    SDR_HIP(hipHostFree(p));
    return SDR_OK;
}

int sdr_reproject(const float* disp, int W, int H, size_t disp_stride, const double Q[16],
                  int handle_missing, float* xyz, size_t xyz_stride) {
    if (!disp || !Q || !xyz) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, disp_stride, 1);
    if (rc) return rc;
    if (xyz_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "xyz_stride < 3*width");
    // per-thread persistent device buffers, staging and stream (per current device)
    struct State {
        int device = -1;
        hipStream_t st = nullptr;
        Buf dd, dx, mins;
        HostXfer hx;
        ~State() {
            if (device < 0) return;
            (void)hipSetDevice(device);
            if (st) (void)hipStreamSynchronize(st);
            for (Buf* b : {&dd, &dx, &mins})
                if (b->p) (void)hipFree(b->p);
            hx.release();
            if (st) (void)hipStreamDestroy(st);
        }
    };
    static thread_local State S;
    int dev = 0;
    SDR_HIP(hipGetDevice(&dev));
    if (S.device != dev) {
        if (S.device >= 0) {
            (void)hipSetDevice(S.device);
            S.~State();
            new (&S) State();
            SDR_HIP(hipSetDevice(dev));
        }
        SDR_HIP(hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking));
        S.device = dev;
    }
    const size_t px = (size_t)W * H;
    if ((rc = ensure(S.dd, px * 4)) || (rc = ensure(S.dx, px * 12)) || (rc = ensure(S.mins, 4))) return rc;
    if ((rc = S.hx.begin(stage_bytes(px * 4) + stage_bytes(px * 12)))) return rc;
    float* dd = (float*)S.dd.p;
    float* dx = (float*)S.dx.p;
    if ((rc = S.hx.upload(dd, (size_t)W * 4, disp, disp_stride * 4, (size_t)W * 4, H, S.st))) return rc;
    sdr::launch_reproject_f32(dd, W, H, W, px, Q, handle_missing, handle_missing ? (int*)S.mins.p : nullptr, dx,
                              (size_t)W * 3, px * 3, 1, S.st);
    SDR_HIP(hipGetLastError());
    if ((rc = S.hx.download(xyz, xyz_stride * 4, dx, (size_t)W * 12, (size_t)W * 12, H, S.st))) return rc;
    return S.hx.drain();
}

int sdr_disp16_to_float_device(const int16_t* d_disp, float* d_out, size_t n, void* stream) {
    if (!d_disp || !d_out) return fail(SDR_ERR_ARG, "null argument");
    sdr::launch_disp16_to_f32(d_disp, d_out, n, (hipStream_t)stream);
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_bgr2gray_device(const uint8_t* d_bgr, int W, int H, size_t bgr_stride, uint8_t* d_gray,
                        size_t gray_stride, int F, void* stream) {
    if (!d_bgr || !d_gray) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, gray_stride, F);
    if (rc) return rc;
    if (bgr_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "bgr_stride < 3*width");
    sdr::launch_bgr2gray(d_bgr, W, H, bgr_stride, d_gray, gray_stride, F, (hipStream_t)stream);
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

int sdr_resize_area_half_device(const uint8_t* d_src, int W, int H, size_t stride, uint8_t* d_dst,
                                size_t dst_stride, int F, void* stream) {
    if (!d_src || !d_dst) return fail(SDR_ERR_ARG, "null argument");
    int rc = check_dims(W, H, stride, F);
    if (rc) return rc;
    if ((W & 1) || (H & 1)) return fail(SDR_ERR_SIZE, "INTER_AREA 0.5x needs even width and height");
    if (dst_stride < (size_t)W / 2) return fail(SDR_ERR_ARG, "dst_stride < width/2");
    sdr::launch_area_half(d_src, W, H, stride, d_dst, dst_stride, F, (hipStream_t)stream);
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

}  // extern "C"

// StereoDisparity::computeDisparity from the half-size gray pair on the device, and optionally
// computeDepth (Q, d_xyz non-null) fused into the WLS epilogue.
static int class_enqueue(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls, const uint8_t* sl,
                         const uint8_t* sr, int w2, int h2, int F, float* d_out,
                         int16_t* d_filtered, float* d_conf, const double* Q, float* d_xyz) {
    if (!left || !sl || !sr || !d_out) return fail(SDR_ERR_ARG, "null argument");
    if (w2 <= 0 || h2 <= 0 || F <= 0) return fail(SDR_ERR_ARG, "bad size");
    if (right && right->device != left->device) return fail(SDR_ERR_ARG, "matchers on different devices");
    if (wls && !right) return fail(SDR_ERR_ARG, "the WLS filter needs the right matcher's disparity");
    SDR_HIP(hipSetDevice(left->device));
    hipStream_t st = left->stream;
    const size_t px2 = (size_t)w2 * h2;
    int rc;
    // dl and dr are one buffer [2F][h][w]: the paired launch writes both
    if ((rc = ensure(left->cls_dl, 2 * F * px2 * 2))) return rc;
    if ((rc = ensure(left->cls_wls, d_filtered ? 0 : F * px2 * 2))) return rc;
    int16_t* dl = (int16_t*)left->cls_dl.p;
    int16_t* dr = dl + F * px2;
    int16_t* dw = d_filtered ? d_filtered : (int16_t*)left->cls_wls.p;
    // matcher->compute(L, R) (stereo_disparity.cpp:27) and right_matcher->compute(R, L) (:28) are
    // independent until the WLS filter.  When the right matcher differs from the left one in
    // minDisparity alone (createRightMatcher after createDisparityWLSFilter: always on the class
    // path) both run as ONE batch of 2F frames through the same launches: at 640x360 a matcher's
    // row chains fill under a third of the chip, and no stream fork/join is needed.  Otherwise
    // the right one runs on a side stream forked from the caller's and joined back before the filter.
    int16_t* fin = nullptr;
    bool paired = false;
    if (right) {
        Eff el, er;
        paired = make_eff(left->p, w2, h2, &el) == SDR_OK && make_eff(right->p, w2, h2, &er) == SDR_OK &&
                 can_pair(el, er);
    }
    if (paired) {
        if ((rc = enqueue_compute(left, sl, sr, w2, h2, w2, px2, 2 * F, dl, nullptr, &fin, 1, &right->p)))
            return rc;
    } else if (right) {
        if (!left->side) {
            SDR_HIP(hipStreamCreateWithFlags(&left->side, hipStreamNonBlocking));
            SDR_HIP(hipEventCreateWithFlags(&left->fork, kOrderEvent));
            SDR_HIP(hipEventCreateWithFlags(&left->join, kOrderEvent));
        }
        SDR_HIP(hipEventRecord(left->fork, st));
        SDR_HIP(hipStreamWaitEvent(left->side, left->fork, 0));
        // the right matcher runs on the side stream and returns to its own stream binding without
        // touching that stream now (a transient one may already be gone): its work is relayed
        // through its own stream and its stream waits on it at its next call (begin_call)
        hipStream_t rs = right->stream;
        const bool rp = right->persistent;
        if ((rc = use_stream(right, left->side, true))) return rc;
        rc = enqueue_compute(right, sr, sl, w2, h2, w2, px2, F, dr, nullptr, &fin);
        const hipError_t re = relay(right, left->side);
        right->pending = false;
        right->stream = rs;
        right->persistent = rp;
        right->needs_wait = true;
        if (rc) return rc;
        SDR_HIP(re);
        SDR_HIP(hipEventRecord(left->join, left->side));
    }
    if (!paired) {
        if ((rc = enqueue_compute(left, sl, sr, w2, h2, w2, px2, F, dl, nullptr, &fin))) return rc;
        if (right) SDR_HIP(hipStreamWaitEvent(st, left->join, 0));
    }
    if (wls) {
        // wls_filter->filter(disp_left, left_small, filtered, disp_right) (stereo_disparity.cpp:31)
        // with filtered_disp.convertTo(CV_32F, 1/16) (:34) and computeDepth (:76-80) in its epilogue
        void* ws = sdr_wls_get_stream(wls);
        (void)sdr_wls_set_stream(wls, st);
        rc = sdr::wls_filter_enqueue(wls, dl, dr, sl, w2, h2, w2, px2, F, dw, d_conf, d_out, Q, d_xyz, left);
        (void)sdr_wls_set_stream(wls, ws);
        if (rc) return rc;
    } else {
        if (d_filtered) SDR_HIP(hipMemcpyAsync(d_filtered, dl, F * px2 * 2, hipMemcpyDeviceToDevice, st));
        sdr::launch_disp16_to_f32(dl, d_out, F * px2, st);
        if (d_xyz)
            sdr::launch_reproject_f32(d_out, w2, h2, w2, px2, Q, 0, nullptr, d_xyz, (size_t)w2 * 3, px2 * 3, F, st);
    }
    SDR_HIP(retire(left));
    SDR_HIP(hipGetLastError());
    return SDR_OK;
}

extern "C" {

int sdr_stereo_class_compute_device(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                                    const uint8_t* sl, const uint8_t* sr, int w2, int h2, int F,
                                    float* d_out, int16_t* d_filtered, float* d_conf) {
    return class_enqueue(left, right, wls, sl, sr, w2, h2, F, d_out, d_filtered, d_conf, nullptr, nullptr);
}

int sdr_stereo_class_depth_device(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                                  const uint8_t* sl, const uint8_t* sr, int w2, int h2, int F,
                                  float* d_out, int16_t* d_filtered, float* d_conf,
                                  const double Q[16], float* d_xyz) {
    if (!Q || !d_xyz) return fail(SDR_ERR_ARG, "null argument");
    return class_enqueue(left, right, wls, sl, sr, w2, h2, F, d_out, d_filtered, d_conf, Q, d_xyz);
}

int sdr_stereo_class_compute(sdr_sgbm* left, sdr_sgbm* right, sdr_wls* wls,
                             const uint8_t* bgr_left, const uint8_t* bgr_right, int W, int H,
                             size_t bgr_stride, float* out, size_t out_stride, int16_t* disp_left,
                             int16_t* disp_right, int16_t* filtered, float* conf) {
    if (!left || !bgr_left || !bgr_right || !out) return fail(SDR_ERR_ARG, "null argument");
    if (W <= 0 || H <= 0 || bgr_stride < (size_t)W * 3) return fail(SDR_ERR_ARG, "bad size/stride");
    if ((W & 1) || (H & 1)) return fail(SDR_ERR_SIZE, "INTER_AREA 0.5x needs even width and height");
    const int w2 = W / 2, h2 = H / 2;
    if (out_stride < (size_t)w2) return fail(SDR_ERR_ARG, "out_stride < width/2");
    int rc;
    if ((rc = precheck(left, w2, h2, 1)) || (right && (rc = precheck(right, w2, h2, 1)))) return rc;
    SDR_HIP(hipSetDevice(left->device));
    hipStream_t st = left->stream;
    const size_t px = (size_t)W * H, px2 = (size_t)w2 * h2;
    if ((rc = ensure(left->cls_bgr, 2 * px * 3))) return rc;
    if ((rc = ensure(left->cls_gray, 2 * px))) return rc;
    if ((rc = ensure(left->cls_small, 2 * px2))) return rc;
    if ((rc = ensure(left->cls_f, px2 * 4))) return rc;
    if ((rc = ensure(left->cls_conf, conf ? px2 * 4 : 0))) return rc;
    if ((rc = ensure(left->cls_filt, px2 * 2))) return rc;
    uint8_t* bgr = (uint8_t*)left->cls_bgr.p;
    uint8_t* gray = (uint8_t*)left->cls_gray.p;
    uint8_t* small = (uint8_t*)left->cls_small.p;
    float* f = (float*)left->cls_f.p;
    int16_t* filt = (int16_t*)left->cls_filt.p;
    float* dconf = conf ? (float*)left->cls_conf.p : nullptr;
    // host copies through the handle's page-locked staging (DMA straight from/to sdr_host_alloc
    // buffers, e.g. the facade's Mats)
    if ((rc = left->hx.begin(2 * stage_bytes(px * 3) + stage_bytes(px2 * 4) * 3 + stage_bytes(px2 * 2) * 3)))
        return rc;
    if ((rc = left->hx.upload(bgr, (size_t)W * 3, bgr_left, bgr_stride, (size_t)W * 3, H, st))) return rc;
    if ((rc = left->hx.upload(bgr + px * 3, (size_t)W * 3, bgr_right, bgr_stride, (size_t)W * 3, H, st))) return rc;
    // cvtColor(BGR2GRAY) x2, resize(0.5, INTER_AREA) x2 (stereo_disparity.cpp:19-24)
    sdr::launch_bgr2gray(bgr, W, H, (size_t)W * 3, gray, W, 2, st);
    sdr::launch_area_half(gray, W, H, W, small, w2, 2, st);
    if ((rc = class_enqueue(left, right, wls, small, small + px2, w2, h2, 1, f, filt, dconf, nullptr, nullptr))) {
        (void)hipStreamSynchronize(st);  // the uploads from the staging buffer have landed
        return rc;
    }
    HostXfer& hx = left->hx;
    if ((rc = hx.download(out, out_stride * 4, f, (size_t)w2 * 4, (size_t)w2 * 4, h2, st))) return rc;
    if (disp_left && (rc = hx.download(disp_left, (size_t)w2 * 2, left->cls_dl.p, (size_t)w2 * 2, (size_t)w2 * 2, h2, st)))
        return rc;
    if (disp_right && right &&
        (rc = hx.download(disp_right, (size_t)w2 * 2, (int16_t*)left->cls_dl.p + px2, (size_t)w2 * 2, (size_t)w2 * 2, h2, st)))
        return rc;
    if (filtered && (rc = hx.download(filtered, (size_t)w2 * 2, filt, (size_t)w2 * 2, (size_t)w2 * 2, h2, st))) return rc;
    if (conf && wls && (rc = hx.download(conf, (size_t)w2 * 4, dconf, (size_t)w2 * 4, (size_t)w2 * 4, h2, st))) return rc;
    return hx.drain();
}

int sdr_sgbm_kernel_time(sdr_sgbm* h, int kind, int reset, float* total_ms, int* count) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    float tot = 0;
    int n = 0;
    if (h->kused) {
        SDR_HIP(hipEventSynchronize(h->kev[2 * h->kused - 1]));
        for (size_t i = 0; i < h->kused; i++) {
            if (kind >= 0 && h->kkind[i] != kind) continue;
            float ms = 0;
            SDR_HIP(hipEventElapsedTime(&ms, h->kev[2 * i], h->kev[2 * i + 1]));
            tot += ms;
            n++;
        }
    }
    if (total_ms) *total_ms = tot;
    if (count) *count = n;
    if (reset) h->kused = 0;
    return SDR_OK;
}

int sdr_sgbm_last_status(sdr_sgbm* h) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    if (!h->status_host) return SDR_OK;  // no sweep batch has run on this handle
    SDR_HIP(hipSetDevice(h->device));
    if (h->persistent) SDR_HIP(hipStreamSynchronize(h->stream));
    SDR_HIP(hipStreamSynchronize(h->own_stream));  // relayed work (transient streams, side stream)
    const int n = __atomic_load_n(h->status_host, __ATOMIC_ACQUIRE);
    if (n == h->status_reported) return SDR_OK;
    h->status_reported = n;  // the device word counts timeouts and is never cleared
    return fail(SDR_ERR_DEVICE, "a MODE_HH row sweep timed out waiting for a neighbouring tile: that "
                                "batch's frames were written as INVALID");
}

int sdr_sgbm_debug_knob(sdr_sgbm* h, int knob, int value) {
    if (!h) return fail(SDR_ERR_ARG, "null handle");
    if (knob != SDR_DEBUG_SWEEP_SPIN) return fail(SDR_ERR_ARG, "unknown knob");
    h->sweep_spin = value > 0 ? value : sdr::kSweepSpin;
    return SDR_OK;
}

int sdr_sgbm_debug_stage(const sdr_sgbm* h, int stage, void* dst, size_t bytes) {
    if (!h || !dst) return fail(SDR_ERR_ARG, "null argument");
    const Buf* b = stage == 0 ? &h->C : stage == 1 ? &h->draw : stage == 2 ? &h->dlr
                 : stage == 3 ? &h->dfin : stage == 4 ? &h->Lr : stage == 5 ? &h->keys2
                 : stage == 6 ? &h->Caux : nullptr;
    if (!b) return fail(SDR_ERR_ARG, "bad stage");
    // front slack (the L records' is P-1 times C's)
    const size_t skip = stage == 0 ? h->path_slack * 2 : stage == 4 ? h->path_lslack * 2
                      : stage == 6 ? h->aux_slack * 2 : 0;
    if (!b->p || bytes + skip > b->n) return fail(SDR_ERR_ARG, "stage buffer smaller than requested");
    SDR_HIP(hipSetDevice(h->device));
    // the LR-checked map is never written by the pipeline: materialise it for this stage
    if (stage == 2 && h->draw.p && h->dlr.p) {
        const size_t px = (size_t)h->lr_g.W * h->lr_g.H;
        if (h->lr_skipped)
            sdr::launch_mask_cols((const int16_t*)h->draw.p, (int16_t*)h->dlr.p, h->lr_g, h->lr_frames, h->stream);
        else
            sdr::launch_lr_apply(h->lr_g, (const int16_t*)h->draw.p, (const uint32_t*)h->keys2.p,
                                 (int16_t*)h->dlr.p, px, h->lr_d12, h->lr_frames, h->stream);
    }
    SDR_HIP(hipStreamSynchronize(h->stream));
    SDR_HIP(hipMemcpy(dst, (const char*)b->p + skip, bytes, hipMemcpyDeviceToHost));
    return SDR_OK;
}

int sdr_stream_probe(int device, size_t bytes, int iters, double* gbs) {
    if (!gbs || bytes < 16 || iters < 1) return fail(SDR_ERR_ARG, "bad argument");
    int ndev = 0;
    SDR_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SDR_ERR_DEVICE, "invalid device index");
    SDR_HIP(hipSetDevice(device));
    return sdr::stream_probe(bytes, iters, gbs) ? fail(SDR_ERR_NOMEM, "stream probe failed") : SDR_OK;
}

int sdr_stream_probe_ex(int device, size_t bytes, int iters, double* gbs3) {
    if (!gbs3 || bytes < 16 || iters < 1) return fail(SDR_ERR_ARG, "bad argument");
    int ndev = 0;
    SDR_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SDR_ERR_DEVICE, "invalid device index");
    SDR_HIP(hipSetDevice(device));
    return sdr::stream_probe_ex(bytes, iters, gbs3) ? fail(SDR_ERR_NOMEM, "stream probe failed") : SDR_OK;
}

int sdr_selftest_wave_ops(int* failures4) {
    if (!failures4) return fail(SDR_ERR_ARG, "null argument");
    return sdr::selftest_wave_ops(failures4) ? fail(SDR_ERR_DEVICE, "selftest launch failed") : SDR_OK;
}

}  // extern "C"
