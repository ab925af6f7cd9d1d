"""cv::StereoSGBM / cv::reprojectImageTo3D surface over the HIP engine (include/sdr/sdr.h).

Mirrors the OpenCV API the reference calls (same names, argument order and meaning):

* ``StereoSGBM.create(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff,
  preFilterCap, uniquenessRatio, speckleWindowSize, speckleRange, mode)``
  -- reference stereo_vision/src/stereo_disparity.cpp:5-9, point_cloud/src/pcd_write.cpp:102-108
* ``matcher.compute(left, right)`` -> CV_16S disparity (1/16 px)
  -- stereo_disparity.cpp:27-28, pcd_write.cpp:111
* ``reprojectImageTo3D(disp, Q, handleMissingValues)`` -> float32 (H, W, 3)
  -- stereo_disparity.cpp:78, pcd_write.cpp:116
* ``createRightMatcher(matcher)`` -- ximgproc, stereo_disparity.cpp:10

Inputs may be numpy arrays (host: H2D + compute + D2H, synchronous) or torch CUDA tensors
(device: enqueued on torch's current stream, no copies).  Errors raise ``SDRError`` where OpenCV
raises ``cv2.error`` (same conditions: size/type mismatch, numDisparities % 16 != 0, ...).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SDRError, SgbmParams, check, lib

try:  # torch is plumbing (device memory / streams); numpy-only use needs no torch
    import torch
except Exception:  # pragma: no cover
    torch = None

MODE_SGBM, MODE_HH, MODE_SGBM_3WAY, MODE_HH4 = 0, 1, 2, 3
UNIQ_AUTO, UNIQ_SCALAR, UNIQ_SIMD = 0, 1, 2
# SDR_KERNEL_* (include/sdr/sdr.h)
(KERNEL_PREFILTER, KERNEL_COST, KERNEL_PATHS, KERNEL_WTA_LR, KERNEL_MEDIAN, KERNEL_SPECKLE,
 KERNEL_REPROJECT, KERNEL_LR_CHECK, KERNEL_SWEEP, KERNEL_WLS_PREP, KERNEL_FGS, KERNEL_WLS_FINAL,
 KERNEL_SWEEP_DOWN, KERNEL_FGS_COEF) = range(14)
DEBUG_SWEEP_SPIN = 1  # sdr_sgbm_debug_knob


def _is_cuda(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _cstream(device_index: int):
    return ctypes.c_void_p(torch.cuda.current_stream(device_index).cuda_stream)


STREAM_PERSISTENT = 1  # SDR_STREAM_PERSISTENT (include/sdr/sdr.h)


def stream_is_pooled(stream_id: int) -> bool:
    """True for torch's default stream and its pooled streams, which live as long as the process;
    False for a torch.cuda.ExternalStream, which its owner may destroy.  c10's StreamId encodes an
    external stream as the stream pointer itself (even, non-zero: c10/cuda/CUDAStream.cpp
    streamIdType) and every stream torch allocates with the low bit set (the default stream is 0)."""
    return stream_id == 0 or (stream_id & 1) == 1


def set_handle_stream(h, device_index: int, stream=None):
    """Points a matcher handle at `stream` (default: the current stream of the device).  torch's
    own streams are bound persistent (the handle's retire event is recorded only at a stream
    switch); an external stream is bound transient, so the caller may destroy it after the call
    (sdr.h sdr_sgbm_set_stream_ex)."""
    s = stream if stream is not None else torch.cuda.current_stream(device_index)
    flags = STREAM_PERSISTENT if stream_is_pooled(int(s.stream_id)) else 0
    check(lib().sdr_sgbm_set_stream_ex(h, ctypes.c_void_p(s.cuda_stream), flags))


def _Q(Q) -> ctypes.Array:
    q = np.ascontiguousarray(np.asarray(Q, dtype=np.float64).reshape(16))
    return (ctypes.c_double * 16)(*q.tolist())


class StereoSGBM:
    MODE_SGBM = MODE_SGBM
    MODE_HH = MODE_HH
    MODE_SGBM_3WAY = MODE_SGBM_3WAY
    MODE_HH4 = MODE_HH4

    def __init__(self, params: SgbmParams, device: int = 0):
        self._p = SgbmParams()
        ctypes.pointer(self._p)[0] = params
        self._device = int(device)
        h = ctypes.c_void_p()
        check(lib().sdr_sgbm_create(ctypes.byref(self._p), self._device, ctypes.byref(h)))
        self._h = h

    @classmethod
    def create(cls, minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0,
               preFilterCap=0, uniquenessRatio=0, speckleWindowSize=0, speckleRange=0,
               mode=MODE_SGBM, *, device=0, nstripes=4, uniq_rule=UNIQ_AUTO) -> "StereoSGBM":
        """cv::StereoSGBM::create with OpenCV's defaults."""
        p = SgbmParams(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff, preFilterCap,
                       uniquenessRatio, speckleWindowSize, speckleRange, mode, nstripes, uniq_rule)
        return cls(p, device)

    # ---- lifetime ----
    def close(self):
        if getattr(self, "_h", None):
            lib().sdr_sgbm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- params (cv::StereoSGBM getters/setters) ----
    def _set(self, name, value):
        setattr(self._p, name, int(value))
        check(lib().sdr_sgbm_set_params(self._h, ctypes.byref(self._p)))

    def params(self) -> SgbmParams:
        p = SgbmParams()
        check(lib().sdr_sgbm_get_params(self._h, ctypes.byref(p)))
        return p

    def getMinDisparity(self): return self._p.minDisparity
    def setMinDisparity(self, v): self._set("minDisparity", v)
    def getNumDisparities(self): return self._p.numDisparities
    def setNumDisparities(self, v): self._set("numDisparities", v)
    def getBlockSize(self): return self._p.blockSize
    def setBlockSize(self, v): self._set("blockSize", v)
    def getP1(self): return self._p.P1
    def setP1(self, v): self._set("P1", v)
    def getP2(self): return self._p.P2
    def setP2(self, v): self._set("P2", v)
    def getDisp12MaxDiff(self): return self._p.disp12MaxDiff
    def setDisp12MaxDiff(self, v): self._set("disp12MaxDiff", v)
    def getPreFilterCap(self): return self._p.preFilterCap
    def setPreFilterCap(self, v): self._set("preFilterCap", v)
    def getUniquenessRatio(self): return self._p.uniquenessRatio
    def setUniquenessRatio(self, v): self._set("uniquenessRatio", v)
    def getSpeckleWindowSize(self): return self._p.speckleWindowSize
    def setSpeckleWindowSize(self, v): self._set("speckleWindowSize", v)
    def getSpeckleRange(self): return self._p.speckleRange
    def setSpeckleRange(self, v): self._set("speckleRange", v)
    def getMode(self): return self._p.mode
    def setMode(self, v): self._set("mode", v)

    # ---- compute ----
    def compute(self, left, right, disp=None):
        """StereoSGBM::compute: 8-bit pair (CV_8UC1, or CV_8UC3 whose channels' costs are summed)
        -> int16 disparity (1/16 px).

        numpy (H, W) or (H, W, 3) -> numpy; torch CUDA uint8 (H, W), (F, H, W), (H, W, 3) or
        (F, H, W, 3) -> torch int16 on the same device, enqueued on the current stream (a 3-dim
        tensor whose last dimension is 3 is one colour frame).
        """
        if _is_cuda(left) or _is_cuda(right):
            return self._compute_device(left, right, disp)
        left = np.asarray(left)
        right = np.asarray(right)
        if left.shape != right.shape or left.dtype != right.dtype:
            raise SDRError(-1, "left and right images must have the same size and type")
        if left.dtype != np.uint8:
            raise SDRError(-5, "images must be 8-bit")
        if left.ndim == 3 and left.shape[2] == 1:
            left, right = left[..., 0], right[..., 0]
        if not (left.ndim == 2 or (left.ndim == 3 and left.shape[2] == 3)):
            raise SDRError(-5, "images must have 1 or 3 channels")
        left = np.ascontiguousarray(left)
        right = np.ascontiguousarray(right)
        h, w = left.shape[:2]
        cn = 1 if left.ndim == 2 else 3
        out = disp if disp is not None else np.empty((h, w), np.int16)
        if out.shape != (h, w) or out.dtype != np.int16 or not out.flags.c_contiguous:
            raise SDRError(-1, "disp must be a C-contiguous int16 (H, W) array")
        check(lib().sdr_sgbm_compute(self._h, left.ctypes.data, right.ctypes.data, w, h, cn, w * cn,
                                     out.ctypes.data, w))
        return out

    def _prep_device(self, left, right):
        if not (_is_cuda(left) and _is_cuda(right)):
            raise SDRError(-1, "left and right must both be CUDA tensors")
        if left.shape != right.shape or left.dtype != right.dtype:
            raise SDRError(-1, "left and right images must have the same size and type")
        if left.dtype != torch.uint8:
            raise SDRError(-5, "images must be 8-bit")
        if left.dim() == 2:
            left, right = left.unsqueeze(0), right.unsqueeze(0)
        if left.dim() != 3:
            raise SDRError(-5, "expected (H, W) or (F, H, W) single-channel tensors")
        if left.device.index != self._device:
            raise SDRError(-1, f"tensors are on cuda:{left.device.index}, matcher on cuda:{self._device}")
        return left.contiguous(), right.contiguous()

    def _compute_device(self, left, right, disp=None):
        if left.dim() == 4 or (left.dim() == 3 and left.shape[-1] == 3):
            return self._compute_device_color(left, right, disp)
        squeeze = left.dim() == 2
        left, right = self._prep_device(left, right)
        f, h, w = left.shape
        out = disp if disp is not None else torch.empty((f, h, w), dtype=torch.int16, device=left.device)
        if out.numel() != f * h * w or out.dtype != torch.int16 or not out.is_contiguous():
            raise SDRError(-1, "disp must be a contiguous int16 tensor of the input shape")
        set_handle_stream(self._h, self._device)
        check(lib().sdr_sgbm_compute_device(self._h, left.data_ptr(), right.data_ptr(), w, h, w,
                                            w * h, f, out.data_ptr(), w, w * h))
        return out[0] if squeeze and disp is None else out

    def _compute_device_color(self, left, right, disp=None):
        if not (_is_cuda(left) and _is_cuda(right)) or left.shape != right.shape or left.dtype != right.dtype:
            raise SDRError(-1, "left and right must be CUDA tensors of the same size and type")
        if left.dtype != torch.uint8 or left.shape[-1] != 3:
            raise SDRError(-5, "expected 8-bit (H, W, 3) or (F, H, W, 3) tensors")
        if left.device.index != self._device:
            raise SDRError(-1, f"tensors are on cuda:{left.device.index}, matcher on cuda:{self._device}")
        squeeze = left.dim() == 3
        if squeeze:
            left, right = left.unsqueeze(0), right.unsqueeze(0)
        left, right = left.contiguous(), right.contiguous()
        f, h, w, _ = left.shape
        out = disp if disp is not None else torch.empty((f, h, w), dtype=torch.int16, device=left.device)
        if out.numel() != f * h * w or out.dtype != torch.int16 or not out.is_contiguous():
            raise SDRError(-1, "disp must be a contiguous int16 tensor of the input's (F, H, W)")
        set_handle_stream(self._h, self._device)
        check(lib().sdr_sgbm_compute_device_cn(self._h, left.data_ptr(), right.data_ptr(), w, h, 3, w * 3,
                                               w * h * 3, f, out.data_ptr(), w, w * h))
        return out[0] if squeeze and disp is None else out

    def compute_reproject(self, left, right, Q, handleMissingValues=False, disp=None, xyz=None):
        """Fused pcd_write.cpp:111-116 hot path: compute -> /16 -> reprojectImageTo3D.

        torch CUDA inputs: on device, returns (disp int16 (F,H,W), xyz float32 (F,H,W,3)).
        numpy (H, W) inputs: the synchronous host-pointer call (sdr_sgbm_compute_reproject),
        returns (disp int16 (H,W), xyz float32 (H,W,3)) as numpy; disp=False skips the disparity."""
        if not (_is_cuda(left) or _is_cuda(right)):
            return self._compute_reproject_host(left, right, Q, handleMissingValues, disp, xyz)
        left, right = self._prep_device(left, right)
        f, h, w = left.shape
        if disp is None:
            disp = torch.empty((f, h, w), dtype=torch.int16, device=left.device)
        if xyz is None:
            xyz = torch.empty((f, h, w, 3), dtype=torch.float32, device=left.device)
        set_handle_stream(self._h, self._device)
        check(lib().sdr_sgbm_compute_reproject_device(
            self._h, left.data_ptr(), right.data_ptr(), w, h, w, w * h, f, disp.data_ptr(), _Q(Q),
            int(bool(handleMissingValues)), xyz.data_ptr()))
        return disp, xyz

    def _compute_reproject_host(self, left, right, Q, hm, disp, xyz):
        left, right = np.asarray(left), np.asarray(right)
        if left.shape != right.shape or left.dtype != np.uint8 or right.dtype != np.uint8 or left.ndim != 2:
            raise SDRError(-5, "expected two 8-bit single-channel (H, W) images")
        left, right = np.ascontiguousarray(left), np.ascontiguousarray(right)
        h, w = left.shape
        if disp is None:
            disp = np.empty((h, w), np.int16)
        if xyz is None:
            xyz = np.empty((h, w, 3), np.float32)
        for a, shape, dt in ((disp, (h, w), np.int16), (xyz, (h, w, 3), np.float32)):
            if a is not False and (a.shape != shape or a.dtype != dt or not a.flags.c_contiguous):
                raise SDRError(-1, f"output must be a C-contiguous {np.dtype(dt).name} {shape} array")
        dptr = disp.ctypes.data if disp is not False else None
        check(lib().sdr_sgbm_compute_reproject(self._h, left.ctypes.data, right.ctypes.data, w, h, w, dptr, w,
                                               _Q(Q), int(bool(hm)), xyz.ctypes.data, w * 3))
        return (disp if disp is not False else None), xyz

    def debug_stage(self, stage: int, shape, dtype):
        """Copy an internal buffer of the last compute (0 C, 1 raw WTA, 2 LR, 3 final, 4 path costs,
        5 disp2 keys)."""
        out = np.empty(shape, dtype)
        check(lib().sdr_sgbm_debug_stage(self._h, int(stage), out.ctypes.data, out.nbytes))
        return out

    def debug_cost_volume(self, H: int, W1: int, D: int) -> np.ndarray:
        """The first frame's cost volume C of the last compute as (H, W1, D) int16."""
        return self.debug_stage(0, (H, W1, D), np.int16)

    def check_status(self):
        """Raises SDRError(SDR_ERR_DEVICE) if a device batch since the last check had a row sweep
        give up waiting (its frames were written as INVALID; sdr_sgbm_last_status).  Synchronises
        the handle's stream."""
        check(lib().sdr_sgbm_last_status(self._h))

    def set_debug_knob(self, knob: int, value: int):
        """Test hook (sdr_sgbm_debug_knob): DEBUG_SWEEP_SPIN = polls before a sweep wait gives up."""
        check(lib().sdr_sgbm_debug_knob(self._h, int(knob), int(value)))

    def enable_timing(self, level=1):
        """0 off, 1 per-stage events, 2 per-stage + per-kernel-launch events."""
        check(lib().sdr_sgbm_enable_timing(self._h, int(level)))

    def kernel_time(self, kind: int, reset: bool = False):
        """(total_ms, launches) of one SDR_KERNEL_* kind since the last reset (timing level 2)."""
        t, n = ctypes.c_float(), ctypes.c_int()
        check(lib().sdr_sgbm_kernel_time(self._h, int(kind), int(bool(reset)), ctypes.byref(t), ctypes.byref(n)))
        return t.value, n.value

    def last_timing(self):
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        check(lib().sdr_sgbm_last_timing(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"cost_ms": a.value, "paths_ms": b.value, "post_ms": c.value}


def host_empty(shape, dtype) -> np.ndarray:
    """A numpy array in page-locked host memory (sdr_host_alloc; the role of cv::cuda::HostMem).
    Given to the host-pointer calls, it is copied by DMA directly, without a staging copy."""
    import weakref
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    n = max(count * dt.itemsize, 1)
    p = ctypes.c_void_p()
    check(lib().sdr_host_alloc(n, ctypes.byref(p)))
    buf = (ctypes.c_char * n).from_address(p.value)
    weakref.finalize(buf, lib().sdr_host_free, p.value)
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


def createRightMatcher(matcher_left: StereoSGBM) -> StereoSGBM:
    """cv::ximgproc::createRightMatcher for an SGBM matcher."""
    r = SgbmParams()
    lib().sdr_right_matcher_params(ctypes.byref(matcher_left._p), ctypes.byref(r))
    return StereoSGBM(r, matcher_left._device)


def reprojectImageTo3D(disparity, Q, handleMissingValues=False):
    """cv::reprojectImageTo3D(disparity, _3dImage, Q, handleMissingValues) -> float32 (..., H, W, 3).

    numpy float32/int16 (H, W) -> numpy; torch CUDA (H, W) / (F, H, W) -> torch on the current
    stream.  As in OpenCV, int16 input is used as-is (no 1/16 scaling); see reproject_disp16 for
    the fused convertTo(CV_32F, 1/16) + reproject of the reference (pcd_write.cpp:112-116)."""
    if _is_cuda(disparity):
        d = disparity
        squeeze = d.dim() == 2
        if squeeze:
            d = d.unsqueeze(0)
        if d.dtype != torch.float32:
            if d.dtype not in (torch.int16, torch.uint8, torch.int32):
                raise SDRError(-5, "disparity must be float32, int16, int32 or uint8")
            d = d.to(torch.float32)
        d = d.contiguous()
        f, h, w = d.shape
        out = torch.empty((f, h, w, 3), dtype=torch.float32, device=d.device)
        check(lib().sdr_reproject_device(d.data_ptr(), w, h, w, _Q(Q), int(bool(handleMissingValues)),
                                         out.data_ptr(), w * 3, f, _cstream(d.device.index)))
        return out[0] if squeeze else out
    d = np.asarray(disparity)
    if d.dtype not in (np.float32, np.int16, np.uint8, np.int32):
        raise SDRError(-5, "disparity must be float32, int16, int32 or uint8")
    d = np.ascontiguousarray(d, dtype=np.float32)
    if d.ndim != 2:
        raise SDRError(-1, "disparity must be 2-D")
    h, w = d.shape
    out = np.empty((h, w, 3), np.float32)
    check(lib().sdr_reproject(d.ctypes.data, w, h, w, _Q(Q), int(bool(handleMissingValues)),
                              out.ctypes.data, w * 3))
    return out


def reproject_disp16(disp16, Q, handleMissingValues=False):
    """Fused disp.convertTo(CV_32F, 1/16) + reprojectImageTo3D on device (pcd_write.cpp:112-116)."""
    if not _is_cuda(disp16) or disp16.dtype != torch.int16:
        raise SDRError(-5, "reproject_disp16 expects a CUDA int16 tensor")
    d = disp16
    squeeze = d.dim() == 2
    if squeeze:
        d = d.unsqueeze(0)
    d = d.contiguous()
    f, h, w = d.shape
    out = torch.empty((f, h, w, 3), dtype=torch.float32, device=d.device)
    check(lib().sdr_disp16_reproject_device(d.data_ptr(), w, h, w, _Q(Q), int(bool(handleMissingValues)),
                                            out.data_ptr(), w * 3, f, _cstream(d.device.index)))
    return out[0] if squeeze else out


def filterSpeckles(img, newVal, maxSpeckleSize, maxDiff):
    """cv::filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) in place on a CUDA int16 tensor
    (H, W) or (F, H, W): 4-connected components of pixels that differ by <= maxDiff, excluding
    newVal pixels, of <= maxSpeckleSize pixels are set to newVal.  Returns img."""
    if not _is_cuda(img) or img.dtype != torch.int16 or not img.is_contiguous():
        raise SDRError(-5, "filterSpeckles expects a contiguous CUDA int16 tensor")
    if img.dim() not in (2, 3):
        raise SDRError(-1, "filterSpeckles expects (H, W) or (F, H, W)")
    f = 1 if img.dim() == 2 else img.shape[0]
    h, w = img.shape[-2:]
    check(lib().sdr_filter_speckles_device(img.data_ptr(), w, h, f, int(newVal), int(maxSpeckleSize),
                                           int(maxDiff), _cstream(img.device.index)))
    return img


def disparity_to_float(disp16):
    """disp.convertTo(f, CV_32F, 1/16) (device tensors stay on device)."""
    if _is_cuda(disp16):
        out = torch.empty(disp16.shape, dtype=torch.float32, device=disp16.device)
        src = disp16.contiguous()
        check(lib().sdr_disp16_to_float_device(src.data_ptr(), out.data_ptr(), src.numel(),
                                               _cstream(src.device.index)))
        return out
    return np.asarray(disp16, dtype=np.int16).astype(np.float32) * np.float32(0.0625)


def cvt_bgr2gray(bgr):
    """cv::cvtColor(bgr, gray, COLOR_BGR2GRAY) on device: uint8 (H, W, 3) or (F, H, W, 3)."""
    if not _is_cuda(bgr):
        raise SDRError(-1, "cvt_bgr2gray expects a CUDA tensor")
    x = bgr.contiguous()
    squeeze = x.dim() == 3
    if squeeze:
        x = x.unsqueeze(0)
    f, h, w, c = x.shape
    if c != 3 or x.dtype != torch.uint8:
        raise SDRError(-5, "expected uint8 BGR")
    out = torch.empty((f, h, w), dtype=torch.uint8, device=x.device)
    check(lib().sdr_bgr2gray_device(x.data_ptr(), w, h, w * 3, out.data_ptr(), w, f,
                                    _cstream(x.device.index)))
    return out[0] if squeeze else out


def resize_area_half(src):
    """cv::resize(src, dst, Size(), 0.5, 0.5, INTER_AREA) on device: uint8 (H, W) or (F, H, W)."""
    if not _is_cuda(src):
        raise SDRError(-1, "resize_area_half expects a CUDA tensor")
    x = src.contiguous()
    squeeze = x.dim() == 2
    if squeeze:
        x = x.unsqueeze(0)
    f, h, w = x.shape
    out = torch.empty((f, h // 2, w // 2), dtype=torch.uint8, device=x.device)
    check(lib().sdr_resize_area_half_device(x.data_ptr(), w, h, w, out.data_ptr(), w // 2, f,
                                            _cstream(x.device.index)))
    return out[0] if squeeze else out


def selftest_wave_ops():
    fails = (ctypes.c_int * 4)()
    check(lib().sdr_selftest_wave_ops(fails))
    return list(fails)
