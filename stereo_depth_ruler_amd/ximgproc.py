"""cv::ximgproc surface the reference's class path uses, over the HIP engine (include/sdr/sdr.h):

* ``createRightMatcher(matcher)``                      -- stereo_disparity.cpp:10
* ``createDisparityWLSFilter(matcher)``                -- stereo_disparity.cpp:11 (mutates the
  left matcher as ximgproc does: disp12MaxDiff 1e6, speckleWindowSize 0, uniquenessRatio 0)
* ``DisparityWLSFilter.setLambda / setSigmaColor``     -- stereo_disparity.cpp:12-13
* ``DisparityWLSFilter.filter(dl, left_view, dr)``     -- stereo_disparity.cpp:31
* ``DisparityWLSFilter.getConfidenceMap()``            -- stereo_disparity.cpp:36
* ``fastGlobalSmootherFilter(guide, src, lambda, sigma_color, attenuation, iters)``

Host numpy inputs run synchronously (H2D, kernels, D2H); torch CUDA tensors run on the current
stream without copies.  No CPU fallback exists: a missing libsdr.so raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import FGS_PCR, FGS_THOMAS, SDRError, WlsParams, check, lib  # noqa: F401
from .sgbm import StereoSGBM, _cstream, _is_cuda, createRightMatcher, torch  # noqa: F401


class DisparityWLSFilter:
    def __init__(self, params: WlsParams, device: int = 0):
        self._p = WlsParams()
        ctypes.pointer(self._p)[0] = params
        self._device = int(device)
        h = ctypes.c_void_p()
        check(lib().sdr_wls_create(ctypes.byref(self._p), self._device, ctypes.byref(h)))
        self._h = h
        self._conf = None

    def close(self):
        if getattr(self, "_h", None):
            lib().sdr_wls_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _set(self, name, value):
        setattr(self._p, name, value)
        check(lib().sdr_wls_set_params(self._h, ctypes.byref(self._p)))

    # ---- cv::ximgproc::DisparityWLSFilter getters / setters ----
    def getLambda(self): return self._p.lambda_
    def setLambda(self, v): self._set("lambda_", float(v))
    def getSigmaColor(self): return self._p.sigma_color
    def setSigmaColor(self, v): self._set("sigma_color", float(v))
    def getLRCthresh(self): return self._p.lrc_thresh
    def setLRCthresh(self, v): self._set("lrc_thresh", int(v))
    def getDepthDiscontinuityRadius(self): return self._p.depth_discontinuity_radius
    def setDepthDiscontinuityRadius(self, v): self._set("depth_discontinuity_radius", int(v))
    # engine extension: the FGS line solver (FGS_THOMAS, the default, or FGS_PCR: sdr.h)
    def getFgsSolver(self): return self._p.fgs_solver
    def setFgsSolver(self, v): self._set("fgs_solver", int(v))

    def params(self) -> WlsParams:
        p = WlsParams()
        check(lib().sdr_wls_get_params(self._h, ctypes.byref(p)))
        return p

    def getROI(self, width: int, height: int):
        """Valid ROI (x, y, w, h) for a width x height left disparity map."""
        r = (ctypes.c_int * 4)()
        check(lib().sdr_wls_get_roi(self._h, int(width), int(height), r))
        return tuple(r)

    def getConfidenceMap(self):
        """Confidence (x255, float32) of the last filter() call, like ximgproc's."""
        return self._conf

    def filter(self, disparity_map_left, left_view, disparity_map_right):
        """DisparityWLSFilter::filter(disp_left, left_view, filtered, disp_right).

        int16 (H, W) maps + 8-bit gray guide (H, W) -> filtered int16 (H, W).  torch CUDA
        tensors may carry a leading frame dimension (F, H, W)."""
        if _is_cuda(disparity_map_left):
            return self._filter_device(disparity_map_left, left_view, disparity_map_right)
        dl = np.asarray(disparity_map_left)
        dr = np.asarray(disparity_map_right)
        g = np.asarray(left_view)
        if dl.dtype != np.int16 or dr.dtype != np.int16:
            raise SDRError(-5, "disparity maps must be CV_16S (int16)")
        if g.dtype != np.uint8:
            raise SDRError(-5, "left_view must be 8-bit")
        if g.ndim == 3 and g.shape[2] == 3:
            from .sgbm import cvt_bgr2gray
            g = cvt_bgr2gray(g)
        if dl.ndim != 2 or dl.shape != dr.shape or g.shape[:2] != dl.shape:
            raise SDRError(-1, "disparity maps and guide must have the same (H, W) size")
        dl = np.ascontiguousarray(dl)
        dr = np.ascontiguousarray(dr)
        g = np.ascontiguousarray(g)
        h, w = dl.shape
        out = np.empty((h, w), np.int16)
        conf = np.empty((h, w), np.float32)
        check(lib().sdr_wls_filter(self._h, dl.ctypes.data, dr.ctypes.data, g.ctypes.data, w, h, w,
                                   out.ctypes.data, conf.ctypes.data))
        self._conf = conf
        return out

    def _filter_device(self, dl, g, dr):
        if not (_is_cuda(dr) and _is_cuda(g)):
            raise SDRError(-1, "disparity maps and guide must all be CUDA tensors")
        squeeze = dl.dim() == 2
        if squeeze:
            dl, dr, g = dl.unsqueeze(0), dr.unsqueeze(0), g.unsqueeze(0)
        if dl.dtype != torch.int16 or dr.dtype != torch.int16 or g.dtype != torch.uint8:
            raise SDRError(-5, "int16 disparity maps and an 8-bit guide are required")
        if dl.shape != dr.shape or g.shape != dl.shape or dl.dim() != 3:
            raise SDRError(-1, "disparity maps and guide must have the same (F, H, W) shape")
        if dl.device.index != self._device:
            raise SDRError(-1, f"tensors are on cuda:{dl.device.index}, filter on cuda:{self._device}")
        dl, dr, g = dl.contiguous(), dr.contiguous(), g.contiguous()
        f, h, w = dl.shape
        out = torch.empty_like(dl)
        conf = torch.empty((f, h, w), dtype=torch.float32, device=dl.device)
        check(lib().sdr_wls_set_stream(self._h, _cstream(self._device)))
        check(lib().sdr_wls_filter_device(self._h, dl.data_ptr(), dr.data_ptr(), g.data_ptr(), w, h,
                                          w, w * h, f, out.data_ptr(), conf.data_ptr()))
        self._conf = conf[0] if squeeze else conf
        return out[0] if squeeze else out


def createDisparityWLSFilter(matcher_left: StereoSGBM) -> DisparityWLSFilter:
    """cv::ximgproc::createDisparityWLSFilter(matcher_left) for an SGBM matcher: ROI offsets
    (max(0, minD+numD), max(0, -minD), 0, 0), radius ceil(0.5*blockSize); the left matcher is
    switched to disp12MaxDiff=1e6, speckleWindowSize=0, uniquenessRatio=0 as ximgproc does."""
    mp = matcher_left.params()
    p = WlsParams()
    lib().sdr_wls_params_for_sgbm(ctypes.byref(mp), ctypes.byref(p))
    matcher_left.setDisp12MaxDiff(mp.disp12MaxDiff)
    matcher_left.setSpeckleWindowSize(mp.speckleWindowSize)
    matcher_left.setUniquenessRatio(mp.uniquenessRatio)
    return DisparityWLSFilter(p, matcher_left._device)


def createDisparityWLSFilterGeneric(use_confidence: bool, device: int = 0) -> DisparityWLSFilter:
    """cv::ximgproc::createDisparityWLSFilterGeneric: zero offsets, min_disp 0.  Only the
    confidence-based variant (use_confidence=True) is implemented."""
    if not use_confidence:
        raise SDRError(-1, "createDisparityWLSFilterGeneric(false) is not implemented")
    p = WlsParams(8000.0, 1.5, 24, 5, 0.001, 0.25, 3, 0, 0, 0, 0, 0, FGS_THOMAS)
    return DisparityWLSFilter(p, device)


def fastGlobalSmootherFilter(guide, src, lambda_, sigma_color, lambda_attenuation=0.25,
                             num_iter=3, solver=FGS_THOMAS):
    """cv::ximgproc::fastGlobalSmootherFilter on a float32 (H, W) image (or (N, H, W) stack
    sharing one guide) with an 8-bit gray guide.  torch CUDA tensors are filtered on the current
    stream; numpy arrays go through the current CUDA device.  solver: FGS_THOMAS (default:
    ximgproc's sequential elimination, bit for bit) or FGS_PCR (include/sdr/sdr.h)."""
    if torch is None:
        raise SDRError(-6, "fastGlobalSmootherFilter needs torch for device memory")
    host = not _is_cuda(src)
    dev = torch.device("cuda", torch.cuda.current_device()) if host else src.device
    s = torch.as_tensor(np.asarray(src, np.float32) if host else src, device=dev)
    g = torch.as_tensor(np.asarray(guide, np.uint8) if host else guide, device=dev)
    if s.dtype != torch.float32 or g.dtype != torch.uint8:
        raise SDRError(-5, "src must be float32 and guide 8-bit")
    squeeze = s.dim() == 2
    s = (s.unsqueeze(0) if squeeze else s).contiguous().clone()
    g = g.contiguous()
    n, h, w = s.shape
    if tuple(g.shape) != (h, w):
        raise SDRError(-1, "guide and src must have the same (H, W) size")
    check(lib().sdr_fgs_filter_device(g.data_ptr(), w, w, h, float(lambda_), float(sigma_color),
                                      float(lambda_attenuation), int(num_iter), s.data_ptr(), n,
                                      int(solver), _cstream(dev.index)))
    out = s[0] if squeeze else s
    return out.cpu().numpy() if host else out
