"""The reference's class surface, class StereoDisparity (stereo_vision/include/stereo_disparity.hpp:8-24,
stereo_vision/src/stereo_disparity.cpp), on the HIP engine.

computeDisparity(left, right): BGR 8UC3 full-res rectified pair -> CV_32F half-res disparity (px):
cvtColor(BGR2GRAY) -> resize(0.5, INTER_AREA) -> left SGBM (3WAY, d=80) and right matcher ->
DisparityWLSFilter (lambda 8000, sigma 1.1) -> /16, all on the GPU (sdr_stereo_class_compute).
computeDepth(disparity): reprojectImageTo3D(disparity, Q) (stereo_disparity.cpp:76-80), with the
reference's quirk of a half-res disparity against the full-res Q kept as is.
show_disparityMap / show_depthMap (stereo_disparity.cpp:42-73, 83-124): the display maps with their
EMA state (prev_vis / prev_depth_vis per object; the depth-range smoothing state is shared by all
objects, as the reference's function-static doubles are), on the GPU (csrc/sdr_display.hip).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SDRError, check, lib
from .display import Display
from .sgbm import MODE_SGBM_3WAY, StereoSGBM, _is_cuda, createRightMatcher, reprojectImageTo3D, torch
from .ximgproc import createDisparityWLSFilter


class StereoDisparity:
    # show_depthMap's `static double zmin_smooth = 1000.0, zmax_smooth = 2000.0` (one per process).
    # One state: it lives where the last call ran (the host array, or a float64 tensor on that
    # call's device) and moves with the first call of the other kind, so a process mixing numpy
    # and device inputs smooths one range as the reference does, and device-only callers stay
    # asynchronous.
    _zrange_host = np.array([1000.0, 2000.0])
    _zrange_dev = {}
    _zrange_owner = None  # None: _zrange_host is current; else the device index holding it

    def __init__(self, Q_matrix, device: int = 0):
        self._device = int(device)
        self.Q = np.asarray(Q_matrix, dtype=np.float64).reshape(4, 4).copy()
        # stereo_disparity.cpp:5-9
        self.matcher = StereoSGBM.create(0, 80, 5, 8 * 5 * 5 * 3, 32 * 5 * 5 * 3, 1, 63, 12, 200, 2,
                                         MODE_SGBM_3WAY, device=device)
        self.right_matcher = createRightMatcher(self.matcher)  # :10
        # :11 -- also switches the left matcher to disp12MaxDiff 1e6, speckle 0, uniqueness 0
        self.wls_filter = createDisparityWLSFilter(self.matcher)
        self.wls_filter.setLambda(8000.0)  # :12
        self.wls_filter.setSigmaColor(1.1)  # :13
        self.last_disp_left = None
        self.last_disp_right = None
        self.last_filtered = None
        self.conf_map = None
        self._display = None

    def computeDisparity(self, left, right):
        left = np.ascontiguousarray(left, dtype=np.uint8)
        right = np.ascontiguousarray(right, dtype=np.uint8)
        if left.shape != right.shape or left.ndim != 3 or left.shape[2] != 3:
            raise SDRError(-5, "computeDisparity expects two equal-size BGR (H, W, 3) images")
        h, w, _ = left.shape
        out = np.empty((h // 2, w // 2), np.float32)
        dl = np.empty((h // 2, w // 2), np.int16)
        dr = np.empty((h // 2, w // 2), np.int16)
        fd = np.empty((h // 2, w // 2), np.int16)
        conf = np.empty((h // 2, w // 2), np.float32)
        check(lib().sdr_stereo_class_compute(self.matcher._h, self.right_matcher._h,
                                             self.wls_filter._h, left.ctypes.data,
                                             right.ctypes.data, w, h, w * 3, out.ctypes.data, w // 2,
                                             dl.ctypes.data, dr.ctypes.data, fd.ctypes.data,
                                             conf.ctypes.data))
        self.last_disp_left, self.last_disp_right, self.last_filtered = dl, dr, fd
        self.conf_map = conf  # wls_filter->getConfidenceMap() (:36)
        return out

    def computeDepth(self, disparity):
        return reprojectImageTo3D(disparity, self.Q, False)

    def get_matcher(self) -> StereoSGBM:
        return self.matcher

    def _disp(self) -> Display:
        if self._display is None:
            self._display = Display(self._device)
        return self._display

    def show_disparityMap(self, disparity):
        """stereo_disparity.cpp:42-73 (numDisparities read from the matcher, :43)."""
        return self._disp().show_disparity_map(disparity, self.matcher.getNumDisparities())

    def show_depthMap(self, depth):
        """stereo_disparity.cpp:83-124 on computeDepth's output (or a Z map)."""
        cls = StereoDisparity
        if _is_cuda(depth):
            dev = depth.device.index
            z = cls._zrange_dev.get(dev)
            if z is None:
                z = torch.empty(2, dtype=torch.float64, device=depth.device)
                cls._zrange_dev[dev] = z
            if cls._zrange_owner != dev:
                src = cls._zrange_host if cls._zrange_owner is None else cls._zrange_dev[cls._zrange_owner].cpu().numpy()
                z.copy_(torch.from_numpy(np.array(src, dtype=np.float64)))
                cls._zrange_owner = dev
            return self._disp().show_depth_map(depth, zrange=z)
        if cls._zrange_owner is not None:
            cls._zrange_host[:] = cls._zrange_dev[cls._zrange_owner].cpu().numpy()
            cls._zrange_owner = None
        return self._disp().show_depth_map(depth, zrange=cls._zrange_host)
