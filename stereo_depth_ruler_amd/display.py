"""The reference's display outputs on the HIP engine (csrc/sdr_display.hip):

* ``Display.show_disparity_map`` -- StereoDisparity::show_disparityMap
  (stereo_vision/src/stereo_disparity.cpp:42-73): gamma 0.6 disparity map with the 0.63 EMA
  against the previous frame (``prev_vis``, stereo_disparity.hpp:11)
* ``Display.show_depth_map`` -- StereoDisparity::show_depthMap (stereo_disparity.cpp:83-124):
  TURBO depth map of the Z channel with the 0.9/0.1 range smoothing (function-static doubles in the
  reference) and the 0.63 EMA (``prev_depth_vis``)
* ``Display.overlay`` -- the live loop's JET heat map + addWeighted(0.7, 0.3) over the half-size
  rectified left view (stereo_vision/src/stereo_displayer.cpp:167-173)
* ``depth_coverage`` -- StereoDisplayer::depth_coverage (stereo_displayer.cpp:105-118)

numpy inputs run the host-pointer ABI (synchronous); torch CUDA inputs stay on the device and are
enqueued on the current stream.  Colour tables are 256 BGR triples (``colormap_lut``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SDRError, check, lib
from .sgbm import _cstream, _is_cuda, torch

COLORMAP_JET, COLORMAP_TURBO = 2, 20


def colormap_lut(colormap: int) -> np.ndarray:
    """(256, 3) uint8 BGR table of cv::COLORMAP_JET / COLORMAP_TURBO (published definitions)."""
    out = np.empty((256, 3), np.uint8)
    check(lib().sdr_colormap_lut(int(colormap), out.ctypes.data))
    return out


def _lut_ptr(lut):
    if lut is None:
        return None, None
    a = np.ascontiguousarray(lut, np.uint8)
    if a.size != 768:
        raise SDRError(-1, "a colour table has 256 BGR entries")
    return a, a.ctypes.data


class Display:
    """Owns the EMA history of one StereoDisparity (prev_vis / prev_depth_vis) and, by default,
    its own depth-range state; pass ``zrange`` to share one state between displays, as the
    reference's function-static doubles are shared by every StereoDisparity in the process."""

    def __init__(self, device: int = 0):
        self._device = int(device)
        h = ctypes.c_void_p()
        check(lib().sdr_display_create(self._device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().sdr_display_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(lib().sdr_display_reset(self._h))

    def _stream(self):
        check(lib().sdr_display_set_stream(self._h, _cstream(self._device)))

    def show_disparity_map(self, disparity, num_disparities: int):
        """float disparity (px): numpy (H, W) -> numpy u8, or CUDA (H, W) / (F, H, W) -> CUDA u8."""
        if _is_cuda(disparity):
            d = disparity.contiguous()
            if d.dtype != torch.float32:
                raise SDRError(-5, "disparity must be float32")
            squeeze = d.dim() == 2
            d = d.unsqueeze(0) if squeeze else d
            f, h, w = d.shape
            out = torch.empty((f, h, w), dtype=torch.uint8, device=d.device)
            self._stream()
            check(lib().sdr_show_disparity_map_device(self._h, d.data_ptr(), w, h, w, w * h, f,
                                                      int(num_disparities), out.data_ptr()))
            return out[0] if squeeze else out
        d = np.ascontiguousarray(disparity, np.float32)
        if d.ndim != 2:
            raise SDRError(-1, "disparity must be (H, W)")
        h, w = d.shape
        out = np.empty((h, w), np.uint8)
        check(lib().sdr_show_disparity_map(self._h, d.ctypes.data, w, h, w, int(num_disparities),
                                           out.ctypes.data, w))
        return out

    def show_depth_map(self, depth, zrange=None, lut=None, coverage=False):
        """computeDepth output (H, W, 3) or Z (H, W) -> BGR u8 (H, W, 3); CUDA (F, H, W, 3) too.
        zrange: float64 [zmin, zmax] state (numpy for host input, CUDA tensor for device input),
        updated in place; None = the display's own.  coverage=True also returns depth_coverage."""
        lt, lp = _lut_ptr(lut)
        if _is_cuda(depth):
            x = depth.contiguous()
            if x.dtype != torch.float32:
                raise SDRError(-5, "depth must be float32")
            ch = 3 if (x.dim() >= 3 and x.shape[-1] == 3) else 1
            base = 3 if ch == 3 else 2
            squeeze = x.dim() == base
            x = x.unsqueeze(0) if squeeze else x
            f, h, w = x.shape[:3]
            out = torch.empty((f, h, w, 3), dtype=torch.uint8, device=x.device)
            zp = None
            if zrange is not None:
                if not (_is_cuda(zrange) and zrange.dtype == torch.float64 and zrange.numel() == 2):
                    raise SDRError(-1, "zrange must be a CUDA float64 tensor of 2 values")
                zp = zrange.data_ptr()
            pct = (ctypes.c_double * f)() if coverage else None
            self._stream()
            check(lib().sdr_show_depth_map_device(self._h, x.data_ptr(), w, h, ch, f, zp, lp,
                                                  out.data_ptr(), pct))
            out = out[0] if squeeze else out
            if coverage:
                cov = list(pct)
                return out, (cov[0] if squeeze else cov)
            return out
        x = np.ascontiguousarray(depth, np.float32)
        ch = 1 if x.ndim == 2 else x.shape[2]
        if x.ndim not in (2, 3) or ch not in (1, 3):
            raise SDRError(-5, "depth must be (H, W) or (H, W, 3)")
        if lut is not None:
            raise SDRError(-1, "a custom colour table needs device input")
        h, w = x.shape[:2]
        out = np.empty((h, w, 3), np.uint8)
        zp = None
        if zrange is not None:
            if not (isinstance(zrange, np.ndarray) and zrange.dtype == np.float64 and zrange.size == 2
                    and zrange.flags.c_contiguous):
                raise SDRError(-1, "zrange must be a contiguous float64 numpy array of 2 values")
            zp = zrange.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        pct = ctypes.c_double()
        check(lib().sdr_show_depth_map(self._h, x.ctypes.data, w, h, ch, zp, out.ctypes.data,
                                       ctypes.byref(pct)))
        return (out, pct.value) if coverage else out

    def overlay(self, vis, left_rect_bgr, lut=None, heat=False):
        """applyColorMap(vis, JET) + addWeighted(resize(left_rect, 0.5, INTER_AREA), 0.7, heat, 0.3):
        vis u8 (H, W) [or CUDA (F, H, W)], left_rect_bgr the FULL-size rectified left view
        (2H, 2W, 3).  Returns the overlay (and the heat map if heat=True)."""
        lt, lp = _lut_ptr(lut)
        if _is_cuda(vis):
            v = vis.contiguous()
            squeeze = v.dim() == 2
            v = v.unsqueeze(0) if squeeze else v
            lr = left_rect_bgr.contiguous()
            lr = lr.unsqueeze(0) if lr.dim() == 3 else lr
            f, h, w = v.shape
            if tuple(lr.shape) != (f, 2 * h, 2 * w, 3):
                raise SDRError(-1, "left_rect must be (F, 2H, 2W, 3)")
            ov = torch.empty((f, h, w, 3), dtype=torch.uint8, device=v.device)
            ht = torch.empty_like(ov) if heat else None
            self._stream()
            check(lib().sdr_disparity_overlay_device(self._h, v.data_ptr(), lr.data_ptr(), 2 * w * 3,
                                                     4 * w * h * 3, w, h, f, lp,
                                                     None if ht is None else ht.data_ptr(), ov.data_ptr()))
            if squeeze:
                ov = ov[0]
                ht = None if ht is None else ht[0]
            return (ov, ht) if heat else ov
        if lut is not None:
            raise SDRError(-1, "a custom colour table needs device input")
        v = np.ascontiguousarray(vis, np.uint8)
        lr = np.ascontiguousarray(left_rect_bgr, np.uint8)
        h, w = v.shape
        if lr.shape != (2 * h, 2 * w, 3):
            raise SDRError(-1, "left_rect must be (2H, 2W, 3)")
        ov = np.empty((h, w, 3), np.uint8)
        ht = np.empty((h, w, 3), np.uint8) if heat else None
        check(lib().sdr_disparity_overlay(self._h, v.ctypes.data, lr.ctypes.data, lr.strides[0], w, h,
                                          None if ht is None else ht.ctypes.data, ov.ctypes.data))
        return (ov, ht) if heat else ov

    def depth_coverage(self, depth, col0: int = 80):
        """StereoDisplayer::depth_coverage: percent of Z in [0, 12000] among columns >= col0."""
        host = not _is_cuda(depth)
        x = torch.as_tensor(np.ascontiguousarray(depth, np.float32)).cuda(self._device) if host \
            else depth.contiguous()
        squeeze = x.dim() == 3
        x = x.unsqueeze(0) if squeeze else x
        f, h, w, c = x.shape
        if c != 3 or x.dtype != torch.float32:
            raise SDRError(-5, "depth must be float32 (H, W, 3)")
        pct = (ctypes.c_double * f)()
        self._stream()
        check(lib().sdr_depth_coverage_device(self._h, x.data_ptr(), w, h, f, int(col0), pct))
        return pct[0] if squeeze else list(pct)
