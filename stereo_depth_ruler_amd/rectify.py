"""The ingest step in front of the hot path on the HIP engine:

* ``initUndistortRectifyMap(K, dist, R, P, size)`` -> (map1 int16 (H, W, 2), map2 uint16 (H, W)),
  cv::initUndistortRectifyMap(..., CV_16SC2) -- reference stereo_vision/src/stereo_rectifier.cpp:7-11
* ``remap(src, map1, map2)`` -- cv::remap(INTER_LINEAR, BORDER_CONSTANT 0), stereo_rectifier.cpp:39-40
* ``StereoRectifier(config).rectify(left, right)`` -- class StereoRectifier
* ``StereoRectifier.rectify_sbs(frames)`` -- the side-by-side split of stereo_displayer.cpp:155-159
  plus rectification (and, fused, the class path's BGR2GRAY + INTER_AREA 0.5x)

numpy inputs are copied to the device and back; torch CUDA tensors stay on the device and run on
the current stream.  No CPU fallback: a missing libsdr.so raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SDRError, check, lib
from .sgbm import _cstream, _is_cuda, torch


def _f64p(a):
    a = np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _pcols(P):
    P = np.asarray(P, np.float64)
    if P.ndim == 2:
        return P.shape[1]
    return 4 if P.size == 12 else 3


def initUndistortRectifyMap(K, dist, R, P, size, device: int = 0):
    """cv::initUndistortRectifyMap(K, dist, R, P, size=(width, height), CV_16SC2)."""
    w, h = int(size[0]), int(size[1])
    Ka, Kp = _f64p(K)
    Ra, Rp = _f64p(R)
    Pa, Pp = _f64p(P)
    if dist is None:
        da, dp, nd = None, None, 0
    else:
        da, dp = _f64p(dist)
        nd = da.size
    m1 = np.empty((h, w, 2), np.int16)
    m2 = np.empty((h, w), np.uint16)
    check(lib().sdr_init_undistort_rectify_map(Kp, dp, nd, Rp, Pp, _pcols(P), w, h, int(device),
                                               m1.ctypes.data, m2.ctypes.data))
    return m1, m2


def remap(src, map1, map2):
    """cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0 on 8-bit images:
    (H, W) gray, (H, W, 3) BGR, or a batch (F, H, W) / (F, H, W, 3).  torch CUDA inputs stay on
    the device (current stream); numpy inputs go through the current CUDA device."""
    if not _is_cuda(src):
        if torch is None:
            raise SDRError(-6, "remap needs torch for device memory")
        dev = torch.device("cuda", torch.cuda.current_device())
        out = remap(torch.from_numpy(np.ascontiguousarray(src, np.uint8)).to(dev),
                    torch.from_numpy(np.ascontiguousarray(map1, np.int16)).to(dev),
                    torch.from_numpy(np.ascontiguousarray(map2, np.uint16).view(np.int16)).to(dev))
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()
    nd = src.dim()
    bgr = nd == 4 or (nd == 3 and src.shape[-1] == 3)
    batched = nd == 4 or (nd == 3 and not bgr)
    s = (src if batched else src.unsqueeze(0)).contiguous()
    cn = 3 if bgr else 1
    f, sh, sw = s.shape[:3]
    dh, dw = map2.shape
    out = torch.empty((f, dh, dw) + ((3,) if bgr else ()), dtype=torch.uint8, device=s.device)
    check(lib().sdr_remap_bilinear_device(s.data_ptr(), sw, sh, sw * cn, sw * sh * cn, cn,
                                          map1.contiguous().data_ptr(), map2.contiguous().data_ptr(),
                                          dw, dh, out.data_ptr(), dw * cn, dw * dh * cn, f,
                                          _cstream(s.device.index)))
    return out if batched else out[0]


class StereoRectifier:
    """class StereoRectifier (reference stereo_vision/include/stereo_rectifier.hpp)."""

    def __init__(self, config, device: int = 0):
        w, h = config.imageSize
        self.W, self.H, self._device = int(w), int(h), int(device)
        args = []
        for K, D, Rr, P in ((config.cameraMatrixLeft, config.distCoeffsLeft, config.R1, config.P1),
                            (config.cameraMatrixRight, config.distCoeffsRight, config.R2, config.P2)):
            Ka, Kp = _f64p(K)
            Ra, Rp = _f64p(Rr)
            Pa, Pp = _f64p(P)
            da, dp = _f64p(D) if D is not None else (None, None)
            args.append((Ka, Kp, da, dp, 0 if da is None else da.size, Ra, Rp, Pa, Pp))
        self._keep = args
        pc = _pcols(config.P1)
        (_, Kl, _, dl, nl, _, R1, _, P1), (_, Kr, _, dr, nr, _, R2, _, P2) = args
        h_ = ctypes.c_void_p()
        check(lib().sdr_rectifier_create(Kl, dl, nl, R1, P1, Kr, dr, nr, R2, P2, pc, self.W, self.H,
                                         self._device, ctypes.byref(h_)))
        self._h = h_

    def close(self):
        if getattr(self, "_h", None):
            lib().sdr_rectifier_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def maps(self, which: int):
        m1 = np.empty((self.H, self.W, 2), np.int16)
        m2 = np.empty((self.H, self.W), np.uint16)
        check(lib().sdr_rectifier_get_maps(self._h, int(which), m1.ctypes.data, m2.ctypes.data))
        return m1, m2

    def _dev(self):
        return torch.device("cuda", self._device)

    def rectify(self, left, right):
        """StereoRectifier::rectify: (H, W, 3) or (H, W) 8-bit pair -> rectified pair."""
        host = not _is_cuda(left)
        L = torch.as_tensor(np.ascontiguousarray(left, np.uint8)).to(self._dev()) if host else left.contiguous()
        R = torch.as_tensor(np.ascontiguousarray(right, np.uint8)).to(self._dev()) if host else right.contiguous()
        if tuple(L.shape[:2]) != (self.H, self.W) or L.shape != R.shape:
            raise SDRError(-1, f"rectify expects two {self.W}x{self.H} images")
        cn = 3 if L.dim() == 3 else 1
        lo, ro = torch.empty_like(L), torch.empty_like(R)
        check(lib().sdr_rectifier_set_stream(self._h, _cstream(self._device)))
        check(lib().sdr_rectify_device(self._h, L.data_ptr(), R.data_ptr(), self.W * cn,
                                       self.W * self.H * cn, cn, 1, lo.data_ptr(), ro.data_ptr(),
                                       self.W * cn, self.W * self.H * cn))
        if host:
            torch.cuda.synchronize(self._dev())
            return lo.cpu().numpy(), ro.cpu().numpy()
        return lo, ro

    def rectify_sbs(self, sbs, bgr=True, small=True):
        """Side-by-side BGR frames (H, 2W, 3) or (F, H, 2W, 3) -> dict with 'left'/'right'
        rectified BGR (if bgr) and 'small_left'/'small_right' half-size gray (if small)."""
        host = not _is_cuda(sbs)
        s = torch.as_tensor(np.ascontiguousarray(sbs, np.uint8)).to(self._dev()) if host else sbs.contiguous()
        squeeze = s.dim() == 3
        if squeeze:
            s = s.unsqueeze(0)
        f, h, w2x, c = s.shape
        if h != self.H or w2x != 2 * self.W or c != 3:
            raise SDRError(-1, f"expected side-by-side BGR frames of {2 * self.W}x{self.H}")
        out = {}
        if bgr:
            out["left"] = torch.empty((f, h, self.W, 3), dtype=torch.uint8, device=s.device)
            out["right"] = torch.empty_like(out["left"])
        if small:
            out["small_left"] = torch.empty((f, h // 2, self.W // 2), dtype=torch.uint8, device=s.device)
            out["small_right"] = torch.empty_like(out["small_left"])
        ptr = lambda k: out[k].data_ptr() if k in out else None  # noqa: E731
        check(lib().sdr_rectifier_set_stream(self._h, _cstream(self._device)))
        check(lib().sdr_rectify_sbs_device(self._h, s.data_ptr(), w2x * 3, w2x * 3 * h, f, ptr("left"),
                                           ptr("right"), ptr("small_left"), ptr("small_right")))
        if squeeze:
            out = {k: v[0] for k, v in out.items()}
        if host:
            torch.cuda.synchronize(self._dev())
            out = {k: v.cpu().numpy() for k, v in out.items()}
        return out
