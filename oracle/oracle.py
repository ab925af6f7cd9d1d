"""ctypes loader for the CPU restatement (oracle/sgbm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / CPU baseline.  The product (stereo_depth_ruler_amd) never imports it.
Parity against real OpenCV 4.6.0 is UNPINNED (see sgbm_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDR_ORACLE_LIB selects another build of the same sources (the ASan/UBSan one of `make asan`)
_LIB_PATH = os.environ.get("SDR_ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

MODE_SGBM, MODE_HH, MODE_SGBM_3WAY = 0, 1, 2
UNIQ_AUTO, UNIQ_SCALAR, UNIQ_SIMD = 0, 1, 2
STAGE_MEDIAN, STAGE_SPECKLE = 1, 2


class OrcParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "minDisparity", "numDisparities", "blockSize", "P1", "P2", "disp12MaxDiff",
        "preFilterCap", "uniquenessRatio", "speckleWindowSize", "speckleRange", "mode",
        "nstripes", "uniq_rule")]


_SOURCES = ("sgbm_oracle.c", "sgbm_oracle.h", "wls_oracle.c", "wls_oracle.h", "rectify_oracle.c",
            "rectify_oracle.h", "pcl_oracle.c", "pcl_oracle.h", "display_oracle.c", "display_oracle.h",
            "Makefile")


_MAKE_TARGET = "all"
# the builds of the same sources: portable (-march=x86-64-v2, the parity checker; built here and
# shipped) and native (-march=native, the CPU baseline's; built on the host that times it)
BUILDS = {"portable": ("_build", "all", "gcc -O3 -march=x86-64-v2 -ffp-contract=off"),
          "native": ("_build_native", "native", "gcc -O3 -march=native -ffp-contract=off")}


def select_build(kind: str) -> str:
    """Chooses which build lib() loads (before its first call); returns the compile line."""
    global _LIB_PATH, _MAKE_TARGET
    d, target, flags = BUILDS[kind]
    path = os.path.join(_HERE, d, "liboracle.so")
    if _lib is not None and path != _LIB_PATH:
        raise RuntimeError(f"the oracle is already loaded from {_LIB_PATH}")
    _LIB_PATH, _MAKE_TARGET = path, target
    return flags


def build(force: bool = False) -> str:
    stale = not os.path.exists(_LIB_PATH) or any(
        os.path.getmtime(os.path.join(_HERE, f)) > os.path.getmtime(_LIB_PATH) for f in _SOURCES)
    if force or stale:
        subprocess.check_call(["make", "-s", "-C", _HERE, _MAKE_TARGET])
    return _LIB_PATH


class WlsParams(ctypes.Structure):
    """orc_wls_params (wls_oracle.h)."""
    _fields_ = [("lambda_", ctypes.c_double), ("sigma_color", ctypes.c_double),
                ("lrc_thresh", ctypes.c_int), ("depth_disc_radius", ctypes.c_int),
                ("roll_off", ctypes.c_float), ("lambda_attenuation", ctypes.c_double),
                ("num_iter", ctypes.c_int), ("roi_x", ctypes.c_int), ("roi_y", ctypes.c_int),
                ("roi_w", ctypes.c_int), ("roi_h", ctypes.c_int), ("min_disp", ctypes.c_int),
                ("fgs_solver", ctypes.c_int)]


FGS_PCR, FGS_THOMAS = 0, 1  # orc_wls_params.fgs_solver (wls_oracle.h)


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i16p = ctypes.POINTER(ctypes.c_int16)
        f32p = ctypes.POINTER(ctypes.c_float)
        f64p = ctypes.POINTER(ctypes.c_double)
        sz = ctypes.c_size_t
        ci = ctypes.c_int
        L.orc_sgbm_compute_stages.argtypes = [u8p, u8p, ci, ci, sz, ctypes.POINTER(OrcParams), i16p, sz, ci]
        L.orc_sgbm_compute_stages.restype = ci
        L.orc_cost_volume.argtypes = [u8p, u8p, ci, ci, sz, ctypes.POINTER(OrcParams), i16p]
        L.orc_cost_volume.restype = ci
        L.orc_sgbm_compute_cn.argtypes = [u8p, u8p, ci, ci, sz, ci, ctypes.POINTER(OrcParams), i16p, sz, ci]
        L.orc_sgbm_compute_cn.restype = ci
        L.orc_cost_volume_cn.argtypes = [u8p, u8p, ci, ci, sz, ci, ctypes.POINTER(OrcParams), i16p]
        L.orc_cost_volume_cn.restype = ci
        L.orc_pixel_cost_row.argtypes = [u8p, u8p, ci, ci, sz, ci, ci, ci, ci, i16p]
        L.orc_pixel_cost_row.restype = ci
        L.orc_median3x3_s16.argtypes = [i16p, i16p, ci, ci]
        L.orc_filter_speckles_s16.argtypes = [i16p, ci, ci, ci, ci, ci]
        L.orc_reproject_f32.argtypes = [f32p, ci, ci, f64p, ci, f32p]
        L.orc_bgr2gray.argtypes = [u8p, ci, ci, sz, u8p]
        L.orc_resize_area_half.argtypes = [u8p, ci, ci, sz, u8p]
        L.orc_disp_to_float.argtypes = [i16p, ci, f32p]
        wp = ctypes.POINTER(WlsParams)
        L.orc_wls_params_for_sgbm.argtypes = [ci, ci, ci, ci, ci, wp]
        L.orc_fgs_lut.argtypes = [ctypes.c_double, f32p]
        L.orc_wls_disc_map.argtypes = [i16p, ci, ci, ci, ci, ci, ci, ci, ctypes.c_float, f32p]
        L.orc_wls_confidence.argtypes = [i16p, i16p, ci, ci, wp, f32p]
        L.orc_fgs_filter_f32_ex.argtypes = [u8p, sz, ci, ci, ctypes.c_double, ctypes.c_double,
                                             ctypes.c_double, ci, ci, f32p]
        L.orc_fgs_filter_f32.argtypes = [u8p, sz, ci, ci, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ci, f32p]
        L.orc_wls_filter.argtypes = [i16p, i16p, u8p, sz, ci, ci, wp, i16p, f32p]
        u16p = ctypes.POINTER(ctypes.c_uint16)
        L.orc_rectify_inv_matrix.argtypes = [f64p, f64p, f64p, ci, f64p]
        L.orc_init_undistort_rectify_map.argtypes = [f64p, f64p, ci, f64p, f64p, ci, ci, ci, i16p, u16p]
        L.orc_xyz_to_cloud.argtypes = [f32p, u8p, ci, ci, f32p]
        L.orc_voxel_grid.argtypes = [f32p, ci, ctypes.c_float, ctypes.c_float, ctypes.c_float, f32p,
                                     ctypes.POINTER(ci)]
        L.orc_voxel_grid.restype = ci
        L.orc_remap_bilinear_u8.argtypes = [u8p, ci, ci, sz, ci, i16p, u16p, ci, ci, u8p, sz]
        L.orc_colormap_lut.argtypes = [ci, u8p]
        L.orc_colormap_lut.restype = ci
        L.orc_show_disparity_map.argtypes = [f32p, ci, ci, ci, u8p, u8p]
        L.orc_depth_range_update.argtypes = [f32p, ci, ci, ci, f64p, f32p, f32p]
        L.orc_show_depth_map.argtypes = [f32p, ci, ci, ci, f64p, u8p, u8p, u8p]
        L.orc_apply_colormap.argtypes = [u8p, sz, u8p, u8p]
        L.orc_add_weighted_u8.argtypes = [u8p, ctypes.c_double, u8p, ctypes.c_double, ctypes.c_double, sz, u8p]
        L.orc_resize_area_half_bgr.argtypes = [u8p, ci, ci, sz, u8p]
        L.orc_depth_coverage.argtypes = [f32p, ci, ci, ci]
        L.orc_depth_coverage.restype = ctypes.c_double
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def make_params(minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0,
                preFilterCap=0, uniquenessRatio=0, speckleWindowSize=0, speckleRange=0,
                mode=MODE_SGBM, nstripes=4, uniq_rule=UNIQ_AUTO) -> OrcParams:
    """Argument order and defaults of cv::StereoSGBM::create."""
    return OrcParams(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff, preFilterCap,
                     uniquenessRatio, speckleWindowSize, speckleRange, mode, nstripes, uniq_rule)


def sgbm_compute(left: np.ndarray, right: np.ndarray, params: OrcParams,
                 stages: int = STAGE_MEDIAN | STAGE_SPECKLE) -> np.ndarray:
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    assert left.shape == right.shape and (left.ndim == 2 or (left.ndim == 3 and left.shape[2] == 3))
    h, w = left.shape[:2]
    cn = 1 if left.ndim == 2 else 3
    out = np.empty((h, w), np.int16)
    rc = lib().orc_sgbm_compute_cn(_p(left, ctypes.c_uint8), _p(right, ctypes.c_uint8), w, h, w * cn, cn,
                                   ctypes.byref(params), _p(out, ctypes.c_int16), w, stages)
    if rc != 0:
        raise ValueError(f"orc_sgbm_compute failed: {rc}")
    return out


def cost_volume(left, right, params: OrcParams) -> np.ndarray:
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    h, w = left.shape[:2]
    cn = 1 if left.ndim == 2 else 3
    minD, D = params.minDisparity, params.numDisparities
    w1 = (w + min(minD, 0)) - max(minD + D, 0)
    out = np.empty((h, w1, D), np.int16)
    rc = lib().orc_cost_volume_cn(_p(left, ctypes.c_uint8), _p(right, ctypes.c_uint8), w, h, w * cn, cn,
                                  ctypes.byref(params), _p(out, ctypes.c_int16))
    if rc != 0:
        raise ValueError(f"orc_cost_volume failed: {rc}")
    return out


def pixel_cost_row(left, right, y, minD, numD, preFilterCap) -> np.ndarray:
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    h, w = left.shape
    w1 = (w + min(minD, 0)) - max(minD + numD, 0)
    out = np.empty((w1, numD), np.int16)
    rc = lib().orc_pixel_cost_row(_p(left, ctypes.c_uint8), _p(right, ctypes.c_uint8), w, h, w, y,
                                  minD, numD, preFilterCap, _p(out, ctypes.c_int16))
    if rc != 0:
        raise ValueError(f"orc_pixel_cost_row failed: {rc}")
    return out


def median3x3(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.int16)
    h, w = src.shape
    dst = np.empty_like(src)
    lib().orc_median3x3_s16(_p(src, ctypes.c_int16), _p(dst, ctypes.c_int16), w, h)
    return dst


def filter_speckles(img: np.ndarray, new_val: int, max_size: int, max_diff: int) -> np.ndarray:
    img = np.array(img, dtype=np.int16, copy=True, order="C")
    h, w = img.shape
    lib().orc_filter_speckles_s16(_p(img, ctypes.c_int16), w, h, new_val, max_size, max_diff)
    return img


def reproject(disp_f32: np.ndarray, Q: np.ndarray, handle_missing: bool = False) -> np.ndarray:
    disp_f32 = np.ascontiguousarray(disp_f32, dtype=np.float32)
    Q = np.ascontiguousarray(Q, dtype=np.float64).reshape(16)
    h, w = disp_f32.shape
    out = np.empty((h, w, 3), np.float32)
    lib().orc_reproject_f32(_p(disp_f32, ctypes.c_float), w, h, _p(Q, ctypes.c_double),
                            int(bool(handle_missing)), _p(out, ctypes.c_float))
    return out


def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    h, w, _ = bgr.shape
    out = np.empty((h, w), np.uint8)
    lib().orc_bgr2gray(_p(bgr, ctypes.c_uint8), w, h, w * 3, _p(out, ctypes.c_uint8))
    return out


def resize_area_half(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape
    out = np.empty((h // 2, w // 2), np.uint8)
    lib().orc_resize_area_half(_p(src, ctypes.c_uint8), w, h, w, _p(out, ctypes.c_uint8))
    return out


def disp_to_float(disp: np.ndarray) -> np.ndarray:
    disp = np.ascontiguousarray(disp, dtype=np.int16)
    out = np.empty(disp.shape, np.float32)
    lib().orc_disp_to_float(_p(disp, ctypes.c_int16), disp.size, _p(out, ctypes.c_float))
    return out


# ---- DisparityWLSFilter / FastGlobalSmootherFilter (wls_oracle.c) ----

def wls_params_for_sgbm(minDisparity, numDisparities, blockSize, width, height, lambda_=8000.0,
                        sigma_color=1.5) -> WlsParams:
    p = WlsParams()
    lib().orc_wls_params_for_sgbm(minDisparity, numDisparities, blockSize, width, height, ctypes.byref(p))
    p.lambda_ = lambda_
    p.sigma_color = sigma_color
    return p


def fgs_lut(sigma_color) -> np.ndarray:
    out = np.empty(65026, np.float32)
    lib().orc_fgs_lut(sigma_color, _p(out, ctypes.c_float))
    return out


def wls_disc_map(d, roi, radius, roll_off=0.001):
    d = np.ascontiguousarray(d, np.int16)
    h, w = d.shape
    out = np.empty((h, w), np.float32)
    lib().orc_wls_disc_map(_p(d, ctypes.c_int16), w, h, *roi, radius, roll_off, _p(out, ctypes.c_float))
    return out


def wls_confidence(dl, dr, p: WlsParams):
    dl = np.ascontiguousarray(dl, np.int16)
    dr = np.ascontiguousarray(dr, np.int16)
    h, w = dl.shape
    out = np.empty((h, w), np.float32)
    lib().orc_wls_confidence(_p(dl, ctypes.c_int16), _p(dr, ctypes.c_int16), w, h, ctypes.byref(p),
                             _p(out, ctypes.c_float))
    return out


def fgs_filter(guide, img, lambda_, sigma_color, attenuation=0.25, num_iter=3, solver=FGS_THOMAS):
    """FastGlobalSmootherFilter; solver FGS_THOMAS (ximgproc's sequential sweep, the engine's
    default) or FGS_PCR."""
    guide = np.ascontiguousarray(guide, np.uint8)
    out = np.array(img, dtype=np.float32, copy=True, order="C")
    h, w = out.shape
    lib().orc_fgs_filter_f32_ex(_p(guide, ctypes.c_uint8), guide.strides[0], w, h, lambda_, sigma_color,
                                attenuation, num_iter, int(solver), _p(out, ctypes.c_float))
    return out


def wls_filter(dl, dr, guide, p: WlsParams, return_conf=False):
    dl = np.ascontiguousarray(dl, np.int16)
    dr = np.ascontiguousarray(dr, np.int16)
    guide = np.ascontiguousarray(guide, np.uint8)
    h, w = dl.shape
    out = np.empty((h, w), np.int16)
    conf = np.empty((h, w), np.float32)
    lib().orc_wls_filter(_p(dl, ctypes.c_int16), _p(dr, ctypes.c_int16), _p(guide, ctypes.c_uint8),
                         guide.strides[0], w, h, ctypes.byref(p), _p(out, ctypes.c_int16),
                         _p(conf, ctypes.c_float))
    return (out, conf) if return_conf else out


# ---- initUndistortRectifyMap / remap (rectify_oracle.c) ----

def _f64(a, n):
    a = np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1))
    assert a.size == n, (a.size, n)
    return a


def rectify_inv_matrix(K, R, P):
    P = np.asarray(P, np.float64)
    pc = P.shape[1] if P.ndim == 2 else (4 if P.size == 12 else 3)
    K, R, P = _f64(K, 9), _f64(R, 9), _f64(P, 3 * pc)
    out = np.empty(9, np.float64)
    lib().orc_rectify_inv_matrix(_p(K, ctypes.c_double), _p(R, ctypes.c_double), _p(P, ctypes.c_double),
                                 pc, _p(out, ctypes.c_double))
    return out.reshape(3, 3)


def init_undistort_rectify_map(K, dist, R, P, width, height):
    """cv::initUndistortRectifyMap(K, dist, R, P, (width, height), CV_16SC2) -> (map1, map2)."""
    P = np.asarray(P, np.float64)
    pc = P.shape[1] if P.ndim == 2 else (4 if P.size == 12 else 3)
    K, R, P = _f64(K, 9), _f64(R, 9), _f64(P, 3 * pc)
    d = np.ascontiguousarray(np.asarray(dist, np.float64).reshape(-1))
    m1 = np.empty((height, width, 2), np.int16)
    m2 = np.empty((height, width), np.uint16)
    lib().orc_init_undistort_rectify_map(_p(K, ctypes.c_double), _p(d, ctypes.c_double), d.size,
                                         _p(R, ctypes.c_double), _p(P, ctypes.c_double), pc, width,
                                         height, _p(m1, ctypes.c_int16), _p(m2, ctypes.c_uint16))
    return m1, m2


def remap_bilinear(src, map1, map2):
    """cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0; src (H, W[, 3]) u8."""
    src = np.ascontiguousarray(src, np.uint8)
    cn = 1 if src.ndim == 2 else src.shape[2]
    sh, sw = src.shape[:2]
    dh, dw = map2.shape
    m1 = np.ascontiguousarray(map1, np.int16)
    m2 = np.ascontiguousarray(map2, np.uint16)
    out = np.empty((dh, dw) + (() if cn == 1 else (cn,)), np.uint8)
    lib().orc_remap_bilinear_u8(_p(src, ctypes.c_uint8), sw, sh, src.strides[0], cn,
                                _p(m1, ctypes.c_int16), _p(m2, ctypes.c_uint16), dw, dh,
                                _p(out, ctypes.c_uint8), out.strides[0])
    return out


# ---- convertCVMatToPCL / VoxelGrid (pcl_oracle.c) ----

def xyz_to_cloud(xyz, bgr=None):
    """convertCVMatToPCL(xyz CV_32FC3, left BGR) -> float32 (H*W, 4) {x, y, z, rgba bits}."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    h, w, _ = xyz.shape
    out = np.empty((h * w, 4), np.float32)
    b = None if bgr is None else np.ascontiguousarray(bgr, np.uint8)
    lib().orc_xyz_to_cloud(_p(xyz, ctypes.c_float), None if b is None else _p(b, ctypes.c_uint8), w, h,
                           _p(out, ctypes.c_float))
    return out


def voxel_grid(points, leaf):
    """pcl::VoxelGrid<PointXYZRGB>::filter -> (points (M, 4), passthrough flag)."""
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 4)
    lx, ly, lz = (leaf, leaf, leaf) if np.isscalar(leaf) else leaf
    out = np.empty_like(pts)
    cnt = ctypes.c_int()
    flag = lib().orc_voxel_grid(_p(pts, ctypes.c_float), pts.shape[0], lx, ly, lz, _p(out, ctypes.c_float),
                                ctypes.byref(cnt))
    return out[:cnt.value].copy(), bool(flag)


# ---- display outputs (display_oracle.c) ----

COLORMAP_JET, COLORMAP_TURBO = 2, 20


def colormap_lut(colormap) -> np.ndarray:
    out = np.empty((256, 3), np.uint8)
    if lib().orc_colormap_lut(int(colormap), _p(out, ctypes.c_uint8)) != 0:
        raise ValueError("unknown colormap")
    return out


def show_disparity_map(disp, num_disp, prev=None) -> np.ndarray:
    d = np.ascontiguousarray(disp, np.float32)
    h, w = d.shape
    out = np.empty((h, w), np.uint8)
    pv = None if prev is None else _p(np.ascontiguousarray(prev, np.uint8), ctypes.c_uint8)
    lib().orc_show_disparity_map(_p(d, ctypes.c_float), w, h, int(num_disp), pv, _p(out, ctypes.c_uint8))
    return out


def show_depth_map(xyz, zrange, lut, prev=None) -> np.ndarray:
    """zrange: float64 array [zmin_smooth, zmax_smooth], updated in place."""
    x = np.ascontiguousarray(xyz, np.float32)
    h, w = x.shape[:2]
    ch = 1 if x.ndim == 2 else x.shape[2]
    out = np.empty((h, w, 3), np.uint8)
    lt = np.ascontiguousarray(lut, np.uint8)
    pv = None if prev is None else _p(np.ascontiguousarray(prev, np.uint8), ctypes.c_uint8)
    assert zrange.dtype == np.float64 and zrange.flags.c_contiguous
    lib().orc_show_depth_map(_p(x, ctypes.c_float), w, h, ch, _p(zrange, ctypes.c_double),
                             _p(lt, ctypes.c_uint8), pv, _p(out, ctypes.c_uint8))
    return out


def depth_range_update(xyz, zrange):
    x = np.ascontiguousarray(xyz, np.float32)
    h, w = x.shape[:2]
    ch = 1 if x.ndim == 2 else x.shape[2]
    a, b = ctypes.c_float(), ctypes.c_float()
    lib().orc_depth_range_update(_p(x, ctypes.c_float), w, h, ch, _p(zrange, ctypes.c_double),
                                 ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def apply_colormap(src, lut) -> np.ndarray:
    s = np.ascontiguousarray(src, np.uint8)
    out = np.empty(s.shape + (3,), np.uint8)
    lt = np.ascontiguousarray(lut, np.uint8)
    lib().orc_apply_colormap(_p(s, ctypes.c_uint8), s.size, _p(lt, ctypes.c_uint8), _p(out, ctypes.c_uint8))
    return out


def add_weighted(a, alpha, b, beta, gamma=0.0) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    assert a.shape == b.shape
    out = np.empty_like(a)
    lib().orc_add_weighted_u8(_p(a, ctypes.c_uint8), alpha, _p(b, ctypes.c_uint8), beta, gamma, a.size,
                              _p(out, ctypes.c_uint8))
    return out


def resize_area_half_bgr(src) -> np.ndarray:
    s = np.ascontiguousarray(src, np.uint8)
    h, w, _ = s.shape
    out = np.empty((h // 2, w // 2, 3), np.uint8)
    lib().orc_resize_area_half_bgr(_p(s, ctypes.c_uint8), w, h, s.strides[0], _p(out, ctypes.c_uint8))
    return out


def depth_coverage(xyz, col0=80) -> float:
    x = np.ascontiguousarray(xyz, np.float32)
    h, w, _ = x.shape
    return lib().orc_depth_coverage(_p(x, ctypes.c_float), w, h, int(col0))
