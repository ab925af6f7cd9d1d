"""ctypes binding of the engine's C ABI (include/sdr/sdr.h -> lib/libsdr.so).

There is no CPU fallback: if the HIP library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libsdr.so")

SDR_OK = 0
ERRORS = {
    -1: "SDR_ERR_ARG", -2: "SDR_ERR_NUMDISP", -3: "SDR_ERR_MODE", -4: "SDR_ERR_SIZE",
    -5: "SDR_ERR_TYPE", -6: "SDR_ERR_DEVICE", -7: "SDR_ERR_NOMEM", -8: "SDR_ERR_LIMIT",
}


class SDRError(RuntimeError):
    """Raised where cv::StereoSGBM / reprojectImageTo3D would throw cv::Exception."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class SgbmParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "minDisparity", "numDisparities", "blockSize", "P1", "P2", "disp12MaxDiff",
        "preFilterCap", "uniquenessRatio", "speckleWindowSize", "speckleRange", "mode",
        "nstripes", "uniq_rule")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class WlsParams(ctypes.Structure):
    """sdr_wls_params (include/sdr/sdr.h)."""
    _fields_ = [("lambda_", ctypes.c_double), ("sigma_color", ctypes.c_double),
                ("lrc_thresh", ctypes.c_int), ("depth_discontinuity_radius", ctypes.c_int),
                ("roll_off", ctypes.c_float), ("lambda_attenuation", ctypes.c_double),
                ("num_iter", ctypes.c_int), ("left_offset", ctypes.c_int),
                ("right_offset", ctypes.c_int), ("top_offset", ctypes.c_int),
                ("bottom_offset", ctypes.c_int), ("min_disp", ctypes.c_int),
                ("fgs_solver", ctypes.c_int)]


FGS_PCR, FGS_THOMAS = 0, 1  # SDR_FGS_* (sdr_wls_params.fgs_solver)


_lib = None
_path = LIB_PATH


def use_library(path: str) -> None:
    """Scripts only (experiment A/B, scripts/kbench.py): load `path` instead of lib/libsdr.so.
    Must be called before the first use of the engine."""
    global _path
    if _lib is not None:
        raise RuntimeError("the engine library is already loaded")
    _path = os.path.abspath(path)

# (name, restype, argtypes) for every function declared in include/sdr/sdr.h
_c = ctypes
_vp = _c.c_void_p
_sz = _c.c_size_t
_i = _c.c_int
_PP = _c.POINTER(SgbmParams)
SIGNATURES = [
    ("sdr_sgbm_params_default", None, [_PP]),
    ("sdr_right_matcher_params", None, [_PP, _PP]),
    ("sdr_sgbm_create", _i, [_PP, _i, _c.POINTER(_vp)]),
    ("sdr_sgbm_destroy", _i, [_vp]),
    ("sdr_sgbm_set_params", _i, [_vp, _PP]),
    ("sdr_sgbm_get_params", _i, [_vp, _PP]),
    ("sdr_sgbm_set_stream", _i, [_vp, _vp]),
    ("sdr_sgbm_set_stream_ex", _i, [_vp, _vp, _i]),
    ("sdr_sgbm_reset_stream", _i, [_vp]),
    ("sdr_sgbm_get_stream", _vp, [_vp]),
    ("sdr_sgbm_compute", _i, [_vp, _vp, _vp, _i, _i, _i, _sz, _vp, _sz]),
    ("sdr_sgbm_compute_device", _i, [_vp, _vp, _vp, _i, _i, _sz, _sz, _i, _vp, _sz, _sz]),
    ("sdr_sgbm_compute_device_cn", _i, [_vp, _vp, _vp, _i, _i, _i, _sz, _sz, _i, _vp, _sz, _sz]),
    ("sdr_host_alloc", _i, [_sz, _c.POINTER(_c.c_void_p)]),
    ("sdr_host_free", _i, [_vp]),
    ("sdr_sgbm_compute_reproject", _i,
     [_vp, _vp, _vp, _i, _i, _sz, _vp, _sz, _c.POINTER(_c.c_double), _i, _vp, _sz]),
    ("sdr_sgbm_compute_reproject_device", _i,
     [_vp, _vp, _vp, _i, _i, _sz, _sz, _i, _vp, _c.POINTER(_c.c_double), _i, _vp]),
    ("sdr_reproject", _i, [_vp, _i, _i, _sz, _c.POINTER(_c.c_double), _i, _vp, _sz]),
    ("sdr_reproject_device", _i, [_vp, _i, _i, _sz, _c.POINTER(_c.c_double), _i, _vp, _sz, _i, _vp]),
    ("sdr_disp16_reproject_device", _i,
     [_vp, _i, _i, _sz, _c.POINTER(_c.c_double), _i, _vp, _sz, _i, _vp]),
    ("sdr_disp16_to_float_device", _i, [_vp, _vp, _sz, _vp]),
    ("sdr_filter_speckles_device", _i, [_vp, _i, _i, _i, _i, _i, _i, _vp]),
    ("sdr_bgr2gray_device", _i, [_vp, _i, _i, _sz, _vp, _sz, _i, _vp]),
    ("sdr_resize_area_half_device", _i, [_vp, _i, _i, _sz, _vp, _sz, _i, _vp]),
    ("sdr_stereo_class_compute", _i,
     [_vp, _vp, _vp, _vp, _vp, _i, _i, _sz, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("sdr_wls_params_for_sgbm", None, [_PP, _c.POINTER(WlsParams)]),
    ("sdr_wls_create", _i, [_c.POINTER(WlsParams), _i, _c.POINTER(_vp)]),
    ("sdr_wls_destroy", _i, [_vp]),
    ("sdr_wls_set_params", _i, [_vp, _c.POINTER(WlsParams)]),
    ("sdr_wls_get_params", _i, [_vp, _c.POINTER(WlsParams)]),
    ("sdr_wls_set_stream", _i, [_vp, _vp]),
    ("sdr_wls_get_stream", _vp, [_vp]),
    ("sdr_wls_reset_stream", _i, [_vp]),
    ("sdr_rectifier_reset_stream", _i, [_vp]),
    ("sdr_wls_get_roi", _i, [_vp, _i, _i, _c.POINTER(_c.c_int)]),
    ("sdr_wls_filter_device", _i, [_vp, _vp, _vp, _vp, _i, _i, _sz, _sz, _i, _vp, _vp]),
    ("sdr_wls_filter", _i, [_vp, _vp, _vp, _vp, _i, _i, _sz, _vp, _vp]),
    ("sdr_init_undistort_rectify_map", _i,
     [_c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _i, _c.POINTER(_c.c_double),
      _c.POINTER(_c.c_double), _i, _i, _i, _i, _vp, _vp]),
    ("sdr_remap_bilinear_device", _i, [_vp, _i, _i, _sz, _sz, _i, _vp, _vp, _i, _i, _vp, _sz, _sz, _i, _vp]),
    ("sdr_rectifier_create", _i,
     [_c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _i, _c.POINTER(_c.c_double),
      _c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _i,
      _c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _i, _i, _i, _i, _c.POINTER(_vp)]),
    ("sdr_rectifier_destroy", _i, [_vp]),
    ("sdr_rectifier_set_stream", _i, [_vp, _vp]),
    ("sdr_rectifier_get_maps", _i, [_vp, _i, _vp, _vp]),
    ("sdr_rectify_device", _i, [_vp, _vp, _vp, _sz, _sz, _i, _i, _vp, _vp, _sz, _sz]),
    ("sdr_rectify_sbs_device", _i, [_vp, _vp, _sz, _sz, _i, _vp, _vp, _vp, _vp]),
    ("sdr_stereo_class_compute_device", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    ("sdr_stereo_class_depth_device", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp,
                                           _c.POINTER(_c.c_double), _vp]),
    ("sdr_xyz_to_cloud_device", _i, [_vp, _vp, _sz, _sz, _i, _i, _i, _vp, _vp]),
    ("sdr_voxel_grid_device", _i, [_vp, _i, _c.c_float, _c.c_float, _c.c_float, _vp,
                                   _c.POINTER(_i), _c.POINTER(_i), _vp]),
    ("sdr_pcd_header", _i, [_i, _i, _c.c_char_p, _sz]),
    ("sdr_write_pcd_binary", _i, [_c.c_char_p, _vp, _i, _i]),
    ("sdr_fgs_filter_device", _i, [_vp, _sz, _i, _i, _c.c_double, _c.c_double, _c.c_double, _i,
                                   _vp, _i, _i, _vp]),
    ("sdr_fgs_rcp_selftest", _i, [_i, _c.POINTER(_c.c_uint)]),
    ("sdr_colormap_lut", _i, [_i, _vp]),
    ("sdr_display_create", _i, [_i, _c.POINTER(_vp)]),
    ("sdr_display_destroy", _i, [_vp]),
    ("sdr_display_set_stream", _i, [_vp, _vp]),
    ("sdr_display_reset_stream", _i, [_vp]),
    ("sdr_display_reset", _i, [_vp]),
    ("sdr_show_disparity_map_device", _i, [_vp, _vp, _i, _i, _sz, _sz, _i, _i, _vp]),
    ("sdr_show_depth_map_device", _i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _c.POINTER(_c.c_double)]),
    ("sdr_depth_coverage_device", _i, [_vp, _vp, _i, _i, _i, _i, _c.POINTER(_c.c_double)]),
    ("sdr_disparity_overlay_device", _i, [_vp, _vp, _vp, _sz, _sz, _i, _i, _i, _vp, _vp, _vp]),
    ("sdr_show_disparity_map", _i, [_vp, _vp, _i, _i, _sz, _i, _vp, _sz]),
    ("sdr_show_depth_map", _i, [_vp, _vp, _i, _i, _i, _c.POINTER(_c.c_double), _vp, _c.POINTER(_c.c_double)]),
    ("sdr_disparity_overlay", _i, [_vp, _vp, _vp, _sz, _i, _i, _vp, _vp]),
    ("sdr_depth_coverage", _i, [_vp, _vp, _i, _i, _i, _c.POINTER(_c.c_double)]),
    ("sdr_sgbm_scratch_bytes", _sz, [_PP, _i, _i, _i]),
    ("sdr_sgbm_scratch_bytes_cn", _sz, [_PP, _i, _i, _i, _i]),
    ("sdr_sgbm_enable_timing", _i, [_vp, _i]),
    ("sdr_sgbm_last_timing", _i, [_vp, _c.POINTER(_c.c_float), _c.POINTER(_c.c_float),
                                  _c.POINTER(_c.c_float)]),
    ("sdr_selftest_wave_ops", _i, [_c.POINTER(_c.c_int)]),
    ("sdr_sgbm_debug_stage", _i, [_vp, _i, _vp, _sz]),
    ("sdr_sgbm_kernel_time", _i, [_vp, _i, _i, _c.POINTER(_c.c_float), _c.POINTER(_c.c_int)]),
    ("sdr_sgbm_last_status", _i, [_vp]),
    ("sdr_stream_probe", _i, [_i, _sz, _i, _c.POINTER(_c.c_double)]),
    ("sdr_stream_probe_ex", _i, [_i, _sz, _i, _c.POINTER(_c.c_double)]),
    ("sdr_sgbm_debug_knob", _i, [_vp, _i, _i]),
    ("sdr_build_id", _c.c_char_p, []),
    ("sdr_last_error", _c.c_char_p, []),
    ("sdr_abi_version", _i, []),
]


def lib():
    """Loads lib/libsdr.so (raises if the HIP extension has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_path):
            raise RuntimeError(
                f"HIP engine library missing: {_path}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950).")
        L = ctypes.CDLL(_path)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int):
    if rc != SDR_OK:
        raise SDRError(rc, lib().sdr_last_error().decode(errors="replace"))
    return rc
