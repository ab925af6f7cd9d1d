"""C-ABI boundary checks that need no GPU: the HIP library loads, exports every function that
include/sdr/sdr.h declares, the ctypes table matches the header, and host-only entry points
(parameter defaults, createRightMatcher) behave like their OpenCV counterparts."""
import ctypes
import os
import re

import pytest

from stereo_depth_ruler_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sdr", "sdr.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(sdr_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_loads():
    assert _lib.lib().sdr_abi_version() == 4


def test_every_declared_symbol_exported():
    names = declared_functions()
    assert len(names) >= 20, names
    dll = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(dll, n), f"{n} declared in sdr.h but not exported"


def test_ctypes_table_matches_header():
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == declared_functions()


def test_params_struct_layout():
    # 13 ints, in cv::StereoSGBM::create order, then nstripes / uniq_rule
    assert ctypes.sizeof(_lib.SgbmParams) == 13 * 4
    assert [f for f, _ in _lib.SgbmParams._fields_][:11] == [
        "minDisparity", "numDisparities", "blockSize", "P1", "P2", "disp12MaxDiff", "preFilterCap",
        "uniquenessRatio", "speckleWindowSize", "speckleRange", "mode"]


def test_params_default_matches_opencv_create_defaults():
    p = _lib.SgbmParams()
    _lib.lib().sdr_sgbm_params_default(ctypes.byref(p))
    assert (p.minDisparity, p.numDisparities, p.blockSize, p.P1, p.P2, p.disp12MaxDiff,
            p.preFilterCap, p.uniquenessRatio, p.speckleWindowSize, p.speckleRange, p.mode) == (
        0, 16, 3, 0, 0, 0, 0, 0, 0, 0, 0)
    assert p.nstripes == 4


def test_right_matcher_params():
    """ximgproc createRightMatcher(StereoSGBM(0,80,5,600,2400,1,63,12,200,2,3WAY))."""
    left = _lib.SgbmParams(0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, 2, 4, 0)
    r = _lib.SgbmParams()
    _lib.lib().sdr_right_matcher_params(ctypes.byref(left), ctypes.byref(r))
    assert (r.minDisparity, r.numDisparities, r.blockSize, r.P1, r.P2) == (-79, 80, 5, 600, 2400)
    assert (r.uniquenessRatio, r.disp12MaxDiff, r.speckleWindowSize, r.mode, r.preFilterCap) == (
        0, 1000000, 0, 2, 63)


def test_scratch_bytes_is_pure_host():
    p = _lib.SgbmParams(0, 128, 5, 600, 2400, 1, 63, 12, 200, 2, 0, 4, 0)
    n = _lib.lib().sdr_sgbm_scratch_bytes(ctypes.byref(p), 1280, 720, 1)
    cells = 720 * 1152 * 128
    assert n >= 2 * cells * 2  # cost volume + path sums, int16
    bad = _lib.SgbmParams(0, 100, 5, 600, 2400, 1, 63, 12, 200, 2, 0, 4, 0)
    assert _lib.lib().sdr_sgbm_scratch_bytes(ctypes.byref(bad), 1280, 720, 1) == 0
    # colour input: three operand sets per image (the L pack and the R pair planes, 36 B/px/channel)
    n3 = _lib.lib().sdr_sgbm_scratch_bytes_cn(ctypes.byref(p), 1280, 720, 3, 1)
    assert n3 - n == 2 * 36 * 1280 * 720
    assert _lib.lib().sdr_sgbm_scratch_bytes_cn(ctypes.byref(p), 1280, 720, 1, 1) == n
    assert _lib.lib().sdr_sgbm_scratch_bytes_cn(ctypes.byref(p), 1280, 720, 2, 1) == 0


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    p = _lib.SgbmParams(0, 16, 3, 0, 0, 0, 0, 0, 0, 0, 0, 4, 0)
    h = ctypes.c_void_p()
    rc = _lib.lib().sdr_sgbm_create(ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == -6 and not h.value
    assert _lib.lib().sdr_last_error()


def test_python_surface_raises_without_gpu():
    import torch

    import stereo_depth_ruler_amd as sdr

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(sdr.SDRError):
        sdr.StereoSGBM.create(0, 16, 3)


def test_null_arguments_rejected():
    L = _lib.lib()
    assert L.sdr_sgbm_compute(None, None, None, 8, 8, 1, 8, None, 8) == -1
    assert L.sdr_reproject(None, 8, 8, 8, None, 0, None, 24) == -1
    assert L.sdr_sgbm_set_params(None, None) == -1


def test_wls_params_for_sgbm_matches_ximgproc(oracle):
    """createDisparityWLSFilter(matcher): ROI offsets, radius, defaults, and the mutation of the
    left matcher (disp12MaxDiff 1e6, speckle 0, uniqueness 0) -- host-only, no GPU."""
    for minD, numD, bs, w, h in ((0, 80, 5, 640, 360), (-20, 64, 3, 300, 100), (5, 32, 7, 200, 50)):
        m = _lib.SgbmParams(minD, numD, bs, 600, 2400, 1, 63, 12, 200, 2, 2, 4, 0)
        p = _lib.WlsParams()
        _lib.lib().sdr_wls_params_for_sgbm(ctypes.byref(m), ctypes.byref(p))
        assert (m.disp12MaxDiff, m.speckleWindowSize, m.uniquenessRatio) == (1000000, 0, 0)
        assert (m.minDisparity, m.numDisparities, m.blockSize, m.P1, m.P2) == (minD, numD, bs, 600, 2400)
        q = oracle.wls_params_for_sgbm(minD, numD, bs, w, h)
        assert (p.left_offset, p.top_offset) == (q.roi_x, q.roi_y)
        assert w - p.left_offset - p.right_offset == q.roi_w and h - p.top_offset - p.bottom_offset == q.roi_h
        assert p.depth_discontinuity_radius == q.depth_disc_radius
        assert (p.lrc_thresh, p.num_iter, p.min_disp) == (q.lrc_thresh, q.num_iter, q.min_disp)
        assert (p.lambda_, p.sigma_color, p.lambda_attenuation) == (q.lambda_, q.sigma_color, q.lambda_attenuation)
        assert abs(p.roll_off - 0.001) < 1e-9


def test_int16_domain_guard_host_only():
    """P2 is bounded by 2*P2 + (2*ftzero+63)*blockSize^2 <= 32767 (OpenCV's SIMD and scalar
    builds disagree past it); checked on the host, before any device work."""
    from test_oracle_sgm_volume import p2_domain_max

    L = _lib.lib()
    for bs, cap, mode in ((5, 63, 0), (11, 63, 1), (1, 15, 2), (7, 127, 0)):
        pmax = p2_domain_max(bs, cap, mode)
        ok = _lib.SgbmParams(0, 64, bs, 10, pmax, 1, cap, 10, 0, 0, mode, 4, 0)
        assert L.sdr_sgbm_scratch_bytes(ctypes.byref(ok), 320, 100, 1) > 0
        bad = _lib.SgbmParams(0, 64, bs, 10, pmax + 1, 1, cap, 10, 0, 0, mode, 4, 0)
        assert L.sdr_sgbm_scratch_bytes(ctypes.byref(bad), 320, 100, 1) == 0
        assert b"int16" in L.sdr_last_error()
    for cap in (128, 255, 1000):  # OpenCV accepts any preFilterCap (its uchar clip table wraps)
        big = _lib.SgbmParams(0, 64, 5, 10, 100, 1, cap, 10, 0, 0, 0, 4, 0)
        assert L.sdr_sgbm_scratch_bytes(ctypes.byref(big), 320, 100, 1) > 0


def test_chain_span_guard_host_only():
    """k_paths addresses a chain with a 32-bit offset: frames whose chain span passes 2 GiB are
    refused (SDR_ERR_SIZE) instead of silently reading zeros."""
    L = _lib.lib()
    p = _lib.SgbmParams(0, 256, 5, 600, 2400, 1, 63, 12, 0, 0, 1, 4, 0)
    assert L.sdr_sgbm_scratch_bytes(ctypes.byref(p), 1920, 1080, 1) > 0  # C5 fits
    assert L.sdr_sgbm_scratch_bytes(ctypes.byref(p), 8192, 1200, 1) == 0
    assert b"2 GiB" in L.sdr_last_error()


def test_build_id_matches_sources():
    """The library in the tree is the build of these sources (build.py source_hash), so the
    prebuilt libsdr.so that travels to the GPU box cannot silently be an older build."""
    from stereo_depth_ruler_amd.build import built_id, source_hash

    assert _lib.lib().sdr_build_id().decode() == source_hash()
    assert built_id() == source_hash()


def test_sweep_status_host_only():
    """sdr_sgbm_last_status / sdr_sgbm_debug_knob reject a null handle without touching a GPU."""
    L = _lib.lib()
    assert L.sdr_sgbm_last_status(None) == -1
    assert L.sdr_sgbm_debug_knob(None, 1, 4) == -1


def test_stream_binding_flags_host_only():
    """torch's default (id 0) and pooled streams (odd ids) bind persistent; an external stream (its
    id is the even, non-zero stream pointer: c10 StreamId) binds transient (sdr.h set_stream_ex).
    Unknown flag bits are refused before any device call."""
    import ctypes

    from stereo_depth_ruler_amd.sgbm import STREAM_PERSISTENT, stream_is_pooled

    assert STREAM_PERSISTENT == 1
    assert stream_is_pooled(0)
    assert stream_is_pooled(1) and stream_is_pooled(0x23) and stream_is_pooled((5 << 5) | 1)
    assert not stream_is_pooled(0x7F3A12345600)
    assert _lib.lib().sdr_sgbm_set_stream_ex(None, None, 0) == -1
    assert _lib.lib().sdr_sgbm_set_stream_ex(ctypes.c_void_p(8), None, 6) == -1
