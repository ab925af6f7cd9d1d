"""Display outputs without a GPU: the oracle (oracle/display_oracle.c) against
an independent numpy statement of the reference's code (stereo_disparity.cpp:42-124,
stereo_displayer.cpp:105-118,164-173), and the engine's host-side colour tables against the
oracle's.  Parity against OpenCV itself is unpinned (colour tables, pow)."""

import numpy as np

from stereo_depth_ruler_amd import _lib


def cv_round_u8(v):
    v = np.asarray(v, np.float32)
    ok = (v > -2147483648.0) & (v < 2147483648.0)
    r = np.rint(np.where(ok, v, 0)).astype(np.int64)
    return np.where(ok, np.clip(r, 0, 255), 0).astype(np.uint8)


def np_add_weighted(a, alpha, b, beta):
    fa = a.astype(np.float64) * np.float64(np.float32(alpha))  # exact in double
    fb = (b.astype(np.float32) * np.float32(beta)).astype(np.float64)
    return cv_round_u8((fa + fb).astype(np.float32))  # fma: one rounding of a*alpha + fl(b*beta)


def test_colormap_tables_match_oracle(oracle):
    for cmap in (oracle.COLORMAP_JET, oracle.COLORMAP_TURBO):
        lut = np.empty((256, 3), np.uint8)
        assert _lib.lib().sdr_colormap_lut(cmap, lut.ctypes.data) == 0
        assert np.array_equal(lut, oracle.colormap_lut(cmap))
    jet = oracle.colormap_lut(oracle.COLORMAP_JET)
    # classic jet: dark blue -> blue -> cyan -> yellow -> red -> dark red (BGR)
    assert tuple(jet[0]) == (128, 0, 0) and tuple(jet[255]) == (0, 0, 128)
    assert jet[64, 0] == 255 and jet[192, 2] == 255 and jet[128, 1] == 255
    assert _lib.lib().sdr_colormap_lut(7, lut.ctypes.data) != 0


def test_show_disparity_map_vs_numpy(oracle):
    rng = np.random.default_rng(0)
    d = rng.uniform(-10, 100, (37, 53)).astype(np.float32)
    d[0, :5] = [np.nan, np.inf, -np.inf, 0.0, 80.0]
    prev = None
    for k in range(3):
        got = oracle.show_disparity_map(d + k, 80, prev)
        m = np.where(d + k > 0, d + k, 0).astype(np.float32) * np.float32(1.0 / 80)
        with np.errstate(all="ignore"):
            g = np.power(m.astype(np.float64), 0.6).astype(np.float32)
        ref = cv_round_u8(g * np.float32(255.0))
        if prev is not None:
            ref = np_add_weighted(prev, 0.63, ref, np.float32(1.0) - np.float32(0.63))
        assert np.array_equal(got, ref)
        prev = got
    assert got[0, 1] == 0  # +inf: cvRound's integer indefinite, saturated to 0


def test_show_depth_map_vs_numpy(oracle):
    rng = np.random.default_rng(1)
    lut = oracle.colormap_lut(oracle.COLORMAP_TURBO)
    xyz = rng.uniform(-100, 12000, (30, 40, 3)).astype(np.float32)
    xyz[0, :4, 2] = [np.nan, np.inf, 5e12, 0.0]
    zr = np.array([1000.0, 2000.0])
    zr_np = [1000.0, 2000.0]
    prev = None
    for k in range(3):
        z = xyz[..., 2] * np.float32(1 + 0.1 * k)
        frame = xyz.copy()
        frame[..., 2] = z
        got = oracle.show_depth_map(frame, zr, lut, prev)
        v = z[(z > 0) & (z < 10000)]
        lo, hi = (float(v.min()), float(v.max())) if v.size else (0.0, 0.0)
        if not hi > lo:
            lo, hi = 1000.0, 2000.0
        zmin = 0.9 * zr_np[0] + 0.1 * lo  # (1.0 - 0.1) == 0.9 in double
        zmax = 0.9 * zr_np[1] + 0.1 * hi
        zmin = max(0.0, min(zmin, 10000.0))
        zmax = max(zmin + 1.0, min(zmax, 10000.0))
        zr_np = [zmin, zmax]
        a = np.float32(255.0 / (zmax - zmin))
        b = np.float32(-255.0 * zmin / (zmax - zmin))
        t = (z.astype(np.float64) * np.float64(a) + np.float64(b)).astype(np.float32)  # fma
        ref = lut[cv_round_u8(t)]
        if prev is not None:
            ref = np_add_weighted(prev, 0.63, ref, np.float32(1.0) - np.float32(0.63))
        assert np.array_equal(got, ref)
        assert list(zr) == zr_np
        prev = got


def test_depth_range_fallbacks(oracle):
    zr = np.array([1000.0, 2000.0])
    empty = np.full((4, 5, 3), np.nan, np.float32)
    oracle.depth_range_update(empty, zr)
    assert list(zr) == [1000.0, 2000.0]  # no valid Z: the 1000/2000 fallback keeps the state
    one = np.zeros((4, 5, 3), np.float32)
    one[1, 1, 2] = 500.0
    oracle.depth_range_update(one, zr)  # a single valid Z: zmax == zmin -> fallback too
    assert list(zr) == [1000.0, 2000.0]


def test_overlay_and_coverage_vs_numpy(oracle):
    rng = np.random.default_rng(2)
    vis = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    left = rng.integers(0, 256, (40, 60, 3), dtype=np.uint8)
    jet = oracle.colormap_lut(oracle.COLORMAP_JET)
    small = oracle.resize_area_half_bgr(left)
    ref_small = ((left[0::2, 0::2].astype(int) + left[0::2, 1::2] + left[1::2, 0::2] + left[1::2, 1::2] + 2)
                 >> 2).astype(np.uint8)
    assert np.array_equal(small, ref_small)
    heat = oracle.apply_colormap(vis, jet)
    assert np.array_equal(heat, jet[vis])
    assert np.array_equal(oracle.add_weighted(small, 0.7, heat, 0.3), np_add_weighted(small, 0.7, heat, 0.3))
    xyz = rng.uniform(-500, 13000, (25, 100, 3)).astype(np.float32)
    xyz[3, 90, 2] = np.nan
    z = xyz[:, 80:, 2]
    ref = np.count_nonzero((z >= 0) & (z <= 12000)) / (25 * 100) * 100
    assert oracle.depth_coverage(xyz, 80) == ref
