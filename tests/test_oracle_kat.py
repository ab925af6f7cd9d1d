"""Pins the CPU oracle (oracle/sgbm_oracle.c) before it is trusted as the GPU checker.

Parity against real OpenCV 4.6 is unpinned (OpenCV is absent; the reference ships no fixtures,
SURVEY.md 8c).  The oracle is pinned instead by
  * analytic known answers (reprojection table of SURVEY.md Appendix B computed from the
    reference's config/stereo.yaml Q; integer-shift pairs; flat images),
  * independent vectorised numpy/scipy restatements of each stage (tests/numpy_ref.py),
  * committed golden fixtures (tests/golden/, regression pin of the oracle itself).
"""
import numpy as np
import pytest

from stereo_depth_ruler_amd import synthetic as S

import numpy_ref as NR

Q = S.REFERENCE_Q

# (x, y, d px) -> (X, Y, Z) in mm, float32 bit patterns via repr
APPENDIX_B = [
    (645.44378662109375, 347.0967903137207, 16.0, 0.0, 0.0, 5029.02685546875),
    (0, 0, 1.0, -77526.875, -41691.20703125, 80464.4296875),
    (100, 50, 16.0, -4094.716796875, -2230.343994140625, 5029.02685546875),
    (1279, 719, 128.0, 594.5234985351562, 348.99066162109375, 628.6283569335938),
    (320, 180, 40.5, -965.1944580078125, -495.5721740722656, 1986.7760009765625),
    (600, 300, 0.0625, -87335.0, -90511.7890625, 1287430.875),
]


def test_reproject_appendix_b(oracle):
    disp = np.zeros((720, 1280), np.float32)
    for x, y, d, X, Y, Z in APPENDIX_B:
        if x != int(x):
            continue  # principal point is not on the pixel grid
        disp[int(y), int(x)] = d
    out = oracle.reproject(disp, Q, False)
    for x, y, d, X, Y, Z in APPENDIX_B:
        if x != int(x):
            continue
        got = out[int(y), int(x)]
        assert got[0] == np.float32(X) and got[1] == np.float32(Y) and got[2] == np.float32(Z), (x, y, got)


def test_reproject_principal_point_formula():
    # Q*(cx, cy, 16, 1): X = Y = 0, Z = f/(16/Tx) -- independent of the pixel grid
    h = Q @ np.array([645.44378662109375, 347.0967903137207, 16.0, 1.0])
    assert h[0] == 0.0 and h[1] == 0.0
    assert np.float32(np.float32(h[2]) * (1.0 / h[3])) == np.float32(5029.02685546875)


@pytest.mark.parametrize("hm", [False, True])
def test_reproject_vs_numpy(oracle, hm):
    rng = np.random.default_rng(3)
    d16 = rng.integers(-16, 128 * 16, size=(37, 53)).astype(np.int16)
    disp = d16.astype(np.float32) * np.float32(0.0625)
    got = oracle.reproject(disp, Q, hm)
    ref = NR.reproject(disp, Q, hm)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_disp_to_float_exact(oracle):
    d = np.arange(-32768, 32768, 7, dtype=np.int16)
    assert np.array_equal(oracle.disp_to_float(d), d.astype(np.float64) / 16.0)


@pytest.mark.parametrize("minD,D,cap", [(0, 16, 63), (0, 48, 31), (-20, 32, 63), (5, 16, 15)])
def test_pixel_cost_vs_numpy(oracle, minD, D, cap):
    L, R, _ = S.make_pair(9, 90, 64, seed=11)
    ref = NR.bt_cost_volume_rows(L, R, minD, D, max(cap, 15) | 1)
    for y in range(9):
        got = oracle.pixel_cost_row(L, R, y, minD, D, cap)
        assert np.array_equal(got, ref[y]), y


@pytest.mark.parametrize("mode,bs,minD,D,H", [
    (0, 5, 0, 16, 23), (0, 3, 0, 32, 17), (1, 5, 0, 16, 19), (0, 7, -16, 32, 14), (1, 3, 4, 16, 9),
    (0, 5, 0, 16, 2), (1, 5, 0, 16, 3),
])
def test_cost_volume_vs_numpy(oracle, mode, bs, minD, D, H):
    L, R, _ = S.make_pair(H, 80, 48, seed=2)
    p = oracle.make_params(minD, D, bs, 8, 2400, 1, 63, 10, 0, 0, mode)
    got = oracle.cost_volume(L, R, p)
    ref = NR.cost_volume(L, R, minD, D, bs, 2400, 63, hh=(mode == 1))
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("shift", [3, 9])
def test_integer_shift_known_answer(oracle, mode, shift):
    L, R = S.shifted_pair(40, 120, shift, seed=4)
    p = oracle.make_params(0, 16, 5, 600, 2400, 1, 63, 10, 0, 0, mode)
    d = oracle.sgbm_compute(L, R, p)
    inner = d[4:-4, 24:-4]
    assert np.all(np.abs(inner.astype(int) - 16 * shift) <= 1), np.unique(inner)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_flat_image(oracle, mode):
    """Textureless pair: every candidate ties in the interior, so WTA's first-minimum rule can
    only ever report d = 0 (or reject); unmatched columns are invalid."""
    L = np.full((24, 64), 100, np.uint8)
    p = oracle.make_params(0, 16, 5, 600, 2400, 1, 63, 10, 0, 0, mode)
    d = oracle.sgbm_compute(L, L.copy(), p)
    assert np.all(d[:, :16] == -16)
    assert set(np.unique(d[:, 16:]).tolist()) <= {0, -16}


def test_unmatched_columns_invalid(oracle):
    L, R, _ = S.make_pair(20, 100, 32, seed=1)
    for minD, D in ((0, 32), (-10, 16), (3, 16)):
        p = oracle.make_params(minD, D, 3, 8, 32, 1, 63, 0, 0, 0, 0)
        d = oracle.sgbm_compute(L, R, p, stages=0)
        maxD = minD + D
        inv = (minD - 1) * 16
        assert np.all(d[:, :max(maxD, 0)] == inv)
        assert np.all(d[:, 100 + min(minD, 0):] == inv)


def test_median_vs_scipy(oracle):
    from scipy.ndimage import median_filter

    rng = np.random.default_rng(0)
    a = rng.integers(-200, 3000, size=(31, 47)).astype(np.int16)
    assert np.array_equal(oracle.median3x3(a), median_filter(a, size=3, mode="nearest"))


def test_speckle_vs_bfs(oracle):
    rng = np.random.default_rng(5)
    base = rng.integers(0, 6, size=(40, 50)) * 40
    img = base.astype(np.int16)
    img[rng.random((40, 50)) < 0.15] = -16
    for ms, md in ((5, 32), (20, 40), (0, 32), (3, 0)):
        assert np.array_equal(oracle.filter_speckles(img, -16, ms, md), NR.speckle_filter(img, -16, ms, md))


def test_bgr2gray_formula(oracle):
    rng = np.random.default_rng(1)
    bgr = rng.integers(0, 256, size=(13, 17, 3)).astype(np.uint8)
    b, g, r = (bgr[..., i].astype(np.int64) for i in range(3))
    ref = ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)
    assert np.array_equal(oracle.bgr2gray(bgr), ref)


def test_resize_area_half_formula(oracle):
    rng = np.random.default_rng(2)
    a = rng.integers(0, 256, size=(14, 22)).astype(np.uint8)
    s = a.astype(np.int32)
    ref = ((s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    assert np.array_equal(oracle.resize_area_half(a), ref)


def test_3way_stripes_change_only_overlap(oracle):
    """3WAY output depends on nstripes only through the restarted vertical path."""
    L, R, _ = S.make_pair(64, 120, 32, seed=8)
    outs = [oracle.sgbm_compute(L, R, oracle.make_params(0, 32, 5, 600, 2400, 1, 63, 10, 0, 0, 2, nstripes=n),
                                stages=0) for n in (1, 4)]
    # stripe 0 (rows < 16) sees identical input history
    assert np.array_equal(outs[0][:16], outs[1][:16])


def test_uniqueness_rules_differ_only_at_threshold(oracle):
    L, R, _ = S.make_pair(60, 160, 48, seed=9)
    a = oracle.sgbm_compute(L, R, oracle.make_params(0, 48, 5, 600, 2400, 1, 63, 15, 0, 0, 0,
                                                     uniq_rule=oracle.UNIQ_SCALAR), stages=0)
    b = oracle.sgbm_compute(L, R, oracle.make_params(0, 48, 5, 600, 2400, 1, 63, 15, 0, 0, 0,
                                                     uniq_rule=oracle.UNIQ_SIMD), stages=0)
    # the two forms agree except on exact-threshold ties
    assert (a != b).mean() < 0.01


def test_right_matcher_range(oracle):
    """createRightMatcher: minD = -(0+80)+1 = -79 -> disparities in [-79*16, 0], invalid -1280."""
    L, R, _ = S.make_pair(48, 200, 80, seed=3)
    p = oracle.make_params(-79, 80, 5, 600, 2400, 1000000, 63, 0, 0, 0, 2)
    d = oracle.sgbm_compute(R, L, p)
    valid = d != -80 * 16
    assert valid.mean() > 0.3
    assert d[valid].min() >= -79 * 16 and d[valid].max() <= 0


def test_native_build_matches_portable(oracle, tmp_path):
    """bench.py's cpu_baseline times the oracle built -O3 -march=native; with FP
    contraction off it must compute exactly what the portable checker build computes: SGBM (5-path
    and 3WAY with LR + speckle), the WLS filter and the reprojection, compared bit for bit."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
from stereo_depth_ruler_amd import synthetic as S
O.select_build(sys.argv[3])
L, R, _ = S.make_pair(72, 200, 48, seed=5)
d5 = O.sgbm_compute(L, R, O.make_params(0, 48, 5, 600, 2400, 1, 63, 12, 100, 2, 0))
d3 = O.sgbm_compute(L, R, O.make_params(0, 48, 5, 600, 2400, 1, 63, 12, 100, 2, 2))
dr = O.sgbm_compute(R, L, O.make_params(-47, 48, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2))
q = O.wls_params_for_sgbm(0, 48, 5, 200, 72, 8000.0, 1.1)
w = O.wls_filter(d3, dr, L, q)
x = O.reproject(O.disp_to_float(w), S.REFERENCE_Q, True)
np.savez(sys.argv[2], d5=d5, d3=d3, w=w, x=x.view(np.uint32))
'''
    outs = {}
    for kind in ("portable", "native"):
        f = tmp_path / f"{kind}.npz"
        subprocess.check_call([sys.executable, "-c", script, root, str(f), kind], cwd=root)
        outs[kind] = np.load(f)
    for k in ("d5", "d3", "w", "x"):
        assert np.array_equal(outs["portable"][k], outs["native"][k]), k
