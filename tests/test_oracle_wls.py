"""Pins the WLS/FGS oracle (oracle/wls_oracle.c) -- the class path's post-filter.

opencv_contrib (ximgproc) is absent from this image and the reference has no fixtures for it, so
parity with OpenCV is unpinned (wls_oracle.h).  The restatement is pinned here by an independent
float64 numpy/scipy restatement (tests/numpy_ref.py: banded solves instead of the Thomas sweep),
by the properties the published algorithm has (each 1-D solve of (I + lam*L) u = f conserves the
line sum; lam = 0 is the identity; constants are fixed points), and by known answers.
"""
import numpy as np
import pytest

import numpy_ref as N


def test_lut_matches_formula(oracle):
    lut = oracle.fgs_lut(1.1)
    i = np.arange(65026, dtype=np.float64)
    ref = -np.exp(-np.sqrt(i) / 1.1)
    # float sqrt/divide before exp: relative error ~ x * 2^-24 for exp(-x), x up to 232
    assert np.allclose(lut, ref.astype(np.float32), rtol=5e-5, atol=1e-37)
    assert lut[0] == -1.0


@pytest.mark.parametrize("shape", [(1, 1), (1, 37), (29, 1), (40, 61), (97, 130), (5, 700)])
@pytest.mark.parametrize("lam,sigma", [(8000.0, 1.1), (50.0, 5.0), (0.5, 20.0)])
def test_fgs_matches_float64_restatement(oracle, shape, lam, sigma):
    """Both line solvers against float64 banded solves.  The sequential sweep (ximgproc's) loses
    ~lambda * 2^-24 relative at lambda = 8000 (its elimination denominators cancel); the PCR
    solver carries each diagonal as a row sum of non-negative terms and stays within a few ulp."""
    rng = np.random.default_rng(sum(shape))
    g = rng.integers(0, 256, shape).astype(np.uint8)
    g[: shape[0] // 2] //= 8  # flat and textured halves
    x = (rng.random(shape) * 1000).astype(np.float32)
    ref = N.fgs_filter(g, x, lam, sigma)
    tho = oracle.fgs_filter(g, x, lam, sigma, solver=oracle.FGS_THOMAS)
    assert np.allclose(tho, ref, rtol=2e-4, atol=2e-2 * max(1.0, float(np.abs(ref).max()) * 1e-3))
    pcr = oracle.fgs_filter(g, x, lam, sigma, solver=oracle.FGS_PCR)
    assert np.allclose(pcr, ref, rtol=4e-6, atol=1e-4)


@pytest.mark.parametrize("solver", [0, 1])
def test_fgs_properties(oracle, solver):
    rng = np.random.default_rng(3)
    g = rng.integers(0, 256, (64, 80)).astype(np.uint8)
    x = (rng.random((64, 80)) * 500).astype(np.float32)
    y = oracle.fgs_filter(g, x, 8000.0, 1.1, solver=solver)
    assert abs(float(y.sum(dtype=np.float64)) - float(x.sum(dtype=np.float64))) < 1e-4 * float(x.sum())
    assert np.array_equal(oracle.fgs_filter(g, x, 0.0, 1.1, solver=solver), x)   # lam = 0: identity
    c = np.full((64, 80), 37.0, np.float32)
    # fixed point; f32 sweeps at condition ~lambda lose ~lambda * 2^-24 relative
    assert np.allclose(oracle.fgs_filter(g, c, 8000.0, 1.1, solver=solver), 37.0, rtol=5e-4)
    # edge-aware: a step in the guide keeps a step in the image
    g2 = np.zeros((32, 64), np.uint8)
    g2[:, 32:] = 200
    s = np.where(np.arange(64)[None, :] < 32, 0.0, 100.0).repeat(32, 0).astype(np.float32)
    out = oracle.fgs_filter(g2, s, 8000.0, 1.1, solver=solver)
    assert out[:, :31].max() < 1.0 and out[:, 33:].min() > 99.0


def test_params_for_reference_matcher(oracle):
    # stereo_disparity.cpp:5-13: SGBM(0, 80, bs 5) on the half-size frame
    p = oracle.wls_params_for_sgbm(0, 80, 5, 640, 360, 8000.0, 1.1)
    assert (p.roi_x, p.roi_y, p.roi_w, p.roi_h) == (80, 0, 560, 360)
    assert (p.depth_disc_radius, p.lrc_thresh, p.num_iter) == (3, 24, 3)
    assert p.lambda_ == 8000.0 and abs(p.sigma_color - 1.1) < 1e-12
    q = oracle.wls_params_for_sgbm(-20, 64, 3, 300, 100)
    assert (q.roi_x, q.roi_w) == (44, 300 - 44 - 20) and q.depth_disc_radius == 2


@pytest.mark.parametrize("radius", [1, 3])
def test_disc_map_matches(oracle, radius):
    rng = np.random.default_rng(radius)
    d = (rng.integers(0, 80, (45, 70)) * 16).astype(np.int16)
    d[10:30, 20:50] = 640
    roi = (12, 2, 50, 41)
    got = oracle.wls_disc_map(d, roi, radius)
    ref = N.wls_disc_map(d, roi, radius)
    assert np.allclose(got, ref, atol=2e-3)
    assert (got[:, :12] == 1).all() and (got[:2] == 1).all()


def stereo_pair_disp(rng, h, w, dmax=60, blk=8):
    """Left / right int16 disparity maps of a piecewise-planar scene (right = -left shifted)."""
    base = (rng.integers(5, dmax, (h // blk + 1, w // blk + 1)) * 16)
    dl = np.repeat(np.repeat(base, blk, 0), blk, 1)[:h, :w].astype(np.int16)
    dr = np.full((h, w), -80 * 16, np.int16)
    for y in range(h):
        for x in range(w):
            xr = x - (dl[y, x] >> 4)
            if 0 <= xr < w:
                dr[y, xr] = -dl[y, x]
    dl[rng.random((h, w)) < 0.03] = -16
    return dl, dr


def test_confidence_matches(oracle):
    rng = np.random.default_rng(7)
    dl, dr = stereo_pair_disp(rng, 60, 150)
    p = oracle.wls_params_for_sgbm(0, 64, 5, 150, 60)
    roi = (p.roi_x, p.roi_y, p.roi_w, p.roi_h)
    got = oracle.wls_confidence(dl, dr, p)
    ref = N.wls_confidence(dl, dr, roi, p.depth_disc_radius)
    assert np.allclose(got, ref, atol=0.5)
    assert (got == 0).any() and (got > 254).any()


def test_wls_filter_matches(oracle):
    rng = np.random.default_rng(11)
    h, w = 72, 180
    dl, dr = stereo_pair_disp(rng, h, w, blk=24)
    # guide edges where the depth edges are (objects), mild texture inside
    guide = (rng.integers(0, 4, (h, w)) + 2 * (dl.clip(0) >> 4) + 40).astype(np.uint8)
    p = oracle.wls_params_for_sgbm(0, 64, 5, w, h, 8000.0, 1.1)
    roi = (p.roi_x, p.roi_y, p.roi_w, p.roi_h)
    got = oracle.wls_filter(dl, dr, guide, p)
    ref = N.wls_filter(dl, dr, guide, roi, p.depth_disc_radius, 8000.0, 1.1, 0)
    assert (got[:, :p.roi_x] == -16).all()
    # compare where FGS(confidence) is representable in float32: where it underflows (regions
    # no confident pixel reaches through the guide's edges) the f32 ratio is noise, as in OpenCV
    x, y, rw, rh = roi
    den = N.fgs_filter(guide[y:y + rh, x:x + rw], N.wls_confidence(dl, dr, roi, p.depth_disc_radius)
                       [y:y + rh, x:x + rw], 8000.0, 1.1)
    ok = den >= 1e-3
    assert ok.mean() > 0.9
    diff = np.abs(got[y:y + rh, x:x + rw].astype(np.float64) - ref[y:y + rh, x:x + rw])[ok]
    assert diff.max() <= 1.0 and (diff > 0.5).mean() < 1e-3


def test_wls_known_answers(oracle):
    h, w = 40, 120
    d = 20 * 16
    dl = np.full((h, w), d, np.int16)
    dr = np.full((h, w), -d, np.int16)
    guide = np.random.default_rng(1).integers(0, 256, (h, w)).astype(np.uint8)
    p = oracle.wls_params_for_sgbm(0, 32, 5, w, h, 8000.0, 1.1)
    out = oracle.wls_filter(dl, dr, guide, p)
    assert (out[:, 32:] == d).all() and (out[:, :32] == -16).all()
    # every LR test fails (x - d always inside the right ROI [0, 88)) -> zero confidence ->
    # 0 inside the ROI (divide-by-zero rule)
    out = oracle.wls_filter(np.full((h, w), 32 * 16, np.int16), np.full((h, w), 5 * 16, np.int16), guide, p)
    assert (out[:, 32:] == 0).all()
    # a match leaving the right ROI keeps the discontinuity confidence (x >= 108 for d = 20)
    conf = oracle.wls_confidence(dl, np.full((h, w), 5 * 16, np.int16), p)
    assert (conf[:, 32:108] == 0).all() and (conf[:, 108:] == 255).all()
    # minDisparity < 0: outside value 16*(minD-1), ROI from both offsets
    q = oracle.wls_params_for_sgbm(-8, 32, 5, w, h)
    out = oracle.wls_filter(dl, dr, guide, q)
    assert (out[:, :24] == -144).all() and (out[:, w - 8:] == -144).all()
