"""Pins the ingest oracle (oracle/rectify_oracle.c: cv::initUndistortRectifyMap CV_16SC2 +
cv::remap INTER_LINEAR).

OpenCV is absent and the reference holds no rectified fixtures, so parity with OpenCV is unpinned
(rectify_oracle.c states the one known divergence: OpenCV's SIMD map loop may round a map entry
differently by one 1/32-px step).  The restatement is pinned by known answers (the identity
calibration, integer shifts, the half-pixel average, the constant border), by an independent
vectorised float64 restatement (tests/numpy_ref.py) on the reference's own calibration
(config/stereo.yaml, copied to tests/golden/stereo.yaml as data), and by geometric properties of
that calibration.
"""
import os

import numpy as np
import pytest

import numpy_ref as N
from stereo_depth_ruler_amd.config import StereoConfiguration

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def cfg():
    c = StereoConfiguration()
    assert c.loadFromFile(os.path.join(GOLDEN, "stereo.yaml"))
    return c


def test_config_loader(cfg):
    assert cfg.imageSize == (1280, 720)
    assert cfg.P1.shape == (3, 4) and cfg.Q.shape == (4, 4) and cfg.distCoeffsLeft.shape == (1, 5)
    assert cfg.Q[3, 2] == 0.00832541998100415
    assert not StereoConfiguration().loadFromFile("/nonexistent.yaml")


def test_identity_calibration_is_identity_map(oracle):
    K = np.array([[700.0, 0, 320.5], [0, 700.0, 240.25], [0, 0, 1]])
    m1, m2 = oracle.init_undistort_rectify_map(K, np.zeros(5), np.eye(3), K, 640, 480)
    yy, xx = np.mgrid[0:480, 0:640]
    assert np.array_equal(m1[..., 0], xx) and np.array_equal(m1[..., 1], yy)
    assert (m2 == 0).all()


def test_maps_match_float64_restatement(oracle, cfg):
    W, H = cfg.imageSize
    for K, D, R, P in ((cfg.cameraMatrixLeft, cfg.distCoeffsLeft, cfg.R1, cfg.P1),
                       (cfg.cameraMatrixRight, cfg.distCoeffsRight, cfg.R2, cfg.P2)):
        m1, m2 = oracle.init_undistort_rectify_map(K, D, R, P, W, H)
        u, v = N.undistort_rectify_uv(K, D, R, P)(H, W)
        iu = m1[..., 0].astype(np.int64) * 32 + (m2 & 31)
        iv = m1[..., 1].astype(np.int64) * 32 + (m2 >> 5)
        eu, ev = np.rint(u * 32), np.rint(v * 32)
        assert np.abs(iu - eu).max() <= 1 and np.abs(iv - ev).max() <= 1
        assert (iu != eu).mean() < 1e-3 and (iv != ev).mean() < 1e-3
        # the rectified principal point looks at (about) the raw principal point
        cx, cy = P[0, 2], P[1, 2]
        j, i = int(round(cx)), int(round(cy))
        assert abs(m1[i, j, 0] - K[0, 2]) < 15 and abs(m1[i, j, 1] - K[1, 2]) < 15


def test_inverse_matrix(oracle, cfg):
    iR = oracle.rectify_inv_matrix(cfg.cameraMatrixLeft, cfg.R1, cfg.P1)
    ref = np.linalg.inv(cfg.P1[:, :3] @ cfg.R1)
    assert np.allclose(iR, ref, rtol=1e-12, atol=1e-15)


def test_remap_known_answers(oracle):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (40, 60, 3)).astype(np.uint8)
    yy, xx = np.mgrid[0:40, 0:60]
    m1 = np.stack([xx, yy], -1).astype(np.int16)
    m2 = np.zeros((40, 60), np.uint16)
    assert np.array_equal(oracle.remap_bilinear(img, m1, m2), img)  # identity
    sh = m1.copy()
    sh[..., 0] += 3                                                   # integer shift, zero border
    out = oracle.remap_bilinear(img, sh, m2)
    assert np.array_equal(out[:, :57], img[:, 3:]) and (out[:, 57:] == 0).all()
    half = np.full((40, 60), 16, np.uint16)                           # x + 0.5: (a + b + 1) >> 1
    out = oracle.remap_bilinear(img[..., 0], m1, half)
    a = img[:, :-1, 0].astype(np.int32)
    b = img[:, 1:, 0].astype(np.int32)
    assert np.array_equal(out[:, :-1], ((a + b + 1) >> 1).astype(np.uint8))
    assert np.array_equal(out[:, -1], ((img[:, -1, 0].astype(np.int32) + 1) >> 1).astype(np.uint8))


@pytest.mark.parametrize("cn", [1, 3])
def test_remap_matches_numpy(oracle, cfg, cn):
    rng = np.random.default_rng(cn)
    W, H = 160, 96
    img = rng.integers(0, 256, (H, W, 3) if cn == 3 else (H, W)).astype(np.uint8)
    m1 = np.stack([rng.integers(-3, W + 3, (H, W)), rng.integers(-3, H + 3, (H, W))], -1).astype(np.int16)
    m2 = rng.integers(0, 1024, (H, W)).astype(np.uint16)
    assert np.array_equal(oracle.remap_bilinear(img, m1, m2), N.remap_bilinear(img, m1, m2))
    # with the reference's calibration maps
    Wf, Hf = cfg.imageSize
    mm1, mm2 = oracle.init_undistort_rectify_map(cfg.cameraMatrixLeft, cfg.distCoeffsLeft, cfg.R1,
                                                 cfg.P1, Wf, Hf)
    big = rng.integers(0, 256, (Hf, Wf, 3) if cn == 3 else (Hf, Wf)).astype(np.uint8)
    assert np.array_equal(oracle.remap_bilinear(big, mm1, mm2), N.remap_bilinear(big, mm1, mm2))
