"""GPU parity for 3-channel input (StereoSGBM::compute on CV_8UC3: calcPixelCostBT's cn == 3
branch sums each channel's Sobel and raw BT costs), bit-exact against the oracle, whose colour
path is itself pinned by the numpy restatement (tests/test_oracle_sgm_volume.py::test_color_*).
The reference always converts to gray first (stereo_disparity.cpp:19-20, pcd_write.cpp:88-89);
this covers the rest of the compute() contract ("1 or 3 ch")."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from stereo_depth_ruler_amd.sgbm import SDRError  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def color_pair(H, W, D, seed):
    """A seeded rectified pair as three channels that differ: the gray pair, an intensity-shifted
    copy, and a second seeded pair (so every channel's costs matter)."""
    L, R, _ = S.make_pair(H, W, D, seed=seed)
    L2, R2, _ = S.make_pair(H, W, D, seed=seed + 100)
    sh = lambda a: np.clip(a.astype(np.int32) + 37, 0, 255).astype(np.uint8)  # noqa: E731
    return np.stack([L, sh(L), L2], -1), np.stack([R, sh(R), R2], -1)


CASES = [
    # (H, W, D, mode, bs, minD, uniq, speckle ws/range, P1, P2, cap, seed)
    (32, 96, 16, 0, 5, 0, 12, (0, 0), 200, 800, 31, 0),
    (40, 140, 48, 1, 3, -8, 10, (20, 2), 100, 900, 15, 1),
    (36, 150, 80, 2, 5, 0, 12, (50, 2), 600, 2400, 31, 2),
    (30, 330, 256, 1, 1, 0, 5, (0, 0), 300, 3000, 63, 3),
    (48, 200, 128, 0, 7, 2, 0, (0, 0), 50, 400, 15, 4),
    (33, 120, 32, 2, 9, 0, 15, (0, 0), 10, 60, 15, 5),
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[-1]}_m{c[3]}_d{c[2]}_bs{c[4]}" for c in CASES])
def test_color_compute_bit_exact(oracle, case):
    H, W, D, mode, bs, minD, uniq, (ws, sr), P1, P2, cap, seed = case
    L, R = color_pair(H, W, D, seed)
    args = (minD, D, bs, P1, P2, 1, cap, uniq, ws, sr, mode)
    ref = oracle.sgbm_compute(L, R, oracle.make_params(*args))
    m = sdr.StereoSGBM.create(*args)
    got = m.compute(L, R)  # host pointers, sdr_sgbm_compute(channels=3)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} px differ"
    # the colour result is not the gray one: the other channels took part
    assert not np.array_equal(ref, oracle.sgbm_compute(L[..., 0], R[..., 0], oracle.make_params(*args)))


def test_color_device_batch_equals_single_frames(oracle):
    """(F, H, W, 3) device batch through sdr_sgbm_compute_device_cn == per-frame host results."""
    args = (0, 64, 5, 600, 2400, 1, 31, 12, 40, 2, 0)
    frames = [color_pair(44, 180, 64, 10 + i) for i in range(3)]
    dev = torch.device("cuda:0")
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).to(dev)
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).to(dev)
    m = sdr.StereoSGBM.create(*args)
    got = m.compute(Lt, Rt).cpu().numpy()
    torch.cuda.synchronize()
    for i, (L, R) in enumerate(frames):
        ref = oracle.sgbm_compute(L, R, oracle.make_params(*args))
        assert np.array_equal(got[i], ref), f"frame {i}: {(got[i] != ref).sum()} px differ"
    one = m.compute(Lt[1], Rt[1]).cpu().numpy()  # (H, W, 3): one colour frame
    assert np.array_equal(one, got[1])


def test_color_equal_channels_and_refusals(oracle):
    """Three equal channels: each pixel cost is 3x the gray one (still bit-exact with the oracle);
    two channels and parameters past the colour int16 domain are refused."""
    L, R, _ = S.make_pair(40, 160, 32, seed=5)
    L3, R3 = np.repeat(L[..., None], 3, -1), np.repeat(R[..., None], 3, -1)
    args = (0, 32, 5, 100, 1200, 1, 15, 10, 0, 0, 0)
    got = sdr.StereoSGBM.create(*args).compute(L3, R3)
    assert np.array_equal(got, oracle.sgbm_compute(L3, R3, oracle.make_params(*args)))
    with pytest.raises(SDRError):
        sdr.StereoSGBM.create(*args).compute(L3[..., :2].copy(), R3[..., :2].copy())
    # gray accepts P2 = 9500 at bs 5 / cap 63 (2*9500 + 189*25 <= 32767), colour (3*189*25) does not
    big = (0, 32, 5, 100, 9500, 1, 63, 10, 0, 0, 0)
    sdr.StereoSGBM.create(*big).compute(L, R)
    with pytest.raises(SDRError):
        sdr.StereoSGBM.create(*big).compute(L3, R3)
