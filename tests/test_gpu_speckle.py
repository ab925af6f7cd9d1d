"""GPU parity of the speckle filter (tile CCL, sdr_post.hip) against the oracle's flood fill.

cv::filterSpeckles is the last stage of StereoSGBM::compute; the GPU
version labels 32x32 tiles locally and merges across tile borders, so these inputs are chosen
to stress exactly that: components snaking through many tiles, sizes on the maxSize boundary,
|diff| == maxDiff joins, newVal holes, ragged frame sizes and batched frames.  Bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import stereo_depth_ruler_amd as sdr  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def gpu_speckle(img, new_val, max_size, max_diff):
    t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.int16)).cuda()
    sdr.filterSpeckles(t, new_val, max_size, max_diff)
    return t.cpu().numpy()


def check(oracle, img, new_val, max_size, max_diff):
    got = gpu_speckle(img, new_val, max_size, max_diff)
    ref = oracle.filter_speckles(img, new_val, max_size, max_diff)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} px differ"
    return ref


def blobs(rng, h, w, cell, levels, noise):
    gh, gw = (h + cell - 1) // cell + 1, (w + cell - 1) // cell + 1
    g = rng.integers(0, levels, (gh, gw)) * 40
    img = np.repeat(np.repeat(g, cell, 0), cell, 1)[:h, :w]
    return (img + rng.integers(-noise, noise + 1, (h, w))).astype(np.int16)


def serpentine(h, w, period):
    """One thin path snaking through the whole frame (crosses every tile border many times)."""
    img = np.full((h, w), 1000, np.int16)
    for y in range(0, h, period):
        img[y, :] = 0
        if (y // period) % 2 == 0:
            img[y:y + period, w - 1] = 0
        else:
            img[y:y + period, 0] = 0
    return img


def spiral(n):
    img = np.full((n, n), 500, np.int16)
    y0, x0, y1, x1 = 0, 0, n - 1, n - 1
    while y0 <= y1 and x0 <= x1:
        img[y0, x0:x1 + 1] = 0
        img[y0:y1 + 1, x1] = 0
        if y1 - 2 >= y0:
            img[y1, x0:x1 + 1] = 0
        if x0 + 2 <= x1:
            img[y0 + 2:y1 + 1, x0] = 0
        y0, x0, y1, x1 = y0 + 2, x0 + 2, y1 - 2, x1 - 2
    return img


@pytest.mark.parametrize("shape", [(1, 1), (1, 200), (200, 1), (33, 65), (64, 64), (97, 250), (360, 640)])
def test_random_blobs(oracle, shape):
    rng = np.random.default_rng(sum(shape))
    img = blobs(rng, *shape, cell=7, levels=6, noise=20)
    img[rng.random(shape) < 0.05] = -16
    for max_size, max_diff in [(50, 32), (200, 16), (1, 0), (10**6, 32)]:
        check(oracle, img, -16, max_size, max_diff)


def test_noise_many_components(oracle):
    rng = np.random.default_rng(1)
    img = rng.integers(-40, 40, (257, 321)).astype(np.int16)
    for max_diff in (0, 5, 20, 40):
        check(oracle, img, -16, 30, max_diff)


def test_serpentine_crosses_all_tiles(oracle):
    img = serpentine(200, 300, 3)
    n = int((img == 0).sum())
    # threshold exactly at the component size: <= maxSize is removed, one less keeps it
    out = check(oracle, img, -16, n, 0)
    assert (out == -16).sum() >= n
    out = check(oracle, img, -16, n - 1, 0)
    assert (out == 0).sum() == n


def test_spiral(oracle):
    img = spiral(161)  # the 500-valued corridor is ONE component spiralling through every tile
    n = int((img == 500).sum())
    out = check(oracle, img, -32, n, 0)
    assert not (out == 500).any()
    out = check(oracle, img, -32, n - 1, 0)
    assert (out == 500).sum() == n


def test_diff_boundary_and_holes(oracle):
    # ramps whose steps equal maxDiff join; one more breaks them; a newVal lattice cuts through
    h, w = 120, 190
    x = np.arange(w)[None, :].repeat(h, 0)
    ramp = (x * 16).astype(np.int16)
    check(oracle, ramp, -16, 150, 16)
    check(oracle, ramp, -16, 150, 15)
    holes = ramp.copy()
    holes[::5, :] = -16
    holes[:, ::7] = -16
    check(oracle, holes, -16, 20, 16)
    check(oracle, np.full((h, w), -16, np.int16), -16, 100, 16)  # all newVal: untouched
    check(oracle, np.zeros((h, w), np.int16), -16, h * w, 0)      # one component == maxSize
    check(oracle, np.zeros((h, w), np.int16), -16, h * w - 1, 0)


def test_batch_frames(oracle):
    rng = np.random.default_rng(5)
    frames = np.stack([blobs(rng, 90, 130, 5, 4, 16) for _ in range(3)])
    t = torch.from_numpy(frames).cuda()
    sdr.filterSpeckles(t, -16, 40, 16)
    got = t.cpu().numpy()
    for i in range(3):
        assert np.array_equal(got[i], oracle.filter_speckles(frames[i], -16, 40, 16)), i


def test_full_size_disparity_like(oracle):
    rng = np.random.default_rng(9)
    img = blobs(rng, 720, 1280, 23, 40, 8)
    img[rng.random(img.shape) < 0.02] = -16
    check(oracle, img, -16, 200, 32)
