"""GPU parity of the display outputs against oracle/display_oracle.c, bit for
bit: show_disparityMap and show_depthMap with their EMA state across frames (one call per frame and
batched frames), the shared depth-range state, the JET overlay over the half-size rectified view,
and StereoDisplayer::depth_coverage -- references stereo_disparity.cpp:42-73,83-124,
stereo_displayer.cpp:105-118,164-173."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def frames_disp(F, H, W, seed):
    rng = np.random.default_rng(seed)
    d = rng.uniform(-5, 90, (F, H, W)).astype(np.float32)
    d[:, 0, :6] = [np.nan, np.inf, -np.inf, 0.0, 80.0, 1e-3]
    d[:, 1] = -1.0  # WLS's invalid value / 16
    return d


def frames_xyz(F, H, W, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-3000, 12500, (F, H, W, 3)).astype(np.float32)
    x[:, 0, :5, 2] = [np.nan, np.inf, -np.inf, 5e12, 0.0]
    x[1, :, :, 2] = np.nan  # a frame with no valid Z: the 1000/2000 fallback
    return x


def test_show_disparity_map_device_and_host(oracle):
    F, H, W = 4, 45, 170
    d = frames_disp(F, H, W, 0)
    ref, prev = [], None
    for f in range(F):
        prev = oracle.show_disparity_map(d[f], 80, prev)
        ref.append(prev)
    dev = sdr.Display()
    got = dev.show_disparity_map(torch.from_numpy(d).cuda(), 80).cpu().numpy()  # batched: EMA in order
    assert np.array_equal(got, np.stack(ref))
    one = sdr.Display()
    for f in range(F):  # per-frame device calls
        assert np.array_equal(one.show_disparity_map(torch.from_numpy(d[f]).cuda(), 80).cpu().numpy(), ref[f])
    host = sdr.Display()
    for f in range(F):  # host-pointer ABI
        assert np.array_equal(host.show_disparity_map(d[f], 80), ref[f])
    host.reset()  # history forgotten: the next frame is not blended
    assert np.array_equal(host.show_disparity_map(d[2], 80), oracle.show_disparity_map(d[2], 80))
    # a size change also restarts the history (prev_vis.size() != show_disp.size())
    assert np.array_equal(host.show_disparity_map(d[3][:20, :30], 80),
                          oracle.show_disparity_map(d[3][:20, :30], 80))


def test_show_depth_map_device_and_host(oracle):
    F, H, W = 4, 36, 150
    x = frames_xyz(F, H, W, 1)
    turbo = oracle.colormap_lut(oracle.COLORMAP_TURBO)
    zr = np.array([1000.0, 2000.0])
    ref, cov, prev = [], [], None
    for f in range(F):
        prev = oracle.show_depth_map(x[f], zr, turbo, prev)
        ref.append(prev)
        cov.append(oracle.depth_coverage(x[f], 80))
    ref = np.stack(ref)
    d = sdr.Display()
    out, c = d.show_depth_map(torch.from_numpy(x).cuda(), coverage=True)  # batched, own range state
    assert np.array_equal(out.cpu().numpy(), ref)
    assert c == cov
    # per-frame on a shared device range state, channel-2-only input
    zdev = torch.tensor([1000.0, 2000.0], dtype=torch.float64, device="cuda")
    d2 = sdr.Display()
    for f in range(F):
        o = d2.show_depth_map(torch.from_numpy(np.ascontiguousarray(x[f][..., 2])).cuda(), zrange=zdev)
        assert np.array_equal(o.cpu().numpy(), ref[f])
    assert zdev.cpu().numpy().tolist() == zr.tolist()
    # host ABI with a host range state
    zh = np.array([1000.0, 2000.0])
    d3 = sdr.Display()
    for f in range(F):
        o, pct = d3.show_depth_map(x[f], zrange=zh, coverage=True)
        assert np.array_equal(o, ref[f]) and pct == cov[f]
    assert zh.tolist() == zr.tolist()


def test_overlay_and_coverage(oracle):
    F, H, W = 2, 40, 96
    rng = np.random.default_rng(3)
    vis = rng.integers(0, 256, (F, H, W), dtype=np.uint8)
    left = rng.integers(0, 256, (F, 2 * H, 2 * W, 3), dtype=np.uint8)
    jet = oracle.colormap_lut(oracle.COLORMAP_JET)
    d = sdr.Display()
    ov, heat = d.overlay(torch.from_numpy(vis).cuda(), torch.from_numpy(left).cuda(), heat=True)
    for f in range(F):
        h = oracle.apply_colormap(vis[f], jet)
        assert np.array_equal(heat[f].cpu().numpy(), h)
        ref = oracle.add_weighted(oracle.resize_area_half_bgr(left[f]), 0.7, h, 0.3)
        assert np.array_equal(ov[f].cpu().numpy(), ref)
        assert np.array_equal(d.overlay(vis[f], left[f]), ref)  # host ABI
    # a caller-provided colour table (e.g. OpenCV's own) is applied as given
    lut = rng.integers(0, 256, (256, 3), dtype=np.uint8)
    ov2 = d.overlay(torch.from_numpy(vis[0]).cuda(), torch.from_numpy(left[0]).cuda(), lut=lut)
    ref2 = oracle.add_weighted(oracle.resize_area_half_bgr(left[0]), 0.7, oracle.apply_colormap(vis[0], lut), 0.3)
    assert np.array_equal(ov2.cpu().numpy(), ref2)
    xyz = frames_xyz(3, 30, 200, 4)
    got = d.depth_coverage(torch.from_numpy(xyz).cuda())
    assert got == [oracle.depth_coverage(xyz[f], 80) for f in range(3)]
    assert d.depth_coverage(xyz[0], col0=0) == oracle.depth_coverage(xyz[0], 0)


def test_class_show_methods(oracle):
    """StereoDisparity.show_disparityMap / show_depthMap (stereo_disparity.hpp:18-21) on the
    class path's own outputs, two frames; the range state is shared by every instance, as the
    reference's function-static doubles are."""
    from stereo_depth_ruler_amd.stereo_disparity import StereoDisparity

    StereoDisparity._zrange_host[:] = [1000.0, 2000.0]
    StereoDisparity._zrange_owner = None
    Lg, Rg, _ = S.make_pair(360, 640, 80, seed=77)
    bgr_l = np.repeat(Lg[:, :, None], 3, 2)
    bgr_r = np.repeat(Rg[:, :, None], 3, 2)
    sd = StereoDisparity(S.REFERENCE_Q)
    disp = sd.computeDisparity(bgr_l, bgr_r)
    depth = sd.computeDepth(disp)
    turbo = oracle.colormap_lut(oracle.COLORMAP_TURBO)
    zr = np.array([1000.0, 2000.0])
    pv = pd = None
    for _ in range(2):
        vis = sd.show_disparityMap(disp)
        dv = sd.show_depthMap(depth)
        pv = oracle.show_disparity_map(disp, 80, pv)
        pd = oracle.show_depth_map(depth, zr, turbo, pd)
        assert np.array_equal(vis, pv) and np.array_equal(dv, pd)
    other = StereoDisparity(S.REFERENCE_Q)  # fresh EMA history, shared range state
    dv2 = other.show_depthMap(depth)
    prev = oracle.show_depth_map(depth, zr, turbo, None)
    assert np.array_equal(dv2, prev)
    assert StereoDisparity._zrange_host.tolist() == zr.tolist()
    # device and host inputs share the one range state: it follows the calls
    dd = torch.from_numpy(depth).cuda()
    for x in (dd, depth, dd, dd, depth):
        got = other.show_depthMap(x)
        got = got.cpu().numpy() if torch.is_tensor(got) else got
        prev = oracle.show_depth_map(depth, zr, turbo, prev)
        assert np.array_equal(got.reshape(prev.shape), prev)
    assert StereoDisparity._zrange_host.tolist() == zr.tolist()
