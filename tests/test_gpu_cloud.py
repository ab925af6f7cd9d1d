"""GPU parity of the point-cloud emit against oracle/pcl_oracle.c, BIT FOR BIT:
convertCVMatToPCL, pcl::VoxelGrid<PointXYZRGB> (centroids summed in the oracle's point order),
PCL's int32-overflow passthrough, and the whole point_cloud/src/pcd_write.cpp:86-141 pipeline
(split -> gray -> SGBM 3WAY d=80 -> /16 -> reprojectImageTo3D(handleMissing) -> cloud coloured by
the left view -> VoxelGrid(5 mm) -> savePCDFileBinary) as one device pipeline.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from stereo_depth_ruler_amd.cloud import VoxelGrid, convertCVMatToPCL, savePCDFileBinary  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def u32(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_cloud_bit_exact(oracle):
    rng = np.random.default_rng(0)
    xyz = rng.normal(0, 1000, (123, 211, 3)).astype(np.float32)
    xyz[rng.random((123, 211)) < 0.05, 2] = np.inf
    xyz[rng.random((123, 211)) < 0.05, 0] = np.nan
    bgr = rng.integers(0, 256, (123, 211, 3)).astype(np.uint8)
    for b in (bgr, None):
        c = convertCVMatToPCL(xyz, b)
        assert (c.width, c.height) == (211, 123)
        assert np.array_equal(u32(c.points), u32(oracle.xyz_to_cloud(xyz, b)))


@pytest.mark.parametrize("leaf,n", [(0.05, 5000), (1.0, 200000), (7.5, 20000), (0.001, 3000)])
def test_voxel_bit_exact(oracle, leaf, n):
    rng = np.random.default_rng(n)
    pts = np.empty((n, 4), np.float32)
    pts[:, :3] = rng.normal(0, 3, (n, 3))
    pts[rng.random(n) < 0.1, :3] = np.nan
    pts.view(np.uint32)[:, 3] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    vg = VoxelGrid()
    vg.setLeafSize(leaf, leaf, leaf)
    got = vg.filter(sdr.cloud.PointCloud(pts, n, 1))
    ref, passthrough = oracle.voxel_grid(pts, leaf)
    assert vg.passthrough == passthrough
    assert np.array_equal(u32(got.points), u32(ref))


def test_voxel_arena_threads_and_sizes(oracle):
    """The voxel grid's leased scratch arenas (sdr_cloud.hip, ArenaLease): calls of growing and
    shrinking sizes reuse and grow one arena, and two threads on two streams lease one each at
    once; every result bit-exact with the oracle."""
    import threading

    cases = []
    for n, leaf in ((3000, 0.05), (150000, 0.5), (500, 0.05), (60000, 0.2)):
        rng = np.random.default_rng(n)
        pts = np.empty((n, 4), np.float32)
        pts[:, :3] = rng.normal(0, 3, (n, 3))
        pts[rng.random(n) < 0.1, :3] = np.nan
        pts.view(np.uint32)[:, 3] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        ref, passthrough = oracle.voxel_grid(pts, leaf)
        cases.append((pts, leaf, ref, passthrough))
    dev = torch.device("cuda", 0)

    def run(order, out, stream, errors):
        try:
            with torch.cuda.stream(stream):
                for i in order:
                    pts, leaf, _, _ = cases[i]
                    vg = VoxelGrid()
                    vg.setLeafSize(leaf, leaf, leaf)
                    got = vg.filter(sdr.cloud.PointCloud(torch.from_numpy(pts).to(dev), len(pts), 1))
                    out.append((i, got.points.cpu().numpy(), vg.passthrough))
        except Exception as e:  # noqa: BLE001 -- re-raised on the main thread
            errors.append(e)

    errors, seq = [], []
    run([0, 1, 2, 3, 1, 0], seq, torch.cuda.current_stream(dev), errors)
    outs = [[], []]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    threads = [threading.Thread(target=run, args=([0, 1, 2, 3] * 3, outs[k], streams[k], errors)) for k in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert len(seq) == 6 and len(outs[0]) == len(outs[1]) == 12
    for i, got, passthrough in seq + outs[0] + outs[1]:
        assert passthrough == cases[i][3]
        assert np.array_equal(u32(got), u32(cases[i][2])), i


def test_voxel_passthrough_and_empty(oracle):
    rng = np.random.default_rng(3)
    xyz = rng.uniform(-500, 500, (60, 80, 3)).astype(np.float32)
    c = convertCVMatToPCL(xyz, rng.integers(0, 256, (60, 80, 3)).astype(np.uint8))
    vg = VoxelGrid()
    vg.setLeafSize(0.005, 0.005, 0.005)
    out = vg.filter(c)
    assert vg.passthrough and (out.width, out.height) == (80, 60)
    assert np.array_equal(u32(out.points), u32(c.points))
    empty = vg.filter(sdr.cloud.PointCloud(np.full((10, 4), np.nan, np.float32), 10, 1))
    assert empty.points.shape == (0, 4)


@pytest.mark.parametrize("leaf", [0.005, 2.0])
def test_cloud_emit_voxel_stage_behind(leaf):
    """bench.py's C5 loop with several streams: each CloudEmit's frames enqueued with voxel=False
    on its own stream, and its voxel stage (CloudEmit.voxel) run only after the other stream's
    frames are queued -- the same counts, passthrough flags and filtered points as
    enqueue(voxel=True) on one stream."""
    from stereo_depth_ruler_amd.pipeline import CloudEmit

    H, W, F = 120, 200, 2
    dev = torch.device("cuda", 0)
    sbs = torch.from_numpy(np.stack([S.sbs_bgr_color_frame(H, W, 64, seed=900 + i) for i in range(2 * F)])).to(dev)
    args = (0, 64, 5, 600, 2400, 1, 63, 12, 100, 2, sdr.MODE_SGBM_3WAY)

    def result(p):
        torch.cuda.synchronize(dev)
        return [(p.counts[f], p.passthrough[f], p.filtered[f, :p.counts[f]].cpu().numpy()) for f in range(F)]

    one = CloudEmit(W, H, args, F, S.REFERENCE_Q, leaf=leaf)
    want = []
    for b in range(2):
        one.enqueue(sbs[b * F:(b + 1) * F], torch.cuda.current_stream(dev))
        want.append(result(one))
    pipes = [CloudEmit(W, H, args, F, S.REFERENCE_Q, leaf=leaf) for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for b in range(2):
        pipes[b].enqueue(sbs[b * F:(b + 1) * F], streams[b], voxel=False)
    for b in range(2):
        pipes[b].voxel(streams[b])
    for b in range(2):
        for (n0, p0, a0), (n1, p1, a1) in zip(want[b], result(pipes[b])):
            assert (n0, p0) == (n1, p1)
            assert np.array_equal(u32(a0), u32(a1))
    for p in [one] + pipes:
        p.close()


@pytest.mark.parametrize("H,W,seed", [(240, 400, 41), (720, 1280, 100)])
def test_pcd_write_pipeline(oracle, tmp_path, H, W, seed):
    """pcd_write.cpp:86-141 end to end on the device, checked byte for byte against the oracle.
    720x1280 is the reference's own geometry: frame 100 of the 2560x720 SBS
    video split into 1280x720 halves, 3WAY d=80 with the LR check (1) and speckle (200/2) active
    (pcd_write.cpp:102-116) -- four 180-row stripes with their overlap rows, W1 = 1200 matched
    columns -- reprojectImageTo3D(handleMissing), the organised cloud and VoxelGrid(5 mm)."""
    Lg, Rg, _ = S.make_pair(H, W, 80, seed=seed)
    rng = np.random.default_rng(seed)
    left = np.stack([Lg, np.roll(Lg, 1, 1), rng.integers(0, 256, Lg.shape)], -1).astype(np.uint8)
    right = np.stack([Rg, np.roll(Rg, 1, 1), rng.integers(0, 256, Rg.shape)], -1).astype(np.uint8)
    dev = torch.device("cuda", 0)
    args = (0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, sdr.MODE_SGBM_3WAY)
    m = sdr.StereoSGBM.create(*args)
    gl = sdr.cvt_bgr2gray(torch.from_numpy(left).to(dev))
    gr = sdr.cvt_bgr2gray(torch.from_numpy(right).to(dev))
    disp, xyz = m.compute_reproject(gl, gr, S.REFERENCE_Q, True)
    cloud = convertCVMatToPCL(xyz[0], torch.from_numpy(left).to(dev))
    vg = VoxelGrid()
    vg.setLeafSize(0.005, 0.005, 0.005)
    filt = vg.filter(cloud)
    savePCDFileBinary(tmp_path / "frame_00100.pcd", filt)
    # oracle chain
    og_l, og_r = oracle.bgr2gray(left), oracle.bgr2gray(right)
    d = oracle.sgbm_compute(og_l, og_r, oracle.make_params(*args))
    got = disp[0].cpu().numpy()
    assert np.array_equal(got, d), f"{(got != d).sum()} px differ"
    # the LR check and the speckle filter are both active: each changes the map
    for off in ((0, 80, 5, 600, 2400, 1000000, 63, 12, 200, 2, sdr.MODE_SGBM_3WAY),
                (0, 80, 5, 600, 2400, 1, 63, 12, 0, 2, sdr.MODE_SGBM_3WAY)):
        assert not np.array_equal(oracle.sgbm_compute(og_l, og_r, oracle.make_params(*off)), d)
    oxyz = oracle.reproject(oracle.disp_to_float(d), S.REFERENCE_Q, True)
    assert np.array_equal(u32(xyz[0].cpu().numpy()), u32(oxyz))
    opts = oracle.xyz_to_cloud(oxyz, left)
    ref, passthrough = oracle.voxel_grid(opts, 0.005)
    assert vg.passthrough == passthrough
    assert np.array_equal(u32(filt.points.cpu().numpy()), u32(ref))
    w, h = (W, H) if passthrough else (ref.shape[0], 1)
    raw = (tmp_path / "frame_00100.pcd").read_bytes()
    hdr = sdr.cloud.pcd_header(w, h)
    assert raw == hdr + ref.tobytes()
