"""Pins the point-cloud emit oracle (oracle/pcl_oracle.c) and checks the
engine's host-side PCD writer (no GPU needed).

PCL is absent from this image and the reference's results/*.pcd are stripped, so parity with PCL
is unpinned.  The restatement is pinned by an independent numpy restatement of convertCVMatToPCL
and pcl::VoxelGrid (float32 sums in point order), by known answers (one voxel -> the mean, colour
means truncated, PCL's int32-overflow passthrough for the reference's 5 mm leaf on a millimetre
cloud) and by the PCD v0.7 binary layout.
"""
import numpy as np
import pytest

from stereo_depth_ruler_amd import synthetic as S


def np_cloud(xyz, bgr):
    h, w, _ = xyz.shape
    x = xyz.reshape(-1, 3)
    fin = np.isfinite(x).all(1)
    out = np.empty((h * w, 4), np.float32)
    out[:, :3] = np.where(fin[:, None], x, np.float32(np.nan))
    rgba = np.full(h * w, 0xFF000000, np.uint32)
    if bgr is not None:
        b = bgr.reshape(-1, 3).astype(np.uint32)
        rgba = np.where(fin, rgba | b[:, 2] << 16 | b[:, 1] << 8 | b[:, 0], rgba)
    out.view(np.uint32)[:, 3] = rgba
    return out


def np_voxel(pts, leaf):
    inv = np.float32(1.0) / np.float32(leaf)
    fin = np.isfinite(pts[:, :3]).all(1)
    q = pts[fin]
    if not len(q):
        return np.empty((0, 4), np.float32)
    mn, mx = q[:, :3].min(0), q[:, :3].max(0)
    d = ((mx - mn) * inv).astype(np.int64) + 1
    assert int(d[0]) * int(d[1]) * int(d[2]) <= 2**31 - 1
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(q[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    out = []
    for v in np.unique(idx):
        sel = q[order][idx[order] == v]
        s = np.zeros(7, np.float32)
        for p in sel:
            c = int(p.view(np.uint32)[3])
            s += np.array([p[0], p[1], p[2], (c >> 16) & 255, (c >> 8) & 255, c & 255, c >> 24], np.float32)
        n = np.float32(len(sel))
        m = (s / n).astype(np.float32)
        rec = np.empty(4, np.float32)
        rec[:3] = m[:3]
        rec.view(np.uint32)[3] = (int(m[6]) << 24) | (int(m[3]) << 16) | (int(m[4]) << 8) | int(m[5])
        out.append(rec)
    return np.array(out, np.float32)


def test_cloud_matches_numpy(oracle):
    rng = np.random.default_rng(0)
    xyz = rng.normal(0, 100, (30, 40, 3)).astype(np.float32)
    xyz[3, 4, 0] = np.inf
    xyz[5, 6, 2] = np.nan
    xyz[7, 8, 1] = -np.inf
    bgr = rng.integers(0, 256, (30, 40, 3)).astype(np.uint8)
    for b in (bgr, None):
        got = oracle.xyz_to_cloud(xyz, b)
        ref = np_cloud(xyz, b)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("leaf", [0.5, 2.0, 7.5])
def test_voxel_matches_numpy(oracle, leaf):
    rng = np.random.default_rng(int(leaf * 10))
    xyz = rng.normal(0, 10, (20, 30, 3)).astype(np.float32)
    xyz[rng.random((20, 30)) < 0.1] = np.nan
    pts = oracle.xyz_to_cloud(xyz, rng.integers(0, 256, (20, 30, 3)).astype(np.uint8))
    got, passthrough = oracle.voxel_grid(pts, leaf)
    assert not passthrough
    ref = np_voxel(pts, leaf)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_voxel_known_answers(oracle):
    pts = np.zeros((4, 4), np.float32)
    pts[:, :3] = [[0.1, 0.1, 0.1], [0.2, 0.3, 0.4], [0.4, 0.2, 0.1], [0.3, 0.3, 0.3]]
    pts.view(np.uint32)[:, 3] = [0xFF0A0B0C, 0xFF0A0B0D, 0xFF0A0B0D, 0xFF0A0B0D]
    got, pt = oracle.voxel_grid(pts, 1.0)
    assert not pt and got.shape == (1, 4)
    assert np.allclose(got[0, :3], pts[:, :3].mean(0), rtol=1e-6)
    assert got.view(np.uint32)[0, 3] == 0xFF0A0B0C  # (12+13*3)/4 = 12.75 truncates to 12
    empty, _ = oracle.voxel_grid(np.full((5, 4), np.nan, np.float32), 1.0)
    assert empty.shape == (0, 4)


def wrapped_extent_product(pts, leaf):
    """dx*dy*dz as PCL's compiled int64 code computes it (two's-complement wrap)."""
    q = pts[np.isfinite(pts[:, :3]).all(1)]
    inv = np.float32(1.0) / np.float32(leaf)
    d = [int(np.int64((q[:, c].max() - q[:, c].min()) * inv)) + 1 for c in range(3)]
    p = (d[0] * d[1] * d[2]) & (2**64 - 1)
    return p - 2**64 if p >= 2**63 else p


def test_voxel_reference_leaf_passes_through(oracle):
    """pcd_write.cpp:123-129: a 5 mm leaf on a metre-sized millimetre cloud overflows PCL's int32
    voxel index (dx*dy*dz > INT32_MAX), so VoxelGrid returns the input unchanged."""
    rng = np.random.default_rng(2)
    xyz = rng.uniform(-500, 500, (60, 80, 3)).astype(np.float32)
    pts = oracle.xyz_to_cloud(xyz, rng.integers(0, 256, (60, 80, 3)).astype(np.uint8))
    assert 2**31 - 1 < wrapped_extent_product(pts, 0.005) < 2**63
    got, passthrough = oracle.voxel_grid(pts, 0.005)
    assert passthrough and np.array_equal(got.view(np.uint32), pts.view(np.uint32))


def test_voxel_extent_product_wraps_like_compiled_pcl(oracle):
    """On the reference's own frame shape the extents (handleMissing Z = 10000, far points at
    1/16-px disparity) make dx*dy*dz exceed int64: compiled PCL wraps, and the restatement decides
    passthrough from the wrapped value exactly as that code would."""
    L, R, _ = S.make_pair(96, 224, 64, seed=1)
    d = oracle.sgbm_compute(L, R, oracle.make_params(0, 64, 5, 600, 2400, 1, 63, 12, 200, 2, 2))
    xyz = oracle.reproject(oracle.disp_to_float(d), S.REFERENCE_Q, True)
    pts = oracle.xyz_to_cloud(xyz, np.repeat(L[..., None], 3, 2))
    w = wrapped_extent_product(pts, 0.005)
    got, passthrough = oracle.voxel_grid(pts, 0.005)
    assert passthrough == (w > 2**31 - 1)
    if not passthrough:
        assert 0 < got.shape[0] <= pts.shape[0]


def test_pcd_writer_layout(tmp_path):
    """savePCDFileBinary layout (host code of the engine library; no GPU)."""
    from stereo_depth_ruler_amd.cloud import PointCloud, pcd_header, savePCDFileBinary

    hdr = pcd_header(3, 2)
    assert hdr == (b"# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\n"
                   b"SIZE 4 4 4 4\nTYPE F F F U\nCOUNT 1 1 1 1\nWIDTH 3\nHEIGHT 2\n"
                   b"VIEWPOINT 0 0 0 1 0 0 0\nPOINTS 6\nDATA binary\n")
    pts = np.arange(24, dtype=np.float32).reshape(6, 4)
    savePCDFileBinary(tmp_path / "a.pcd", PointCloud(pts, 3, 2))
    raw = (tmp_path / "a.pcd").read_bytes()
    assert raw[:len(hdr)] == hdr and raw[len(hdr):] == pts.tobytes()
