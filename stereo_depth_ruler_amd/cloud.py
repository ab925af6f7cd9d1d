"""Point-cloud emit after the hot path, reference point_cloud/src/pcd_write.cpp:

* ``convertCVMatToPCL(xyz, bgr)``       -> organised PointXYZRGB cloud (:17-51, :119)
* ``VoxelGrid(leaf).filter(cloud)``     -> pcl::VoxelGrid<PointXYZRGB> (:122-130), including PCL's
  int32-overflow passthrough (the reference's 5 mm leaf on millimetre clouds returns the input)
* ``savePCDFileBinary(path, cloud)``    -> pcl::io::savePCDFileBinary (:141)

A cloud is a float32 array/tensor (N, 4) {x, y, z, rgba bits} (16-byte PointXYZRGB records) with an
organised shape (width, height) carried alongside.  Device work runs on the HIP engine.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SDRError, check, lib
from .sgbm import _cstream, _is_cuda, torch


class PointCloud:
    """pcl::PointCloud<PointXYZRGB>: points (N, 4) float32 + width/height (height 1 = unorganised)."""

    def __init__(self, points, width, height, is_dense=False):
        self.points, self.width, self.height, self.is_dense = points, int(width), int(height), is_dense

    def size(self):
        return self.width * self.height

    def rgba(self):
        p = self.points
        return p.view(torch.int32)[:, 3] if _is_cuda(p) else np.asarray(p).view(np.uint32)[:, 3]


def convertCVMatToPCL(xyz, bgr=None) -> PointCloud:
    """xyz float32 (H, W, 3) (+ BGR uint8 (H, W, 3)) -> organised cloud; non-finite -> NaN."""
    host = not _is_cuda(xyz)
    dev = torch.device("cuda", torch.cuda.current_device()) if host else xyz.device
    x = torch.as_tensor(np.ascontiguousarray(xyz, np.float32)).to(dev) if host else xyz.contiguous()
    if x.dim() != 3 or x.shape[2] != 3 or x.dtype != torch.float32:
        raise SDRError(-5, "pointCloud must be CV_32FC3 (H, W, 3) float32")
    h, w, _ = x.shape
    b = None
    if bgr is not None:
        b = torch.as_tensor(np.ascontiguousarray(bgr, np.uint8)).to(dev) if host else bgr.contiguous()
        if tuple(b.shape) != (h, w, 3):
            b = None  # hasColor: colour only when the image has the cloud's size
    out = torch.empty((h * w, 4), dtype=torch.float32, device=dev)
    check(lib().sdr_xyz_to_cloud_device(x.data_ptr(), None if b is None else b.data_ptr(), 0, 0, w, h,
                                        1, out.data_ptr(), _cstream(dev.index)))
    if host:
        torch.cuda.synchronize(dev)
        out = out.cpu().numpy()
    return PointCloud(out, w, h, False)


class VoxelGrid:
    """pcl::VoxelGrid<PointXYZRGB> (downsample_all_data, min_points_per_voxel 0)."""

    def __init__(self):
        self.leaf = (1.0, 1.0, 1.0)
        self.passthrough = False

    def setLeafSize(self, lx, ly, lz):
        self.leaf = (float(lx), float(ly), float(lz))

    def filter(self, cloud: PointCloud) -> PointCloud:
        host = not _is_cuda(cloud.points)
        dev = torch.device("cuda", torch.cuda.current_device()) if host else cloud.points.device
        p = torch.as_tensor(np.ascontiguousarray(cloud.points, np.float32)).to(dev) if host else cloud.points.contiguous()
        n = p.shape[0]
        out = torch.empty_like(p)
        cnt, pt = ctypes.c_int(), ctypes.c_int()
        check(lib().sdr_voxel_grid_device(p.data_ptr(), n, *self.leaf, out.data_ptr(), ctypes.byref(cnt),
                                          ctypes.byref(pt), _cstream(dev.index)))
        self.passthrough = bool(pt.value)
        out = out[:cnt.value]
        if host:
            out = out.cpu().numpy()
        if self.passthrough:  # output = *input_: organised shape kept
            return PointCloud(out, cloud.width, cloud.height, cloud.is_dense)
        return PointCloud(out, cnt.value, 1, True)


def pcd_header(width, height) -> bytes:
    n = lib().sdr_pcd_header(int(width), int(height), None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    check(min(0, lib().sdr_pcd_header(int(width), int(height), buf, n + 1)))
    return buf.raw[:n]


def savePCDFileBinary(path: str, cloud: PointCloud):
    pts = cloud.points.cpu().numpy() if _is_cuda(cloud.points) else np.ascontiguousarray(cloud.points, np.float32)
    check(lib().sdr_write_pcd_binary(str(path).encode(), pts.ctypes.data, cloud.width, cloud.height))
