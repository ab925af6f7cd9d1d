"""Device pipelines for the reference's two per-frame loops, built from the engine's C ABI:

* ``LiveLoop`` -- stereo_vision/src/stereo_displayer.cpp:145-185 (``show_disparity_overlay``):
  side-by-side BGR frame -> split + StereoRectifier::rectify -> StereoDisparity::computeDisparity
  (BGR2GRAY, INTER_AREA 0.5x, left 3WAY + right matcher, WLS, /16) -> computeDepth, and with
  ``display=True`` the loop's display outputs (show_depthMap, show_disparityMap, the JET overlay
  on the half-size rectified left view; :164-173), frames of a batch in order through the EMAs.
* ``CloudEmit`` -- point_cloud/src/pcd_write.cpp:81-130 (``save_and_display_pointcloud``):
  side-by-side BGR frame -> split -> BGR2GRAY -> StereoSGBM::compute -> /16 ->
  reprojectImageTo3D(handleMissing) -> convertCVMatToPCL(left) -> VoxelGrid.

Both take device-resident frames (torch uint8 (F, H, 2W, 3)), enqueue on the given stream and keep
all scratch per instance, so several instances can keep frames in flight on separate streams.
The CPU is never used for pixels; a missing libsdr.so raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib
from .display import Display
from .sgbm import MODE_SGBM_3WAY, StereoSGBM, _Q, createRightMatcher, set_handle_stream, torch
from .ximgproc import createDisparityWLSFilter


def _vp(x):
    return ctypes.c_void_p(x)


class LiveLoop:
    """The reference app's per-frame loop on one device (see module docstring)."""

    def __init__(self, rectifier, Q, batch: int, device: int = 0, args=None, display: bool = False):
        self.rect = rectifier
        self.W, self.H = rectifier.W, rectifier.H
        self.Q = np.asarray(Q, np.float64)
        self.batch = int(batch)
        self.dev = torch.device("cuda", device)
        args = args or (0, 80, 5, 8 * 5 * 5 * 3, 32 * 5 * 5 * 3, 1, 63, 12, 200, 2, MODE_SGBM_3WAY)
        self.left = StereoSGBM.create(*args, device=device)          # stereo_disparity.cpp:5-9
        self.right = createRightMatcher(self.left)                     # :10
        self.wls = createDisparityWLSFilter(self.left)                 # :11
        self.wls.setLambda(8000.0)                                     # :12
        self.wls.setSigmaColor(1.1)                                    # :13
        h2, w2 = self.H // 2, self.W // 2
        self.h2, self.w2 = h2, w2
        z = dict(device=self.dev)
        self.small_l = torch.empty((batch, h2, w2), dtype=torch.uint8, **z)
        self.small_r = torch.empty_like(self.small_l)
        self.disp = torch.empty((batch, h2, w2), dtype=torch.float32, **z)     # computeDisparity()
        self.filtered = torch.empty((batch, h2, w2), dtype=torch.int16, **z)
        self.depth = torch.empty((batch, h2, w2, 3), dtype=torch.float32, **z)  # computeDepth()
        self.display = Display(device) if display else None
        if display:
            self.left_rect = torch.empty((batch, self.H, self.W, 3), dtype=torch.uint8, **z)
            self.vis = torch.empty((batch, h2, w2), dtype=torch.uint8, **z)           # show_disparityMap
            self.depth_vis = torch.empty((batch, h2, w2, 3), dtype=torch.uint8, **z)  # show_depthMap
            self.overlay = torch.empty((batch, h2, w2, 3), dtype=torch.uint8, **z)    # overlay

    def matcher(self):
        return self.left

    def enqueue(self, sbs, stream, ingest_events=None):
        """sbs: uint8 (batch, H, 2W, 3) on the device; everything runs on `stream`.
        ingest_events (optional): two torch.cuda.Event recorded on `stream` around the ingest
        (split + rectify + gray + INTER_AREA), for per-kernel timing."""
        s = _vp(stream.cuda_stream)
        L = lib()
        check(L.sdr_rectifier_set_stream(self.rect._h, s))
        disp_on = self.display is not None
        if ingest_events:
            ingest_events[0].record(stream)
        check(L.sdr_rectify_sbs_device(self.rect._h, sbs.data_ptr(), self.W * 6, self.W * 6 * self.H,
                                       self.batch, self.left_rect.data_ptr() if disp_on else None, None,
                                       self.small_l.data_ptr(), self.small_r.data_ptr()))
        if ingest_events:
            ingest_events[1].record(stream)
        set_handle_stream(self.left._h, self.left._device, stream)
        # computeDisparity + computeDepth: reprojectImageTo3D(half-res disparity, full-res Q)
        # (stereo_disparity.cpp:76-80), fused into the WLS filter's epilogue
        check(L.sdr_stereo_class_depth_device(self.left._h, self.right._h, self.wls._h,
                                              self.small_l.data_ptr(), self.small_r.data_ptr(),
                                              self.w2, self.h2, self.batch, self.disp.data_ptr(),
                                              self.filtered.data_ptr(), None, _Q(self.Q),
                                              self.depth.data_ptr()))
        if disp_on:  # stereo_displayer.cpp:164-173
            d, F, w2, h2 = self.display, self.batch, self.w2, self.h2
            check(L.sdr_display_set_stream(d._h, s))
            check(L.sdr_show_depth_map_device(d._h, self.depth.data_ptr(), w2, h2, 3, F, None, None,
                                              self.depth_vis.data_ptr(), None))
            check(L.sdr_show_disparity_map_device(d._h, self.disp.data_ptr(), w2, h2, w2, w2 * h2, F,
                                                  self.left.getNumDisparities(), self.vis.data_ptr()))
            check(L.sdr_disparity_overlay_device(d._h, self.vis.data_ptr(), self.left_rect.data_ptr(),
                                                 self.W * 3, self.W * 3 * self.H, w2, h2, F, None, None,
                                                 self.overlay.data_ptr()))
        return self.filtered

    def close(self):
        for o in (self.left, self.right, self.wls, self.display):
            if o is not None:
                o.close()


class CloudEmit:
    """pcd_write.cpp's single-frame path as a batched device pipeline (see module docstring)."""

    def __init__(self, W, H, args, batch: int, Q, leaf=0.005, device: int = 0):
        self.W, self.H, self.batch = int(W), int(H), int(batch)
        self.Q = np.asarray(Q, np.float64)
        self.leaf = float(leaf)
        self.dev = torch.device("cuda", device)
        self.m = StereoSGBM.create(*args, device=device)
        z = dict(device=self.dev)
        self.gray_l = torch.empty((batch, H, W), dtype=torch.uint8, **z)
        self.gray_r = torch.empty_like(self.gray_l)
        self.disp = torch.empty((batch, H, W), dtype=torch.int16, **z)
        self.xyz = torch.empty((batch, H, W, 3), dtype=torch.float32, **z)
        self.points = torch.empty((batch, H * W, 4), dtype=torch.float32, **z)
        self.filtered = torch.empty((batch, H * W, 4), dtype=torch.float32, **z)
        self.counts = [0] * batch
        self.passthrough = [False] * batch

    def matcher(self):
        return self.m

    def enqueue(self, sbs, stream, voxel=True):
        """sbs: uint8 (batch, H, 2W, 3) on the device.  The voxel grid returns host counts, so that
        stage synchronises `stream` once per frame; voxel=False leaves it to voxel(), which a
        caller running several pipelines can call after enqueueing the next one's frames, so the
        GPU has work queued while the host waits."""
        s = _vp(stream.cuda_stream)
        L = lib()
        W, H, F = self.W, self.H, self.batch
        row = 2 * W * 3
        # frame(Rect(0, 0, W, H)) / frame(Rect(W, 0, W, H)) -> cvtColor(BGR2GRAY)  (pcd_write.cpp:83-89)
        check(L.sdr_bgr2gray_device(sbs.data_ptr(), W, H, row, self.gray_l.data_ptr(), W, F, s))
        check(L.sdr_bgr2gray_device(sbs.data_ptr() + W * 3, W, H, row, self.gray_r.data_ptr(), W, F, s))
        # sgbm->compute -> convertTo(1/16) -> reprojectImageTo3D(handleMissing)  (:111-116)
        set_handle_stream(self.m._h, self.m._device, stream)
        check(L.sdr_sgbm_compute_reproject_device(self.m._h, self.gray_l.data_ptr(), self.gray_r.data_ptr(),
                                                  W, H, W, W * H, F, self.disp.data_ptr(), _Q(self.Q), 1,
                                                  self.xyz.data_ptr()))
        # convertCVMatToPCL(pointCloud_CV, left)  (:119)
        check(L.sdr_xyz_to_cloud_device(self.xyz.data_ptr(), sbs.data_ptr(), row, row * H, W, H, F,
                                        self.points.data_ptr(), s))
        if voxel:
            self.voxel(stream)
        return self.disp

    def voxel(self, stream):
        """VoxelGrid 5 mm (:122-130) of the frames the last enqueue left in `points`, on the stream
        that enqueued them (synchronous: the counts are host values)."""
        s = _vp(stream.cuda_stream)
        L = lib()
        W, H = self.W, self.H
        cnt, pt = ctypes.c_int(), ctypes.c_int()
        for f in range(self.batch):
            check(L.sdr_voxel_grid_device(self.points[f].data_ptr(), W * H, self.leaf, self.leaf,
                                          self.leaf, self.filtered[f].data_ptr(), ctypes.byref(cnt),
                                          ctypes.byref(pt), s))
            self.counts[f], self.passthrough[f] = cnt.value, bool(pt.value)

    def close(self):
        self.m.close()
