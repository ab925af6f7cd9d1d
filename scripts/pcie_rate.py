"""PCIe-inclusive rate of the host-buffer drop-in (the reference's own call pattern).

    python scripts/pcie_rate.py [--frames 200]

C2 workload (1280x720, d=128, MODE_SGBM) through the synchronous host-pointer entry points, one
frame per call, inputs and outputs in pageable host memory (numpy), as the reference makes them:

  separate  StereoSGBM::compute(host L, host R) -> host int16 disparity, then convertTo(1/16) +
            reprojectImageTo3D(handleMissing) from and to host memory (pcd_write.cpp:111-116 call
            for call: sdr_sgbm_compute + sdr_reproject);
  fused     sdr_sgbm_compute_reproject: the same outputs (int16 disparity and XYZ) from one call,
            the float disparity never leaving the device;
  fused_pinned  the fused call on page-locked host buffers (sdr.host_empty, the role of
            cv::cuda::HostMem): DMA straight to and from the caller's buffers.

Prints one JSON line (fps, Mpix/s and ms per frame of each pattern).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    W, H, D = 1280, 720, 128
    Ls, Rs = S.make_batch(4, H, W, D, seed0=0)
    m = sdr.StereoSGBM.create(0, D, 5, 600, 2400, 1, 63, 12, 200, 2, sdr.MODE_SGBM)
    disp = np.empty((H, W), np.int16)
    xyz = np.empty((H, W, 3), np.float32)

    def separate(i):
        d = m.compute(Ls[i % 4], Rs[i % 4], disp)
        return sdr.reprojectImageTo3D(d.astype(np.float32) * np.float32(0.0625), S.REFERENCE_Q, True)

    def fused(i):
        return m.compute_reproject(Ls[i % 4], Rs[i % 4], S.REFERENCE_Q, True, disp=disp, xyz=xyz)[1]

    # the same fused call with every host buffer page-locked (sdr.host_empty, cf. cv::cuda::HostMem)
    pL = [sdr.host_empty((H, W), np.uint8) for _ in range(4)]
    pR = [sdr.host_empty((H, W), np.uint8) for _ in range(4)]
    for i in range(4):
        pL[i][:], pR[i][:] = Ls[i], Rs[i]
    pdisp = sdr.host_empty((H, W), np.int16)
    pxyz = sdr.host_empty((H, W, 3), np.float32)

    def fused_pinned(i):
        return m.compute_reproject(pL[i % 4], pR[i % 4], S.REFERENCE_Q, True, disp=pdisp, xyz=pxyz)[1]

    # the patterns give the same bytes
    ref = separate(0).view(np.uint32).copy()
    assert np.array_equal(ref, fused(0).view(np.uint32))
    assert np.array_equal(ref, fused_pinned(0).view(np.uint32))
    res = {"workload": "C2 host-pointer drop-in, synchronous, 1 frame per call, pageable host buffers",
           "frames": a.frames}
    for name, fn in (("separate", separate), ("fused", fused), ("fused_pinned", fused_pinned)):
        for i in range(5):
            fn(i)
        t0 = time.perf_counter()
        for i in range(a.frames):
            fn(i)
        el = (time.perf_counter() - t0) / a.frames
        res[name] = {"fps": round(1 / el, 1), "Mpix_s": round(W * H / el / 1e6, 1), "ms_per_frame": round(el * 1e3, 3)}
    t0 = time.perf_counter()
    for i in range(a.frames):
        m.compute(Ls[i % 4], Rs[i % 4], disp)
    el = (time.perf_counter() - t0) / a.frames
    res["compute_only"] = {"fps": round(1 / el, 1), "ms_per_frame": round(el * 1e3, 3)}
    m.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
