"""PCIe-inclusive rate of the host-buffer drop-in (the reference's own call pattern).

    python scripts/pcie_rate.py [--frames 200]

C2 workload through the synchronous host-pointer entry points, one call after the other as
pcd_write.cpp:111-116 makes them: StereoSGBM::compute(host L, host R) -> host int16 disparity,
then convertTo(1/16) + reprojectImageTo3D(handleMissing) from and to host memory.  Prints one
JSON line (fps, Mpix/s, ms per frame for each call).
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
    for i in range(5):
        d = m.compute(Ls[i % 4], Rs[i % 4])
        sdr.reprojectImageTo3D(d.astype(np.float32) * np.float32(0.0625), S.REFERENCE_Q, True)
    tc = tr = 0.0
    t0 = time.perf_counter()
    for i in range(a.frames):
        t1 = time.perf_counter()
        d = m.compute(Ls[i % 4], Rs[i % 4])
        t2 = time.perf_counter()
        sdr.reprojectImageTo3D(d.astype(np.float32) * np.float32(0.0625), S.REFERENCE_Q, True)
        t3 = time.perf_counter()
        tc += t2 - t1
        tr += t3 - t2
    el = time.perf_counter() - t0
    m.close()
    fps = a.frames / el
    print(json.dumps({"workload": "C2 host-pointer drop-in, synchronous, 1 frame per call", "frames": a.frames,
                      "fps": round(fps, 1), "Mpix_s": round(fps * W * H / 1e6, 1),
                      "compute_ms": round(tc / a.frames * 1e3, 3), "reproject_ms": round(tr / a.frames * 1e3, 3)}))


if __name__ == "__main__":
    main()
