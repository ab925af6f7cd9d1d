"""Class-path (C4) output dump for experiment A/B of engine builds: one build per process.

    python scripts/class_ab.py --lib stereo_depth_ruler_amd/lib/libsdr-x.so --out gpurun_out/x.npz
    python scripts/class_ab.py --compare gpurun_out/a.npz gpurun_out/b.npz

Runs the reference's per-frame loop (LiveLoop: ingest, both matchers, WLS, computeDepth) on four
synthetic ZED2 side-by-side frames and saves the disparity (float), the filtered disparity and the
depth; --compare reports whether two dumps are bit-identical.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(lib, out):
    from stereo_depth_ruler_amd import _lib
    _lib.use_library(lib)
    import torch
    from stereo_depth_ruler_amd import synthetic as S
    from stereo_depth_ruler_amd.config import StereoConfiguration
    from stereo_depth_ruler_amd.pipeline import LiveLoop
    from stereo_depth_ruler_amd.rectify import StereoRectifier

    dev = torch.device("cuda", 0)
    cfg = StereoConfiguration()
    assert cfg.loadFromFile(os.path.join(ROOT, "tests", "golden", "stereo.yaml"))
    H, W, F = 720, 1280, 4
    sbs = torch.stack([torch.from_numpy(S.sbs_bgr_color_frame(H, W, 80, seed=7 + i)) for i in range(F)]).to(dev)
    rect = StereoRectifier(cfg, device=0)
    loop = LiveLoop(rect, cfg.Q, F, device=0)
    st = torch.cuda.current_stream(dev)
    loop.enqueue(sbs, st)
    torch.cuda.synchronize()
    np.savez(out, disp=loop.disp.cpu().numpy(), filtered=loop.filtered.cpu().numpy(),
             depth=loop.depth.cpu().numpy())
    loop.close()
    rect.close()


def compare(a, b):
    A, B = np.load(a), np.load(b)
    same = True
    for k in A.files:
        eq = np.array_equal(A[k], B[k], equal_nan=True) if A[k].dtype.kind == "f" else np.array_equal(A[k], B[k])
        print(f"{k}: {'identical' if eq else 'DIFFERENT'}")
        same &= eq
    return same


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        sys.exit(0 if compare(*a.compare) else 1)
    dump(a.lib, a.out)
