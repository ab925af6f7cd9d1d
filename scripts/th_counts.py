"""Diagnostic: how the sequential FGS passes' chunks ran (reciprocal form / exact from the start /
redone) on the class path's own frame (StereoDisparity.computeDisparity: both matchers + WLS on a
synthetic 1280x720 pair), from a library built with -DSDR_TH_STAMPS.
python scripts/th_counts.py stereo_depth_ruler_amd/lib/libsdr-thstamps.so"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from stereo_depth_ruler_amd import _lib  # noqa: E402

_lib.use_library(sys.argv[1])
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from stereo_depth_ruler_amd.stereo_disparity import StereoDisparity  # noqa: E402

lib = ctypes.CDLL(sys.argv[1])
Q = np.eye(4)
sd = StereoDisparity(Q)
for seed in range(3):
    left, right, _ = S.make_pair(720, 1280, 160, seed=seed)
    L = np.repeat(left[:, :, None], 3, axis=2)
    R = np.repeat(right[:, :, None], 3, axis=2)
    sd.computeDisparity(L, R)
    c = np.zeros(4, np.uint32)
    assert lib.sdr_th_counts(c.ctypes.data_as(ctypes.c_void_p)) == 0
    conf = sd.conf_map
    print(f"seed {seed}: chunks fast {c[0]}, exact from the start {c[1]}, redone {c[2]}; "
          f"confidence zero on {np.mean(conf == 0):.3f} of the map, disp invalid {np.mean(sd.last_disp_left < 0):.3f}")
buf = np.zeros((6, 1024), np.uint64)
if lib.sdr_th_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0 and buf[0, 0]:
    t0 = int(buf[0, 0])
    S_ = lambda r, i: (int(buf[r, i]) - t0) if buf[r, i] else None  # noqa: E731
    for base, name in ((0, "forward"), (512, "back")):
        print(f"-- {name}: c, solver start, solver end, loader issued, loader ready, writer put, steps 0/16/32/48")
        for c in range(64):
            if not buf[0, base + c]:
                break
            print(c, S_(0, base + c), S_(1, base + c), S_(2, base + c), S_(3, base + c),
                  S_(4, base + c) if base == 0 else "", [S_(5, 8 * c + q) for q in range(4)] if base == 0 else "")
blk = np.zeros((512, 3), np.uint64)
if lib.sdr_th_blocks(blk.ctypes.data_as(ctypes.c_void_p)) == 0 and blk[0, 0]:
    used = [i for i in range(512) if blk[i, 0]]
    t0 = min(int(blk[i, 0]) for i in used)
    rows = sorted(((int(blk[i, 2]) - int(blk[i, 0]), int(blk[i, 1]) - int(blk[i, 0]), int(blk[i, 0]) - t0, i) for i in used),
                  reverse=True)
    print("workgroups of the stamped launch, slowest first: (total cycles, forward cycles, start offset, block)")
    for r in rows[:8]:
        print("  ", r)
    print("   fastest:", rows[-3:])
