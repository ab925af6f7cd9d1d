"""Diagnostic: per-workgroup s_memtime stamps of k_fgs_lrjob (the FGS coefficient jobs) of the last
FGS call, from a library built with -DSDR_TH_STAMPS:
  python scripts/lj_stamps.py stereo_depth_ruler_amd/lib/libsdr-thstamps.so
Per job (medians over its workgroups, cycles from the workgroup's entry): chunk 0 prepared, solver
past its first barrier, solver done, writer done, prep done; and the launch span."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from stereo_depth_ruler_amd import _lib  # noqa: E402

_lib.use_library(sys.argv[1])
from stereo_depth_ruler_amd.ximgproc import FGS_THOMAS, fastGlobalSmootherFilter  # noqa: E402

rng = np.random.default_rng(0)
h, w = 360, 560
dev = torch.device("cuda", 0)
for name, guide in (("noise guide", rng.integers(0, 256, (h, w))),
                    ("smooth guide", (np.add.outer(np.arange(h), np.arange(w)) // 7) % 256)):
    g = torch.from_numpy(guide.astype(np.uint8)).to(dev)
    x = torch.from_numpy((rng.random((2, h, w)) * 1000).astype(np.float32)).to(dev)
    for _ in range(4):
        fastGlobalSmootherFilter(g, x, 8000.0, 1.1, solver=FGS_THOMAS)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(sys.argv[1])
    b = np.zeros((512, 8), np.uint64)
    assert lib.sdr_lj_blocks(b.ctypes.data_as(ctypes.c_void_p)) == 0
    b = b.astype(np.int64)
    nb = int((b[:, 0] > 0).sum())
    b = b[:nb]
    t0 = b[:, 0].min()
    clk = np.median((b[:, 3] - b[:, 0]) / ((b[:, 7] - b[:, 6]) / 100e6) / 1e9)
    print(f"-- {name}: {nb} workgroups, launch span {int(b[:, [3, 4, 5]].max() - t0)} cycles, clock {clk:.2f} GHz")
    # jobs in launch order: rows (h lines of w) and columns (w lines of h), three iterations
    lpb_r = 16 if w <= 384 else 8 if w <= 768 else 4
    lpb_c = 16 if h <= 384 else 8 if h <= 768 else 4
    nr, nc = (h + lpb_r - 1) // lpb_r, (w + lpb_c - 1) // lpb_c
    o = 0
    for j in range(6):
        n = nr if j % 2 == 0 else nc
        s = b[o:o + n]
        o += n
        if not len(s):
            break
        med = lambda v: int(np.median(v))  # noqa: E731
        e = s[:, 0]
        print(f"job {j} ({'rows' if j % 2 == 0 else 'columns'}, {len(s)} wg): start +{med(e - t0)}, "
              f"chunk0 prepared {med(s[:, 1] - e)}, solver start {med(s[:, 2] - e)}, solver done {med(s[:, 3] - e)}, "
              f"writer done {med(s[:, 4] - e)}, prep done {med(s[:, 5] - e)}")
