"""Diagnostic: per-chunk s_memtime stamps of one sequential-FGS launch (workgroup 0), from a library
built with -DSDR_TH_STAMPS:  python stereo_depth_ruler_amd/build.py thstamps SDR_TH_STAMPS
SDR_TH_STAMP_LAUNCH=K python scripts/th_stamps.py stereo_depth_ruler_amd/lib/libsdr-thstamps.so
(launch K of the process: 7 a filter call, 0 = coefficient jobs, 1 = the first row pass ...)."""
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
g = torch.from_numpy(rng.integers(0, 256, (h, w)).astype(np.uint8)).to(dev)
x = torch.from_numpy((rng.random((2, h, w)) * 1000).astype(np.float32)).to(dev)
for _ in range(4):
    fastGlobalSmootherFilter(g, x, 8000.0, 1.1, solver=FGS_THOMAS)
torch.cuda.synchronize()
lib = ctypes.CDLL(sys.argv[1])
buf = np.zeros((6, 1024), np.uint64)
assert lib.sdr_th_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
t0 = int(buf[0, 0])
S = lambda r, i: (int(buf[r, i]) - t0) if buf[r, i] else None  # noqa: E731
for base, name in ((0, "forward"), (512, "back")):
    print(f"-- {name} (cycles from the solver's first chunk start): c, solver start, solver end, "
          "loader issued, loader ready, writer put")
    for c in range(64):
        if not buf[0, base + c]:
            break
        print(c, S(0, base + c), S(1, base + c), S(2, base + c), S(3, base + c), S(4, base + c) if base == 0 else "",
              "steps 0/16/32/48:" if base == 0 else "", [S(5, 8 * c + q) for q in range(4)] if base == 0 else "")
