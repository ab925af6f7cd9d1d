"""Diagnostic: per-workgroup s_memtime stamps of the six k_fgs_lr passes of one FGS call, from a
library built with -DSDR_TH_STAMPS:
  python stereo_depth_ruler_amd/build.py thstamps SDR_TH_STAMPS
  python scripts/lr_stamps.py stereo_depth_ruler_amd/lib/libsdr-thstamps.so
Per pass (medians over workgroups, cycles): entry -> first chunk landed, forward, back, the writers'
tail after the back substitution, the kernel's span (first entry to last exit) and the clock."""
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
    for _ in range(16):  # fill every slot; the last call's passes are the last six slots written
        fastGlobalSmootherFilter(g, x, 8000.0, 1.1, solver=FGS_THOMAS)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(sys.argv[1])
    buf = np.zeros((16, 512, 8), np.uint64)
    assert lib.sdr_lr_blocks(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    print(f"-- {name}: pass, workgroups, first chunk, forward, back, writer tail, span (cycles); clock GHz")
    for p, slot in enumerate(range(10, 16)):  # 16 calls x 6 passes = 96 launches: the last call's are slots 10-15
        b = buf[slot].astype(np.int64)
        nb = int((b[:, 0] > 0).sum())
        b = b[:nb]
        med = lambda v: int(np.median(v))  # noqa: E731
        span = int(b[:, [4, 5]].max() - b[:, 0].min())
        clk = np.median((b[:, 5] - b[:, 0]) / ((b[:, 7] - b[:, 6]) / 100e6) / 1e9)
        print(f"pass {p} ({'rows' if p % 2 == 0 else 'columns'}) wg={nb}: {med(b[:, 1] - b[:, 0])} "
              f"{med(b[:, 2] - b[:, 1])} {med(b[:, 3] - b[:, 2])} {med(b[:, 4] - b[:, 3])} span {span}; "
              f"{clk:.2f} GHz; forward max {int((b[:, 2] - b[:, 1]).max())}")
