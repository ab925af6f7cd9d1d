"""Diagnostic: per-wave cycle split of k_south_wta (build variant with -DSDR_SOUTH_STAMP=1).

    SDR_LIB_VARIANT=stamp python scripts/south_stamps.py
Runs one C2 frame, reads the stamp words the kernel leaves in the disp2-key buffer (debug stage 5),
prints total and barrier-wait cycles of the producer and the consumer waves."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

W, H, D = 1280, 720, 128
L, R, _ = S.make_pair(H, W, D, seed=1)
m = sdr.StereoSGBM.create(0, D, 5, 600, 2400, 1, 63, 12, 200, 2, 0)
Ld, Rd = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
for _ in range(3):
    m.compute(Ld, Rd)
torch.cuda.synchronize()
from stereo_depth_ruler_amd import _lib

print("library:", _lib.LIB_PATH)
raw = m.debug_stage(5, (H * W,), np.uint32).view(np.uint64)
print("first words:", [hex(int(v)) for v in raw[:6]])
W1 = W - D
nw = 4
st = raw[: 2 * W1 * nw].reshape(W1, nw, 2).astype(np.float64)
for role, sl in (("producer", st[:, 0]), ("consumers", st[:, 1:].reshape(-1, 2))):
    tot, wait = sl[:, 0], sl[:, 1]
    print(f"{role:9s} total {tot.mean():10.0f} cyc (min {tot.min():.0f} max {tot.max():.0f})  "
          f"in barriers {wait.mean():10.0f} cyc = {100 * wait.mean() / tot.mean():.1f} %")
