"""Sweep records vs k_paths' per-direction records (debug stage 4) for one failing case."""
import numpy as np
import torch

import stereo_depth_ruler_amd as sdr
from stereo_depth_ruler_amd import synthetic as S

F, H, W, D = 8, 40, 200, 64
args = (0, D, 5, 600, 2400, 1, 63, 10, 30, 2, sdr.MODE_HH)
Ls = np.empty((F, H, W), np.uint8)
Rs = np.empty((F, H, W), np.uint8)
for i in range(F):
    Ls[i], Rs[i], _ = S.make_pair(H, W, D, 1 + i)
W1 = W - D
m = sdr.StereoSGBM.create(*args)
m.compute(torch.from_numpy(Ls).cuda(), torch.from_numpy(Rs).cuda())
torch.cuda.synchronize()
rec = m.debug_stage(4, (F, H, W1, 4, D), np.int16)
m1 = sdr.StereoSGBM.create(*args)
for f in range(F):
    m1.compute(Ls[f], Rs[f])
    one = m1.debug_stage(4, (1, H, W1, 7, D), np.int16)[0].astype(np.int32)
    up = np.minimum(one[:, :, 2] + one[:, :, 5] + one[:, :, 6], 32767)
    dn = np.minimum(one[:, :, 3] + one[:, :, 4], 32767)
    for name, got, ref in (("E", rec[f, :, :, 0], one[:, :, 0]), ("W", rec[f, :, :, 1], one[:, :, 1]),
                           ("up", rec[f, :, :, 2], up), ("down", rec[f, :, :, 3], dn)):
        bad = np.argwhere((got != ref).any(-1))
        if not len(bad):
            continue
        print("frame", f, name, "bad pixels", len(bad), bad[:24].tolist())
        y, x = bad[0]
        dd = np.nonzero(got[y, x] != ref[y, x])[0]
        print("  first", (y, x), "d", dd[:10].tolist(), got[y, x][dd[:5]].tolist(), ref[y, x][dd[:5]].tolist())
print("done")
