"""Wide-block (blockSize 13..17) cost volume vs the oracle's, per case: where do they differ?"""
import numpy as np

import stereo_depth_ruler_amd as sdr
from oracle import oracle as O
from stereo_depth_ruler_amd import synthetic as S

cases = [("binary", 20, 100, (0, 32, 13, 10, 500, 1, 15, 10, 0, 2, 0)),
         ("noise", 24, 90, (-5, 16, 15, 10, 500, 1, 15, 10, 0, 2, 1)),
         ("textured", 30, 120, (0, 48, 17, 10, 500, 1, 15, 10, 0, 2, 0)),
         ("binary", 8, 60, (0, 16, 13, 10, 500, 1, 15, 10, 0, 2, 0)),
         ("binary", 20, 40, (0, 16, 13, 10, 500, 1, 15, 10, 0, 2, 0))]
for kind, H, W, args in cases:
    L, R = S.adversarial_pair(kind, H, W, args[1], seed=3)
    m = sdr.StereoSGBM.create(*args)
    m.compute(L, R)
    minD, D = args[0], args[1]
    W1 = W + min(minD, 0) - max(minD + D, 0)
    C = m.debug_cost_volume(H, W1, D)
    ref = O.cost_volume(L, R, O.make_params(*args))
    bad = np.argwhere(C != ref)
    print(kind, H, W, args[2], args[10], "W1", W1, "bad", len(bad), bad[:8].tolist())
    if len(bad):
        y, x, d = bad[0]
        print("   got", C[y, x, d], "ref", ref[y, x, d], "rows bad", sorted(set(bad[:, 0].tolist()))[:20],
              "cols bad", sorted(set(bad[:, 1].tolist()))[:20])
