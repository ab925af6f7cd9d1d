"""Wide-block cases per mode: final and LR-stage maps vs the oracle."""
import numpy as np

import stereo_depth_ruler_amd as sdr
from oracle import oracle as O
from stereo_depth_ruler_amd import synthetic as S

for mode in (0, 1, 2):
    for kind in ("binary", "noise", "textured"):
        for bs in (13, 17):
            for minD in (0, -7):
                H, W, D = 26, 110, 32
                args = (minD, D, bs, 10, 500, 1, 15, 10, 0, 2, mode)
                L, R = S.adversarial_pair(kind, H, W, D, seed=bs + mode)
                for ns in ((1, 4) if mode == 2 else (4,)):
                    m = sdr.StereoSGBM.create(*args, nstripes=ns)
                    got = m.compute(L, R)
                    p = O.make_params(*args, nstripes=ns)
                    ref = O.sgbm_compute(L, R, p)
                    W1 = W + min(minD, 0) - max(minD + D, 0)
                    C = m.debug_cost_volume(H, W1, D)
                    cb = int((C != O.cost_volume(L, R, p)).sum())
                    raw = m.debug_stage(1, (H, W), np.int16)
                    rref = O.sgbm_compute(L, R, p, stages=-1) if False else None
                    bad = np.argwhere(got != ref)
                    if len(bad) or cb:
                        print("mode", mode, kind, "bs", bs, "minD", minD, "ns", ns, "cost bad", cb, "final bad", len(bad),
                              "rows", sorted(set(bad[:, 0].tolist()))[:12], "cols", sorted(set(bad[:, 1].tolist()))[:12])
print("done")
