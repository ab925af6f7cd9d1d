"""3WAY short last stripes (ylim < s0 + SH2): engine vs oracle at blockSize <= 11."""
import numpy as np

import stereo_depth_ruler_amd as sdr
from oracle import oracle as O
from stereo_depth_ruler_amd import synthetic as S

for bs in (5, 7, 9, 11):
    for H in range(8, 30):
        for ns in (4, 8):
            args = (0, 32, bs, 10, 500, 1, 15, 10, 0, 2, 2)
            L, R = S.adversarial_pair("noise", H, 90, 32, seed=H)
            got = sdr.StereoSGBM.create(*args, nstripes=ns).compute(L, R)
            ref = O.sgbm_compute(L, R, O.make_params(*args, nstripes=ns))
            n = int((got != ref).sum())
            if n:
                print("bs", bs, "H", H, "ns", ns, "bad", n)
print("done")
