"""3WAY stripe-start rows (debug stage 6) vs numpy_ref's boxed stripe rows, wide block."""
import math
import sys

import numpy as np

sys.path.insert(0, "tests")
import numpy_ref as N  # noqa: E402
import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

for bs in (11, 17):
    H, W, D, minD = 26, 110, 32, 0
    args = (minD, D, bs, 10, 500, 1, 15, 10, 0, 2, 2)
    L, R = S.adversarial_pair("noise", H, W, D, seed=bs)
    m = sdr.StereoSGBM.create(*args, nstripes=4)
    m.compute(L, R)
    SH2 = bs // 2
    pix = N.bt_cost_volume_rows(L, R, minD, D, 15)
    W1 = pix.shape[1]
    xi = np.clip(np.arange(W1)[:, None] + np.arange(-SH2, SH2 + 1)[None, :], 0, W1 - 1)
    hs = pix[:, xi, :].sum(2)
    sz = math.ceil(H / 4)
    ov = (bs // 2 + 1) + math.ceil(0.1 * sz)
    st = []
    for s in range(4):
        out0 = s * sz
        s0 = max(min(s * sz - ov, H), 0)
        end = min((s + 1) * sz, H)
        ylim = max(H - 1 - SH2, s0)
        aux = 0 if s0 == 0 else (SH2 if ylim >= s0 + SH2 else end - s0)
        st.append((s0, end, aux))
    amax = max(a for _, _, a in st)
    Ca = m.debug_stage(6, (4, amax, W1, D), np.int16)
    for s, (s0, end, aux) in enumerate(st):
        if not aux:
            continue
        exp = (N._box_rows(hs, s0, end, SH2, False)[:aux] + 500).astype(np.int16)
        got = Ca[s, :aux]
        bad = np.argwhere(got != exp)
        print("bs", bs, "stripe", s, "s0", s0, "aux", aux, "bad", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:10])
