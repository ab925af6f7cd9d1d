"""Generates tests/golden/*.npz: seeded small synthetic pairs, parameters and the oracle's outputs.

The reference holds no fixtures for this path and OpenCV is absent, so these are
golden vectors of the C restatement (oracle/sgbm_oracle.c): they pin the oracle against
regressions and give the GPU tests fixed inputs.  Re-run only when the oracle intentionally
changes:  python scripts/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

# name: (H, W, seed, create-args)
CASES = {
    "sgbm5_d32": (40, 112, 1, (0, 32, 5, 600, 2400, 1, 63, 12, 50, 2, 0)),
    "hh8_d48": (36, 120, 2, (0, 48, 5, 600, 2400, 1, 63, 10, 30, 1, 1)),
    "3way_d80_ref": (64, 200, 3, (0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, 2)),
    "3way_right_matcher": (64, 200, 3, (-79, 80, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2)),
    "sgbm5_neg_mind_bs3": (30, 96, 4, (-8, 16, 3, 8, 32, 2, 31, 5, 0, 0, 0)),
    "3way_bs7_uniq20": (50, 130, 5, (0, 32, 7, 200, 800, 1, 63, 20, 20, 1, 2)),
}


def main():
    out_dir = os.path.join(ROOT, "tests", "golden")
    os.makedirs(out_dir, exist_ok=True)
    for name, (h, w, seed, args) in CASES.items():
        L, R, _ = S.make_pair(h, w, max(args[1], 16), seed=seed)
        if args[0] < 0:  # right matcher: compute(right, left)
            L, R = R, L
        p = O.make_params(*args)
        full = O.sgbm_compute(L, R, p)
        raw = O.sgbm_compute(L, R, p, stages=0)
        xyz = O.reproject(O.disp_to_float(full), S.REFERENCE_Q, True)
        np.savez_compressed(os.path.join(out_dir, f"{name}.npz"), left=L, right=R,
                            params=np.array(args, np.int32), disp=full, disp_raw=raw, xyz=xyz)
        print(name, L.shape, "valid", float((full > (args[0] - 1) * 16).mean()))


if __name__ == "__main__":
    main()
