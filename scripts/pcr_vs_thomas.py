"""How far the PCR line solver's WLS output is from ximgproc's sequential (THOMAS) order, over random
shapes, lambda, sigma and guides.  Both are the oracle's restatements
(oracle/wls_oracle.c fgs_line vs fgs_line_pcr); the GPU is bit-exact with each.

    python scripts/pcr_vs_thomas.py [cases] [seed] > profiles/r5_pcr_vs_thomas.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

GUIDES = ("flat", "edge", "noise", "scene")


def case(rng, i):
    W = int(rng.choice([64, 200, 640, 1280, 2048, 3840, 4096])) if i % 3 else int(rng.integers(40, 700))
    H = int(rng.integers(8, 48)) if W > 1500 else int(rng.integers(8, 160))
    lam = float(np.exp(rng.uniform(np.log(10), np.log(2e4))))
    sig = float(rng.uniform(0.5, 5.0))
    kind = GUIDES[i % len(GUIDES)]
    D = 80
    if kind == "scene":  # the matcher pair of a synthetic frame: realistic confidence
        L, R, _ = S.make_pair(H, W, D, seed=int(rng.integers(1 << 30)))
        g = L
        dl = O.sgbm_compute(L, R, O.make_params(0, D, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2))
        dr = O.sgbm_compute(R, L, O.make_params(-(D - 1), D, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2))
    else:
        if kind == "flat":
            g = np.full((H, W), int(rng.integers(0, 256)), np.uint8)
        elif kind == "edge":
            g = np.zeros((H, W), np.uint8)
            g[:, int(rng.integers(1, W)):] = 255
            g[int(rng.integers(1, H)):, :] ^= 255
        else:
            g = rng.integers(0, 256, (H, W), dtype=np.uint8)
        blocks = rng.integers(0, D * 16, ((H + 7) // 8, (W + 7) // 8))
        dl = np.repeat(np.repeat(blocks, 8, 0), 8, 1)[:H, :W].astype(np.int16)
        dl[rng.random((H, W)) < 0.1] = -16
        dr = -np.clip(dl, 0, None).astype(np.int16)
    q = O.wls_params_for_sgbm(0, D, 5, W, H, lam, sig)
    q.fgs_solver = O.FGS_PCR
    a = O.wls_filter(dl, dr, g, q).astype(np.int32)
    q.fgs_solver = O.FGS_THOMAS
    b = O.wls_filter(dl, dr, g, q).astype(np.int32)
    d = np.abs(a - b)
    return {"W": W, "H": H, "lambda": round(lam, 2), "sigma": round(sig, 3), "guide": kind,
            "max_levels": int(d.max()), "frac_differ": float((d > 0).mean()),
            "frac_over_1": float((d > 1).mean())}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 2024)
    rows = [case(rng, i) for i in range(n)]
    over = [r for r in rows if r["max_levels"] > 1]
    by = {k: max((r["max_levels"] for r in rows if r["guide"] == k), default=0) for k in GUIDES}
    print(json.dumps({"cases": n, "cases_over_1_level": len(over), "worst_by_guide": by,
                      "worst": max(rows, key=lambda r: (r["max_levels"], r["frac_differ"])), "rows": rows},
                     indent=1))


if __name__ == "__main__":
    main()
