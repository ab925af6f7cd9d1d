"""Golden fixtures (tests/golden/, made by scripts/make_golden.py from the oracle) -- CPU side:
the oracle must reproduce its committed vectors bit for bit."""
import glob
import os

import numpy as np
import pytest

from stereo_depth_ruler_amd import synthetic as S

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def test_golden_present():
    assert len(GOLDEN) >= 6


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(oracle, path):
    g = np.load(path)
    p = oracle.make_params(*[int(v) for v in g["params"]])
    assert np.array_equal(oracle.sgbm_compute(g["left"], g["right"], p), g["disp"])
    assert np.array_equal(oracle.sgbm_compute(g["left"], g["right"], p, stages=0), g["disp_raw"])
    xyz = oracle.reproject(oracle.disp_to_float(g["disp"]), S.REFERENCE_Q, True)
    assert np.array_equal(xyz.view(np.uint32), g["xyz"].view(np.uint32))
