"""Stage-by-stage GPU-vs-oracle diagnostics (cost volume, LR-checked WTA, final)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from stereo_depth_ruler_amd.sgbm import selftest_wave_ops  # noqa: E402


def case(h, w, D, mode, bs=5, minD=0, uniq=12, sp=(0, 0), d12=1, seed=0, P=(600, 2400), cap=63):
    L, R, _ = S.make_pair(h, w, max(D, 16), seed=seed)
    args = (minD, D, bs, P[0], P[1], d12, cap, uniq, sp[0], sp[1], mode)
    m = sdr.StereoSGBM.create(*args)
    t = time.time()
    out = m.compute(L, R)
    tg = time.time() - t
    p = O.make_params(*args)
    w1 = w + min(minD, 0) - max(minD + D, 0)
    C_g = m.debug_cost_volume(h, w1, D)
    lr_g = m.debug_stage(2, (h, w), np.int16)
    res = {}
    if mode != 2:
        C_o = O.cost_volume(L, R, p)
        res["C"] = int((C_g != C_o).sum())
    lr_o = O.sgbm_compute(L, R, p, stages=0)
    res["lr"] = int((lr_g != lr_o).sum())
    fin_o = O.sgbm_compute(L, R, p)
    res["fin"] = int((out != fin_o).sum())
    ok = all(v == 0 for v in res.values())
    print(f"{'OK ' if ok else 'BAD'} h={h} w={w} D={D} mode={mode} bs={bs} minD={minD} uniq={uniq} sp={sp} "
          f"mismatch={res} gpu_s={tg:.3f} valid={(fin_o > (minD-1)*16).mean():.2f}", flush=True)
    if not ok and "lr" in res and res["lr"]:
        ys, xs = np.nonzero(lr_g != lr_o)
        print("   first lr diffs:", [(int(y), int(x), int(lr_g[y, x]), int(lr_o[y, x])) for y, x in zip(ys[:8], xs[:8])])
    if not ok and res.get("C"):
        idx = np.argwhere(C_g != C_o)[:5]
        print("   first C diffs:", [(tuple(int(v) for v in i), int(C_g[tuple(i)]), int(C_o[tuple(i)])) for i in idx])
    return ok


def main():
    print("selftest wave ops failures:", selftest_wave_ops(), flush=True)
    allok = True
    for args in [
        dict(h=32, w=64, D=16, mode=0),
        dict(h=32, w=64, D=16, mode=1),
        dict(h=32, w=64, D=16, mode=2),
        dict(h=40, w=96, D=32, mode=0, bs=3),
        dict(h=48, w=160, D=64, mode=0),
        dict(h=48, w=200, D=128, mode=0),
        dict(h=48, w=200, D=80, mode=2),
        dict(h=60, w=320, D=256, mode=1),
        dict(h=50, w=160, D=48, mode=0, minD=-20),
        dict(h=64, w=200, D=64, mode=0, sp=(50, 2)),
        dict(h=90, w=200, D=80, mode=2, sp=(200, 2)),
        dict(h=45, w=150, D=32, mode=2, bs=7, uniq=5),
        dict(h=120, w=400, D=128, mode=0, sp=(200, 2)),
        dict(h=100, w=333, D=32, mode=1, sp=(30, 1), seed=5),
        dict(h=720, w=1280, D=128, mode=0, sp=(200, 2)),
        dict(h=360, w=640, D=80, mode=2, sp=(200, 2)),
    ]:
        allok &= case(**args)
    print("ALL_OK" if allok else "SOME_FAILED")


if __name__ == "__main__":
    main()
