"""Kernel A/B harness: several builds of the engine in ONE process, interleaved rounds, per-kernel
HIP-event timing (sdr_sgbm_kernel_time) on the same resident inputs, plus a bit-exactness check of
every build's output against the first one.

    python scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so lib/libsdr-x.so [--config c2]

Each library is loaded through its own ctypes handle (RTLD_LOCAL), so the builds do not share
symbols; the inputs are torch tensors on cuda:0.  Experiment builds come from
`python -m stereo_depth_ruler_amd.build <variant> NAME=VALUE ...`.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereo_depth_ruler_amd import _lib  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

CONFIGS = {  # W, H, D, mode, frames
    "c2": (1280, 720, 128, 0, 1),
    "c3": (1280, 720, 256, 1, 8),
    "c0": (640, 360, 80, 2, 1),
    "c5": (1920, 1080, 256, 1, 1),
    "c4": (640, 360, 80, 2, 2),  # the class path's two matchers as two frames (1440 E/W chains)
    "c5b8": (1920, 1080, 256, 1, 8),  # C5 as benched: 8 frames through the row sweeps
    "hh128": (1280, 720, 128, 1, 8),  # the sweeps at two disparities per lane
    "c3b32": (1280, 720, 256, 1, 32),  # C3 as benched: 32 frames per call
}
KINDS = ["prefilter", "k_cost", "k_paths", "k_south_wta", "median", "speckle", "reproject", "k_lr_check",
         "k_sweep", "k_wls_prep", "fgs_pass", "k_wls_final", "k_sweep_down"]  # SDR_KERNEL_* order


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, res, args in _lib.SIGNATURES:
        fn = getattr(L, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    W, H, D, mode, F = CONFIGS[a.config]
    Ls, Rs = S.make_batch(F, H, W, D, seed0=100)
    dev = torch.device("cuda", 0)
    dl, dr = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    libs = [load(p) for p in a.libs]
    params = _lib.SgbmParams(0, D, 5, 600, 2400, 1, 63, 12, 200, 2, mode, 4, 0)
    handles, outs = [], []
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for L in libs:
        h = ctypes.c_void_p()
        assert L.sdr_sgbm_create(ctypes.byref(params), 0, ctypes.byref(h)) == 0, L.sdr_last_error()
        L.sdr_sgbm_set_stream(h, stream)
        handles.append(h)
        outs.append(torch.empty((F, H, W), dtype=torch.int16, device=dev))
    res = {p: {k: [] for k in KINDS + ["frame"]} for p in a.libs}
    for r in range(a.rounds):
        for p, L, h, o in zip(a.libs, libs, handles, outs):
            run = lambda: L.sdr_sgbm_compute_device(h, dl.data_ptr(), dr.data_ptr(), W, H, W, W * H, F,
                                                    o.data_ptr(), W, W * H)
            for _ in range(3):
                assert run() == 0, L.sdr_last_error()
            L.sdr_sgbm_enable_timing(h, 2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[p]["frame"].append(e0.elapsed_time(e1) * 1000 / a.iters / F)
            for kind, name in enumerate(KINDS):
                t, n = ctypes.c_float(), ctypes.c_int()
                L.sdr_sgbm_kernel_time(h, kind, 0, ctypes.byref(t), ctypes.byref(n))
                if n.value:
                    res[p][name].append(t.value * 1000 / n.value)
            L.sdr_sgbm_enable_timing(h, 0)
    ref = outs[0].cpu().numpy()
    print(f"config {a.config}: W={W} H={H} D={D} mode={mode} frames/call={F}; us (median of {a.rounds} rounds)")
    cols = ["frame"] + [k for k in KINDS if any(res[p][k] for p in a.libs)]
    print(f"{'lib':40s} " + " ".join(f"{c:>11s}" for c in cols) + "  exact")
    for p, o in zip(a.libs, outs):
        same = np.array_equal(o.cpu().numpy(), ref)
        vals = [np.median(res[p][c]) if res[p][c] else float("nan") for c in cols]
        print(f"{os.path.basename(p):40s} " + " ".join(f"{v:11.1f}" for v in vals) + f"  {same}")


if __name__ == "__main__":
    main()
