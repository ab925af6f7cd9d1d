"""FGS (fastGlobalSmootherFilter) device timing on the class path's shape: two right-hand sides of
one 560x360 ROI (the C0/C4 WLS filter), both solvers.
python scripts/fgs_bench.py [iters] [--lib PATH] [--thomas-only] [--noise-guide]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from stereo_depth_ruler_amd.ximgproc import FGS_PCR, FGS_THOMAS, fastGlobalSmootherFilter  # noqa: E402

args = sys.argv[1:]
if "--lib" in args:
    from stereo_depth_ruler_amd import _lib  # noqa: E402

    i = args.index("--lib")
    _lib.use_library(args[i + 1])
    del args[i:i + 2]
only = "--thomas-only" in args
noise = "--noise-guide" in args
args = [a for a in args if a not in ("--thomas-only", "--noise-guide")]
it = int(args[0]) if args else 50
rng = np.random.default_rng(0)
h, w = 360, 560
dev = torch.device("cuda", 0)
# the guide: the synthetic scene's left view (the matcher's input; --noise-guide: uniform noise,
# every neighbour pair a random step, the sequential solver's slowest case)
if noise:
    g = torch.from_numpy(rng.integers(0, 256, (h, w)).astype(np.uint8)).to(dev)
else:
    from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

    g = torch.from_numpy(np.ascontiguousarray(S.make_pair(h, w, 64, seed=3)[0])).to(dev)
x = torch.from_numpy((rng.random((2, h, w)) * 1000).astype(np.float32)).to(dev)
for solver, name in ((FGS_PCR, "pcr"), (FGS_THOMAS, "thomas"))[1 if only else 0:]:
    for _ in range(3):
        fastGlobalSmootherFilter(g, x, 8000.0, 1.1, solver=solver)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fastGlobalSmootherFilter(g, x, 8000.0, 1.1, solver=solver)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / it * 1e6:.1f} us per call (3 iterations, 2 images, host sync per call)")
