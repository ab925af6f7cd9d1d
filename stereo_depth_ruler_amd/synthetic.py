"""Seeded synthetic rectified stereo pairs (SURVEY.md section 8d recipe).

The reference's assets (assets/output.mp4, cam.mp4) are git-ignored and absent from the snapshot
(reference .gitignore, .MISSING_LARGE_BLOBS), so every benchmark and parity input is synthetic:

* left: uniform noise blurred by a 5x5 box, contrast-stretched to [0, 255];
* ground-truth disparity: slanted planes in [4, D-8] px, quantised to 1/16 px;
* right: inverse warp of the left view by the ground truth (bilinear) + Gaussian noise sigma=2.
"""
from __future__ import annotations

import numpy as np

# Calibration Q of the reference (config/stereo.yaml:91-97), millimetres.
REFERENCE_Q = np.array([
    [1.0, 0.0, 0.0, -645.44378662109375],
    [0.0, 1.0, 0.0, -347.0967903137207],
    [0.0, 0.0, 0.0, 669.90015369541641],
    [0.0, 0.0, 0.00832541998100415, 0.0],
], dtype=np.float64)


def _box5(a: np.ndarray) -> np.ndarray:
    p = np.pad(a, 2, mode="reflect")
    c = np.cumsum(np.cumsum(p, 0), 1)
    c = np.pad(c, ((1, 0), (1, 0)))
    h, w = a.shape
    return (c[5:5 + h, 5:5 + w] - c[0:h, 5:5 + w] - c[5:5 + h, 0:w] + c[0:h, 0:w]) / 25.0


def texture(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = _box5(rng.uniform(0, 255, size=(h, w)))
    lo, hi = t.min(), t.max()
    return np.clip((t - lo) * (255.0 / max(hi - lo, 1e-6)), 0, 255).astype(np.uint8)


def gt_disparity(h: int, w: int, num_disp: int, seed: int) -> np.ndarray:
    """Piecewise-planar disparity field (px, float32, quantised to 1/16) in [4, D-8]."""
    rng = np.random.default_rng(seed + 1000)
    lo, hi = 4.0, max(float(num_disp) - 8.0, 5.0)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    out = np.empty((h, w))
    # 4 planes split by a vertical line and a slanted line
    xs = rng.uniform(0.35, 0.65) * w
    slope = rng.uniform(-0.3, 0.3)
    region = (xx > xs).astype(int) + 2 * (yy > h * 0.5 + slope * (xx - w / 2)).astype(int)
    for r in range(4):
        base = rng.uniform(lo + 2, hi - 2)
        gx, gy = rng.uniform(-0.01, 0.01, size=2) * (hi - lo)
        plane = base + gx * (xx - w / 2) / w * 8 + gy * (yy - h / 2) / h * 8
        out[region == r] = plane[region == r]
    out = np.clip(out, lo, hi)
    return (np.round(out * 16) / 16).astype(np.float32)


def make_pair(h: int, w: int, num_disp: int, seed: int = 0, noise: float = 2.0):
    """Returns (left u8, right u8, gt disparity f32) for a rectified pair."""
    left = texture(h, w, seed).astype(np.float64)
    gt = gt_disparity(h, w, num_disp, seed).astype(np.float64)
    # right(xr) = left(xr + d): sample disparity at the right pixel (slanted planes ~ smooth)
    xr = np.arange(w, dtype=np.float64)[None, :] + gt
    x0 = np.floor(xr).astype(np.int64)
    fx = xr - x0
    x0c = np.clip(x0, 0, w - 1)
    x1c = np.clip(x0 + 1, 0, w - 1)
    rows = np.arange(h)[:, None]
    right = left[rows, x0c] * (1 - fx) + left[rows, x1c] * fx
    rng = np.random.default_rng(seed + 1)
    right = right + rng.normal(0.0, noise, size=right.shape)
    right = np.clip(np.round(right), 0, 255).astype(np.uint8)
    return left.astype(np.uint8), right, gt.astype(np.float32)


def make_batch(n: int, h: int, w: int, num_disp: int, seed0: int = 0):
    L = np.empty((n, h, w), np.uint8)
    R = np.empty((n, h, w), np.uint8)
    for i in range(n):
        L[i], R[i], _ = make_pair(h, w, num_disp, seed0 + i)
    return L, R


def shifted_pair(h: int, w: int, shift: int, seed: int = 0):
    """Constant-disparity pair: right(x) = left(x + shift) (exact integer shift, no noise)."""
    big = texture(h, w + shift + 8, seed)
    left = big[:, :w].copy()
    right = big[:, shift:shift + w].copy()
    # right(xr) = big(xr + shift) = left(xr + shift)  =>  left(x) matches right(x - shift)
    return left, right


ADVERSARIAL_KINDS = ("noise", "binary", "steps", "periodic", "flat", "textured")


def adversarial_pair(kind: str, h: int, w: int, num_disp: int = 16, seed: int = 0):
    """Pairs that push the int16 cost arithmetic to its edges (parity tests only):

    * noise: independent uniform noise left and right (large block costs, no true match);
    * binary: independent 0/255 pixels (the largest BT cost per pixel, so C, L_r and the
      saturated S sum reach their maxima);
    * steps: 0/255 vertical bars of random widths, identical rows (ties along x, flat columns);
    * periodic: a horizontal period dividing the disparity range, the right view shifted by a
      whole period (several disparities match exactly: first-minimum ties, uniqueness at equality);
    * flat: one constant grey level (every cost equal);
    * textured: the section 8d pair (make_pair)."""
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return (rng.integers(0, 256, (h, w), dtype=np.uint8),
                rng.integers(0, 256, (h, w), dtype=np.uint8))
    if kind == "binary":
        return (rng.integers(0, 2, (h, w), dtype=np.uint8) * 255,
                rng.integers(0, 2, (h, w), dtype=np.uint8) * 255)
    if kind == "steps":
        edges = np.cumsum(rng.integers(1, 9, size=w + 1))
        bars = (np.searchsorted(edges, np.arange(w + 8), side="right") & 1).astype(np.uint8) * 255
        left = np.tile(bars[:w], (h, 1))
        s = int(rng.integers(1, max(2, min(num_disp, 8))))
        return left, np.tile(bars[s:s + w], (h, 1))
    if kind == "periodic":
        period = int(rng.choice([2, 4, 8]))
        base = rng.integers(0, 256, size=period).astype(np.uint8)
        row = base[np.arange(w + period) % period]
        left = np.tile(row[:w], (h, 1))
        return left, np.tile(row[period:period + w], (h, 1))
    if kind == "flat":
        v = np.uint8(rng.integers(0, 256))
        return np.full((h, w), v, np.uint8), np.full((h, w), v, np.uint8)
    if kind == "textured":
        left, right, _ = make_pair(h, w, max(num_disp, 16), seed=seed)
        return left, right
    raise ValueError(kind)


def sbs_bgr_frame(h: int, w: int, num_disp: int, seed: int = 0):
    """A ZED2-style side-by-side BGR frame (2w x h x 3) with gray replicated over channels."""
    left, right, _ = make_pair(h, w, num_disp, seed)
    frame = np.empty((h, 2 * w, 3), np.uint8)
    frame[:, :w, :] = left[:, :, None]
    frame[:, w:, :] = right[:, :, None]
    return frame


def sbs_bgr_color_frame(h: int, w: int, num_disp: int, seed: int = 0):
    """A ZED2-style side-by-side BGR frame (h x 2w x 3) whose channels differ: B = the seeded gray
    view, G = the view shifted by one column, R = seeded noise (so BGR2GRAY is exercised)."""
    left, right, _ = make_pair(h, w, num_disp, seed)
    rng = np.random.default_rng(seed + 7)
    frame = np.empty((h, 2 * w, 3), np.uint8)
    for k, v in enumerate((left, right)):
        frame[:, k * w:(k + 1) * w, 0] = v
        frame[:, k * w:(k + 1) * w, 1] = np.roll(v, 1, 1)
        frame[:, k * w:(k + 1) * w, 2] = rng.integers(0, 256, v.shape, dtype=np.uint8)
    return frame
