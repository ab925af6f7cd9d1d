"""Independent numpy restatements of single stages (vectorised, written from the published
formulas, not from oracle/sgbm_oracle.c) used to pin the C oracle.  Test helpers only."""
import numpy as np


def prefilter_channels(img, ftzero):
    """x-Sobel clipped to [0, 2*ftzero] and raw intensity; cols 0 / W-1 = ftzero (tab[0]).  The
    clip table holds uchar values: past preFilterCap 127 they wrap mod 256."""
    I = img.astype(np.int32)
    H, W = I.shape
    up = np.vstack([I[:1], I[:-1]])
    dn = np.vstack([I[1:], I[-1:]])
    sob = np.full((H, W), ftzero & 0xff, np.int32)
    raw = np.full((H, W), ftzero & 0xff, np.int32)
    g = 2 * (I[:, 2:] - I[:, :-2]) + (up[:, 2:] - up[:, :-2]) + (dn[:, 2:] - dn[:, :-2])
    sob[:, 1:-1] = (np.clip(g, -ftzero, ftzero) + ftzero) & 0xff
    raw[:, 1:-1] = I[:, 1:-1]
    return sob, raw


def cost_channels(img, ftzero):
    """calcPixelCostBT's channels with their cost shifts: gray -> (sobel, 0), (raw, 2); an
    interleaved 3-channel image -> the three sobels (shift 0), then the three raws (shift 2)."""
    if img.ndim == 2:
        s, r = prefilter_channels(img, ftzero)
        return [(s, 0), (r, 2)]
    per = [prefilter_channels(img[:, :, c], ftzero) for c in range(img.shape[2])]
    return [(s, 0) for s, _ in per] + [(r, 2) for _, r in per]


def envelope(ch):
    """(lo, hi) over the value and its two half-sample neighbours (truncating average)."""
    W = ch.shape[1]
    a = ch.copy()
    b = ch.copy()
    a[:, :-1] = (ch[:, :-1] + ch[:, 1:]) // 2
    b[:, 1:] = (ch[:, 1:] + ch[:, :-1]) // 2
    return np.minimum(np.minimum(a, b), ch), np.maximum(np.maximum(a, b), ch)


def bt_cost_volume_rows(L, R, minD, D, ftzero):
    """Pixel cost [H][W1][D] = sum over channels of BT(sobel) + (BT(raw) >> 2)."""
    H, W = L.shape[:2]
    maxD = minD + D
    minX1, maxX1 = max(maxD, 0), W + min(minD, 0)
    out = np.zeros((H, maxX1 - minX1, D), np.int32)
    xs = np.arange(minX1, maxX1)
    for (u, scale), (v, _) in zip(cost_channels(L, ftzero), cost_channels(R, ftzero)):
        u0, u1 = envelope(u)
        v0, v1 = envelope(v)
        for di, d in enumerate(range(minD, maxD)):
            xr = xs - d
            uu, uu0, uu1 = u[:, xs], u0[:, xs], u1[:, xs]
            vv, vv0, vv1 = v[:, xr], v0[:, xr], v1[:, xr]
            c0 = np.maximum(0, np.maximum(uu - vv1, vv0 - uu))
            c1 = np.maximum(0, np.maximum(vv - uu1, uu0 - vv))
            out[:, :, di] += np.minimum(c0, c1) >> scale
    return out


def cost_volume(L, R, minD, D, bs, P2, ftzero, hh=False):
    """P2 + box(bs x bs) of the pixel costs with OpenCV's border rules (replicate inside
    [0, W1) x [0, H); rows past H-1-SH2 repeat row H-1-SH2, or stay P2 for MODE_HH)."""
    pix = bt_cost_volume_rows(L, R, minD, D, ftzero)
    H, W1, _ = pix.shape
    s = bs // 2
    xi = np.clip(np.arange(W1)[:, None] + np.arange(-s, s + 1)[None, :], 0, W1 - 1)
    hs = pix[:, xi, :].sum(2)
    C = np.empty_like(hs)
    ylim = max(H - 1 - s, 0)
    for y in range(H):
        if hh and y > 0 and y + s >= H:
            C[y] = 0
            continue
        t = min(y, ylim)
        rows = np.clip(np.arange(t - s, t + s + 1), 0, H - 1)
        C[y] = hs[rows].sum(0)
    return (C + P2).astype(np.int16)


# ---- StereoSGBM A.4-A.9: a materialised-volume formulation ----
#
# A second, structurally different statement of the SGM core, written from the published rules
# and not from oracle/sgbm_oracle.c: the cost volume is a direct (non-running) box sum, every path
# direction is its own full [H][W1][D] volume computed in int64 with no int16 storage, S is an
# explicit saturated sum, and the WTA / uniqueness / subpixel / disp2 / LR rules are vectorised over
# whole rows.  The oracle instead follows OpenCV's row drivers (ring buffers, running sums, packed
# per-pixel loops).  Agreement between the two pins the oracle's transcription of A.4-A.9.

SGM_SGBM, SGM_HH, SGM_3WAY, SGM_HH4 = 0, 1, 2, 3
_BIG = 1 << 40  # the d = -1 / d = D neighbours: never the minimum

# predecessor offsets: the predecessor of (x, y) along r is (x - dx, y - dy)
SGM_DIRS = {
    SGM_SGBM: [(1, 0), (1, 1), (0, 1), (-1, 1), (-1, 0)],
    SGM_HH: [(1, 0), (1, 1), (0, 1), (-1, 1), (-1, 0), (-1, -1), (0, -1), (1, -1)],
    SGM_3WAY: [(1, 0), (-1, 0), (0, 1)],
    SGM_HH4: [(1, 0), (-1, 0), (0, 1), (0, -1)],
}


def sgm_effective(minD, D, bs, P1, P2, d12, cap, uniq, mode, uniq_rule=0):
    """OpenCV's parameter defaulting (StereoSGBM::create / computeDisparitySGBM /
    SGBM3WayMainLoop): returns a dict of the values the algorithm actually uses."""
    if mode == SGM_3WAY:
        sw2 = bs // 2 if bs > 0 else 1
    else:
        sw2 = (bs if bs > 0 else 5) // 2
    p1 = P1 if P1 > 0 else 2
    p2 = max(P2 if P2 > 0 else 5, p1 + 1)
    u = uniq if uniq >= 0 else 10
    simd = {1: False, 2: True}.get(uniq_rule, mode == SGM_3WAY)
    return dict(minD=minD, D=D, maxD=minD + D, SW2=sw2, SH2=sw2, P1=p1, P2=p2,
                d12=d12 if d12 > 0 else 1, ftzero=max(cap, 15) | 1, uniq=u, simd=simd, bs=bs)


def _box_rows(hs, s0, end, SH2, hh_bottom):
    """Box-summed rows [s0, end) of a chain whose vertical window clamps at s0 (top) and H-1
    (bottom); rows whose window would pass the bottom repeat the last full window (or, for
    MODE_HH's full-DP buffer, stay 0)."""
    H = hs.shape[0]
    out = np.zeros((end - s0,) + hs.shape[1:], np.int64)
    ylim = max(H - 1 - SH2, s0)
    for y in range(s0, end):
        if hh_bottom and y > 0 and y + SH2 >= H:
            continue
        t = min(y, ylim)
        rows = np.clip(np.arange(t - SH2, t + SH2 + 1), s0, H - 1)
        out[y - s0] = hs[rows].sum(0)
    return out


def _path_volume(C, dx, dy, P1, P2):
    """L_r(p, d) = C(p, d) + min(Lp(d), Lp(d-1) + P1, Lp(d+1) + P1, minLp + P2) - (minLp + P2),
    with Lp the predecessor's L (0 and minLp = 0 before a chain's first pixel), as a full volume."""
    H, W1, D = C.shape
    L = np.zeros_like(C)

    def step(c, lp, mlp):
        delta = (mlp + P2)[..., None]
        pad = np.full(lp.shape[:-1] + (D + 2,), _BIG, np.int64)
        pad[..., 1:-1] = lp
        nb = np.minimum(pad[..., :-2], pad[..., 2:]) + P1
        return c + np.minimum(np.minimum(lp, nb), delta) - delta

    if dy == 0:
        lp = np.zeros((H, D), np.int64)
        for x in (range(W1) if dx > 0 else range(W1 - 1, -1, -1)):
            L[:, x] = step(C[:, x], lp, lp.min(-1))  # zeros before the first pixel: minLp = 0
            lp = L[:, x]
        return L
    src = np.arange(W1) - dx
    ok = (src >= 0) & (src < W1)
    prev = None
    for y in (range(H) if dy > 0 else range(H - 1, -1, -1)):
        lp = np.zeros((W1, D), np.int64)
        mlp = np.zeros(W1, np.int64)
        if prev is not None:
            lp[ok] = prev[src[ok]]
            mlp[ok] = prev[src[ok]].min(-1)
        L[y] = step(C[y], lp, mlp)
        prev = L[y]
    return L


def _c_div(n, d):
    """C integer division (truncation toward zero), d > 0."""
    return np.sign(n) * (np.abs(n) // d)


def _wta_rows(S, e, W, minX1):
    """A.8 + A.9 on saturated sums S [rows][W1][D] -> disparity rows [rows][W] (1/16 px)."""
    rows, W1, D = S.shape
    inv = (e["minD"] - 1) * 16
    out = np.full((rows, W), inv, np.int64)
    best = S.argmin(-1)  # first minimum
    minS = S.min(-1)
    dd = np.arange(D)
    far = np.abs(dd[None, None, :] - best[..., None]) > 1
    if e["simd"]:
        if e["uniq"] > 0:
            thr = (100 * minS) // (100 - e["uniq"]) + 1
            thr = ((thr + 32768) % 65536) - 32768  # (short)(thresh + 1)
            reject = ((S < thr[..., None]) & far).any(-1)
        else:
            reject = np.zeros(best.shape, bool)
    else:
        reject = ((S * (100 - e["uniq"]) < minS[..., None] * 100) & far).any(-1)
    # the first-minimum scan starts from (MAX_COST, bestDisp = -1) with a strict '<': a pixel whose
    # every S saturated keeps bestDisp = -1, i.e. the value (-1 + minD) * 16 = INVALID, and its
    # disp2 candidate (cost MAX_COST) never replaces the initial one
    reject |= minS >= 32767
    inner = (best > 0) & (best < D - 1)
    bm = np.clip(best - 1, 0, D - 1)
    bp = np.clip(best + 1, 0, D - 1)
    Sm = np.take_along_axis(S, bm[..., None], -1)[..., 0]
    Sp = np.take_along_axis(S, bp[..., None], -1)[..., 0]
    den = np.maximum(Sm + Sp - 2 * minS, 1)
    d16 = best * 16 + np.where(inner, _c_div((Sm - Sp) * 16 + den, 2 * den), 0) + e["minD"] * 16
    xs = np.arange(W1)
    for r in range(rows):
        acc = ~reject[r]
        out[r, minX1 + xs[acc]] = d16[r, acc]
        # disp2: right-view WTA; per target column the smallest minS wins, ties -> the largest x
        # (OpenCV scans x descending and replaces only on a strictly smaller cost)
        disp2 = np.full(W, inv, np.int64)
        xa = xs[acc]
        x2 = xa + minX1 - best[r, acc] - e["minD"]
        inr = (x2 >= 0) & (x2 < W)
        xa, x2, ms, b = xa[inr], x2[inr], minS[r, acc][inr], best[r, acc][inr]
        order = np.lexsort((-xa, ms, x2))
        first = np.ones(order.size, bool)
        first[1:] = x2[order][1:] != x2[order][:-1]
        win = order[first]
        disp2[x2[win]] = b[win] + e["minD"]
        # A.9: invalidate when both floor/ceil correspondences disagree by more than disp12MaxDiff
        d1 = out[r]
        xx = np.arange(W)
        chk = (xx >= minX1) & (xx < minX1 + W1) & (d1 != inv)
        lo, hi = d1 >> 4, (d1 + 15) >> 4
        bad = np.ones(W, bool)
        for dv in (lo, hi):
            xs2 = xx - dv
            inb = (xs2 >= 0) & (xs2 < W)
            t = disp2[np.clip(xs2, 0, W - 1)]
            bad &= inb & (t >= e["minD"]) & (np.abs(t - dv) > e["d12"])
        out[r, chk & bad] = inv
    return out


def sgm_full_volume(L, R, minD, D, bs, P1, P2, d12, cap, uniq, ws=0, sr=0, mode=SGM_SGBM,
                    nstripes=4, uniq_rule=0, stages=3):
    """StereoSGBM::compute as a materialised-volume formulation.  stages: 1 median, 2 speckle."""
    e = sgm_effective(minD, D, bs, P1, P2, d12, cap, uniq, mode, uniq_rule)
    H, W = L.shape[:2]
    minX1, maxX1 = max(e["maxD"], 0), W + min(minD, 0)
    W1 = maxX1 - minX1
    inv = (minD - 1) * 16
    if W1 <= 0:
        return np.full((H, W), inv, np.int16)
    pix = bt_cost_volume_rows(L, R, minD, D, e["ftzero"]).astype(np.int64)
    s = e["SW2"]
    xi = np.clip(np.arange(W1)[:, None] + np.arange(-s, s + 1)[None, :], 0, W1 - 1)
    hs = pix[:, xi, :].sum(2)
    if mode == SGM_3WAY:
        segs = []
        sz = int(np.ceil(H / nstripes))
        overlap = (bs // 2 + 1) + int(np.ceil(0.1 * sz))
        for k in range(nstripes):
            if k * sz >= H:
                break
            segs.append((max(min(k * sz - overlap, H), 0), min((k + 1) * sz, H), k * sz))
    else:
        segs = [(0, H, 0)]
    raw = np.full((H, W), inv, np.int64)
    for s0, end, out0 in segs:
        C = e["P2"] + _box_rows(hs, s0, end, e["SH2"], mode in (SGM_HH, SGM_HH4))
        assert C.max() <= 32767, "outside the int16 cost domain"
        Ssum = np.zeros_like(C)
        for dx, dy in SGM_DIRS[mode]:
            Lr = _path_volume(C, dx, dy, e["P1"], e["P2"])
            assert Lr.min() >= 0 and Lr.max() <= 32767
            Ssum += Lr
        Ssum = np.minimum(Ssum, 32767)
        raw[out0:end] = _wta_rows(Ssum[out0 - s0:], e, W, minX1)
    out = raw.astype(np.int16)
    if stages & 1:
        from scipy.ndimage import median_filter
        out = median_filter(out, size=3, mode="nearest")
    if (stages & 2) and ws > 0:
        out = speckle_filter(out, inv, ws, 16 * sr)
    return out


def speckle_filter(img, new_val, max_size, max_diff):
    """Components by BFS over 4-neighbours joined when both != new_val and |diff| <= max_diff."""
    H, W = img.shape
    out = img.copy()
    lab = -np.ones((H, W), np.int64)
    n = 0
    v = img.astype(np.int32)
    for y0 in range(H):
        for x0 in range(W):
            if v[y0, x0] == new_val or lab[y0, x0] >= 0:
                continue
            stack = [(y0, x0)]
            lab[y0, x0] = n
            comp = []
            while stack:
                y, x = stack.pop()
                comp.append((y, x))
                for yy, xx in ((y + 1, x), (y - 1, x), (y, x + 1), (y, x - 1)):
                    if 0 <= yy < H and 0 <= xx < W and lab[yy, xx] < 0 and v[yy, xx] != new_val \
                            and abs(v[y, x] - v[yy, xx]) <= max_diff:
                        lab[yy, xx] = n
                        stack.append((yy, xx))
            if len(comp) <= max_size:
                for y, x in comp:
                    out[y, x] = new_val
            n += 1
    return out


def reproject(disp, Q, handle_missing=False):
    """float64 Q @ (x, y, d, 1), sequential sums, Vec3f then * (1/w), Z=10000 at min(disp)."""
    H, W = disp.shape
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    d = disp.astype(np.float64)
    h = []
    for i in range(4):
        s = np.zeros_like(d)
        s = s + Q[i, 0] * x
        s = s + Q[i, 1] * y
        s = s + Q[i, 2] * d
        s = s + Q[i, 3] * 1.0
        h.append(s)
    ia = 1.0 / h[3]
    with np.errstate(all="ignore"):
        out = np.stack([(h[i].astype(np.float32).astype(np.float64) * ia).astype(np.float32)
                        for i in range(3)], -1)
    if handle_missing:
        m = float(disp.min())
        out[..., 2][np.abs(d - m) <= np.finfo(np.float32).eps] = 10000.0
    return out


# ---- DisparityWLSFilter / FastGlobalSmootherFilter, float64 (independent of wls_oracle.c) ----

def fgs_weights(guide, sigma):
    """4-neighbour weights w = exp(-|dI|/sigma): (horizontal [h, w-1], vertical [h-1, w])."""
    g = guide.astype(np.float64)
    return np.exp(-np.abs(np.diff(g, axis=1)) / sigma), np.exp(-np.abs(np.diff(g, axis=0)) / sigma)


def _solve_lines(f, wgt, lam):
    """Rows of f: (I + lam * L_w) u = f with L_w the 1-D weighted path Laplacian (Neumann)."""
    from scipy.linalg import solve_banded

    n = f.shape[1]
    out = np.empty_like(f)
    for r in range(f.shape[0]):
        w = wgt[r]
        diag = np.ones(n)
        diag[:-1] += lam * w
        diag[1:] += lam * w
        ab = np.zeros((3, n))
        ab[0, 1:] = -lam * w
        ab[1] = diag
        ab[2, :-1] = -lam * w
        out[r] = solve_banded((1, 1), ab, f[r])
    return out


def fgs_filter(guide, img, lam, sigma, attenuation=0.25, num_iter=3):
    wh, wv = fgs_weights(guide, sigma)
    u = img.astype(np.float64)
    for _ in range(num_iter):
        u = _solve_lines(u, wh, lam)
        u = _solve_lines(u.T, wv.T, lam).T
        lam *= attenuation
    return u


def _reflect101(idx, n):
    if n == 1:
        return np.zeros_like(idx)
    idx = np.abs(idx)
    period = 2 * n - 2
    idx = idx % period
    return np.where(idx >= n, period - idx, idx)


def wls_disc_map(d, roi, radius, roll_off=0.001):
    x, y, w, h = roi
    out = np.ones(d.shape, np.float64)
    if w <= 0 or h <= 0:
        return out
    sub = d[y:y + h, x:x + w].astype(np.float64)
    rr = _reflect101(np.arange(-radius, h + radius), h)
    cc = _reflect101(np.arange(-radius, w + radius), w)
    pad = sub[rr][:, cc]
    k = 2 * radius + 1
    win = np.lib.stride_tricks.sliding_window_view(pad, (k, k))
    mean = win.mean(axis=(-1, -2))
    msq = (win ** 2).mean(axis=(-1, -2))
    out[y:y + h, x:x + w] = np.maximum(1.0 - roll_off * (msq - mean ** 2), 0.0)
    return out


def wls_confidence(dl, dr, roi, radius, lrc_thresh=24, roll_off=0.001):
    x, y, w, h = roi
    W = dl.shape[1]
    rroi = (W - (x + w), y, w, h)
    cl = wls_disc_map(dl, roi, radius, roll_off)
    cr = wls_disc_map(dr, rroi, radius, roll_off)
    conf = cl.copy()
    rows = np.arange(dl.shape[0])[:, None]
    cols = np.arange(x, x + w)[None, :]
    lv = dl[:, x:x + w].astype(np.int64)
    ridx = cols - (lv >> 4)
    inr = (ridx >= rroi[0]) & (ridx < rroi[0] + rroi[2])
    rc = np.clip(ridx, 0, W - 1)
    ok = np.abs(lv + dr[rows, rc].astype(np.int64)) < lrc_thresh
    sub = conf[:, x:x + w]
    sub[inr & ok] = np.minimum(cl[:, x:x + w], cr[rows, rc])[inr & ok]
    sub[inr & ~ok] = 0.0
    return 255.0 * conf


def wls_filter(dl, dr, guide, roi, radius, lam, sigma, min_disp, lrc_thresh=24):
    x, y, w, h = roi
    conf = wls_confidence(dl, dr, roi, radius, lrc_thresh)
    out = np.full(dl.shape, 16 * (min_disp - 1), np.float64)
    c = conf[y:y + h, x:x + w]
    g = guide[y:y + h, x:x + w]
    num = fgs_filter(g, c * dl[y:y + h, x:x + w], lam, sigma)
    den = fgs_filter(g, c, lam, sigma)
    out[y:y + h, x:x + w] = np.where(den != 0, num / np.where(den != 0, den, 1), 0)
    return out


# ---- initUndistortRectifyMap / remap (independent vectorised restatement) ----

def undistort_rectify_uv(K, dist, R, P):
    """Per-pixel (u, v) source coordinates of cv::initUndistortRectifyMap in float64, with
    x/y/w evaluated directly per pixel (OpenCV accumulates them along the row; the two agree to
    a few ulp), returned as functions of the (H, W) grid."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    R = np.asarray(R, np.float64).reshape(3, 3)
    P = np.asarray(P, np.float64)
    P = P.reshape(3, -1)[:, :3]
    iR = np.linalg.inv(P @ R)
    k = np.zeros(14)
    d = np.asarray(dist, np.float64).reshape(-1)
    k[:d.size] = d
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = k[:12]

    def uv(H, W):
        i, j = np.mgrid[0:H, 0:W].astype(np.float64)
        X = j * iR[0, 0] + i * iR[0, 1] + iR[0, 2]
        Y = j * iR[1, 0] + i * iR[1, 1] + iR[1, 2]
        Wh = j * iR[2, 0] + i * iR[2, 1] + iR[2, 2]
        x, y = X / Wh, Y / Wh
        r2 = x * x + y * y
        kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
        xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x) + s1 * r2 + s2 * r2 * r2
        yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y + s3 * r2 + s4 * r2 * r2
        return K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]
    return uv


def remap_bilinear(src, map1, map2):
    """cv::remap INTER_LINEAR BORDER_CONSTANT(0) with CV_16SC2 maps, 8-bit, vectorised."""
    src = np.asarray(src)
    img = src[..., None] if src.ndim == 2 else src
    H, W, C = img.shape
    sx = map1[..., 0].astype(np.int64)
    sy = map1[..., 1].astype(np.int64)
    ax = (map2 & 31).astype(np.int64)
    ay = (map2.astype(np.int64) >> 5) & 31
    acc = np.zeros(map2.shape + (C,), np.int64)
    for dy, dx, w in ((0, 0, (32 - ax) * (32 - ay)), (0, 1, ax * (32 - ay)),
                      (1, 0, (32 - ax) * ay), (1, 1, ax * ay)):
        xx, yy = sx + dx, sy + dy
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = img[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)].astype(np.int64)
        acc += np.where(ok[..., None], v, 0) * (w * 32)[..., None]
    out = np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)
    return out[..., 0] if src.ndim == 2 else out
