"""Adversarial and hypothesis-driven GPU parity, bit-exact against
the oracle: random sizes, disparity ranges (D in 16Z up to 256, minDisparity < 0), all three modes,
every block size, P1 < P2 up to the int16 domain bound, both uniqueness rules, 3WAY stripe counts,
speckle on/off -- on inputs built to reach the int16 edges where a packed-int16 GPU formulation and
a scalar restatement can part ways: saturated S sums (every disparity at 32767), first-minimum ties
(periodic textures), uniqueness at equality, 0/255 steps and textureless frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from conftest import hyp_examples  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from test_oracle_sgm_volume import p2_domain_max  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def check_case(oracle, kind, H, W, args, nstripes=4, uniq_rule=0, seed=0):
    L, R = S.adversarial_pair(kind, H, W, args[1], seed=seed)
    m = sdr.StereoSGBM.create(*args, nstripes=nstripes, uniq_rule=uniq_rule)
    got = m.compute(L, R)
    p = oracle.make_params(*args, nstripes=nstripes, uniq_rule=uniq_rule)
    ref = oracle.sgbm_compute(L, R, p)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} px differ"
    # the LR-checked map before median/speckle as well
    raw = m.debug_stage(2, (H, W), np.int16)
    assert np.array_equal(raw, oracle.sgbm_compute(L, R, p, stages=0))
    m.close()


@st.composite
def sgbm_cases(draw):
    mode = draw(st.sampled_from([0, 1, 2]))
    D = 16 * draw(st.integers(1, 32))  # up to 512 (four pairs per lane past 256)
    bs = draw(st.sampled_from([1, 3, 5, 7, 9, 11]))
    minD = draw(st.integers(-40, 8))
    H = draw(st.integers(4, 48))
    W1 = draw(st.integers(bs // 2 + 1, 160))  # matched columns (0 < W1 <= SW2 is an OpenCV error)
    W = W1 - min(minD, 0) + max(minD + D, 0)
    cap = draw(st.sampled_from([c for c in (15, 31, 63, 127, 128, 200, 255, 300)
                                if p2_domain_max(bs, c, mode) >= 64]))
    pmax = p2_domain_max(bs, cap, mode)
    P1 = draw(st.integers(1, max(1, min(pmax - 1, 2000))))
    P2 = draw(st.one_of(st.just(pmax), st.integers(P1 + 1, max(P1 + 1, pmax))))
    uniq = draw(st.sampled_from([0, 1, 5, 10, 15, 50]))
    ws = draw(st.sampled_from([0, 0, 10, 100]))
    sr = draw(st.integers(1, 4))
    d12 = draw(st.sampled_from([1, 2, 5, 1000000]))
    kind = draw(st.sampled_from(S.ADVERSARIAL_KINDS))
    return dict(kind=kind, H=H, W=W, args=(minD, D, bs, P1, P2, d12, cap, uniq, ws, sr, mode),
                nstripes=draw(st.sampled_from([1, 2, 3, 4, 8])), uniq_rule=draw(st.integers(0, 2)),
                seed=draw(st.integers(0, 10**6)))


@settings(max_examples=hyp_examples(80), deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(case=sgbm_cases())
def test_hypothesis_bit_exact(oracle, case):
    check_case(oracle, case["kind"], case["H"], case["W"], case["args"], case["nstripes"],
               case["uniq_rule"], case["seed"])


# Deterministic edge cases at medium size (every mode, both int16 extremes of the domain).
EDGE = [
    # kind, H, W, (minD, D, bs, P1, P2, d12, cap, uniq, ws, sr, mode)
    ("binary", 40, 300, (0, 128, 11, 81, p2_domain_max(11, 63, 1), 1, 63, 10, 0, 0, 1)),
    ("binary", 40, 300, (-3, 48, 11, 81, p2_domain_max(11, 63, 0), 1000000, 63, 5, 0, 0, 0)),
    ("binary", 40, 300, (0, 64, 11, 81, p2_domain_max(11, 63, 2), 1, 63, 15, 0, 0, 2)),
    ("noise", 64, 400, (0, 256, 9, 300, p2_domain_max(9, 63, 1), 1, 63, 12, 100, 2, 1)),
    ("noise", 64, 400, (-79, 80, 5, 600, p2_domain_max(5, 63, 2), 1000000, 63, 0, 0, 2, 2)),
    ("periodic", 32, 256, (0, 64, 3, 8, 32, 1, 63, 0, 0, 0, 0)),
    ("periodic", 32, 256, (0, 64, 1, 1, 2, 1, 15, 15, 50, 1, 1)),
    ("steps", 48, 320, (0, 96, 5, 600, 2400, 1, 63, 12, 200, 2, 0)),
    ("steps", 48, 320, (0, 96, 7, 50, 12000, 2, 31, 10, 30, 1, 2)),
    ("flat", 30, 200, (0, 32, 5, 600, 2400, 1, 63, 12, 0, 0, 0)),
    ("flat", 30, 200, (0, 32, 5, 600, 2400, 1, 63, 0, 0, 0, 2)),
    ("textured", 90, 420, (0, 128, 11, 200, p2_domain_max(11, 63, 0), 1, 63, 12, 200, 2, 0)),
]


@pytest.mark.parametrize("kind,H,W,args", EDGE, ids=[f"{e[0]}_m{e[3][10]}_bs{e[3][2]}_P2{e[3][4]}" for e in EDGE])
def test_edge_cases_bit_exact(oracle, kind, H, W, args):
    for rule in (0, 1, 2):
        check_case(oracle, kind, H, W, args, uniq_rule=rule, seed=H * W)


@st.composite
def wide_block_cases(draw):
    """blockSize 13..17: the engine's two-pass cost path (k_hsum_generic / k_vsum_generic)."""
    mode = draw(st.sampled_from([0, 1, 2]))
    bs = draw(st.sampled_from([13, 15, 17]))
    D = 16 * draw(st.integers(1, 16))
    minD = draw(st.integers(-30, 8))
    H = draw(st.integers(4, 40))
    W1 = draw(st.integers(bs // 2 + 1, 120))
    W = W1 - min(minD, 0) + max(minD + D, 0)
    cap = draw(st.sampled_from([c for c in (15, 21, 31) if p2_domain_max(bs, c, mode) >= 64]))
    pmax = p2_domain_max(bs, cap, mode)
    P1 = draw(st.integers(1, max(1, min(pmax - 1, 2000))))
    P2 = draw(st.one_of(st.just(pmax), st.integers(P1 + 1, max(P1 + 1, pmax))))
    kind = draw(st.sampled_from(S.ADVERSARIAL_KINDS))
    return dict(kind=kind, H=H, W=W, args=(minD, D, bs, P1, P2, draw(st.sampled_from([1, 1000000])), cap,
                                            draw(st.sampled_from([0, 10])), draw(st.sampled_from([0, 30])), 2, mode),
                nstripes=draw(st.sampled_from([1, 3, 4])), uniq_rule=draw(st.integers(0, 2)),
                seed=draw(st.integers(0, 10**6)))


@settings(max_examples=hyp_examples(30), deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(case=wide_block_cases())
def test_wide_blocks_bit_exact(oracle, case):
    check_case(oracle, case["kind"], case["H"], case["W"], case["args"], case["nstripes"],
               case["uniq_rule"], case["seed"])


@pytest.mark.parametrize("bs,mode", [(13, 0), (15, 1), (17, 2), (17, 1), (13, 2)])
def test_wide_blocks_domain_edge(oracle, bs, mode):
    """The largest P2 of the int16 domain at 1280-class widths (binary pairs: saturated sums)."""
    args = (0, 128, bs, 81, p2_domain_max(bs, 15, mode), 1, 15, 10, 50, 2, mode)
    check_case(oracle, "binary", 36, 300, args, seed=bs)
    check_case(oracle, "textured", 60, 360, args, seed=bs + 1)


def test_block_19_is_outside_the_domain():
    L = np.zeros((30, 120), np.uint8)
    with pytest.raises(sdr.SDRError) as e:
        sdr.StereoSGBM.create(0, 16, 19, 1, 2, 1, 15).compute(L, L)
    assert e.value.code == -8


def test_outside_int16_domain_is_refused():
    L = np.zeros((20, 100), np.uint8)
    pmax = p2_domain_max(5, 63, 0)
    sdr.StereoSGBM.create(0, 16, 5, 10, pmax, 1, 63).compute(L, L)
    with pytest.raises(sdr.SDRError) as e:
        sdr.StereoSGBM.create(0, 16, 5, 10, pmax + 1, 1, 63).compute(L, L)
    assert e.value.code == -8


def test_one_matcher_two_streams(oracle):
    """A matcher used back to back from two torch streams: the handle orders the second stream
    after the first one's use of its scratch (no overlap, no corruption)."""
    dev = torch.device("cuda", 0)
    args = (0, 64, 5, 600, 2400, 1, 63, 12, 100, 2, 0)
    m = sdr.StereoSGBM.create(*args)
    pairs = [S.make_pair(200, 480, 64, seed=60 + i)[:2] for i in range(4)]
    dl = [(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)) for a, b in pairs]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = []
    for i, (a, b) in enumerate(dl):
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            outs.append(m.compute(a, b))
    torch.cuda.synchronize(dev)
    p = oracle.make_params(*args)
    for (a, b), o in zip(pairs, outs):
        assert np.array_equal(o.cpu().numpy(), oracle.sgbm_compute(a, b, p))


@pytest.mark.parametrize("bs", [7, 9, 11, 13, 17])
def test_3way_short_last_stripes(oracle, bs):
    """MODE_SGBM_3WAY stripes whose every row keeps its window clamped at the stripe start (H-1-SH2
    < s0 + SH2, the short last stripes of small frames at larger block sizes): their output rows'
    horizontal passes run on the stripe's own cost rows (a round-3 fix; found by the wide-block
    tests)."""
    for H in (14, 15, 17, 18, 21, 26):
        for ns in (4, 8):
            args = (0, 32, bs, 10, 500, 1, 15, 10, 0, 2, 2)
            check_case(oracle, "noise", H, 90, args, nstripes=ns, seed=H)


# numDisparities 272..512 (round 3): four disparity pairs per lane in k_paths / the fused WTA
# (its consumers' last lane masked past D), the two-pass cost path, no row sweeps
WIDE_D = [
    # kind, H, W, (minD, D, bs, P1, P2, d12, cap, uniq, ws, sr, mode), nstripes
    ("textured", 40, 620, (0, 512, 5, 600, 2400, 1, 63, 10, 100, 2, 0), 4),
    ("noise", 30, 400, (-20, 272, 3, 8, 200, 1, 31, 5, 0, 0, 1), 4),
    ("binary", 24, 420, (0, 304, 5, 81, p2_domain_max(5, 63, 2), 1000000, 63, 15, 0, 0, 2), 3),
    ("periodic", 20, 520, (0, 384, 7, 50, 1500, 2, 31, 10, 30, 1, 0), 4),
    ("steps", 36, 600, (-5, 496, 1, 10, 100, 1, 63, 0, 0, 0, 3), 4),
    ("textured", 50, 700, (0, 448, 9, 300, 2400, 1, 15, 12, 50, 2, 1), 4),
]


@pytest.mark.parametrize("kind,H,W,args,ns", WIDE_D, ids=[f"{w[0]}_D{w[3][1]}_m{w[3][10]}" for w in WIDE_D])
def test_wide_disparity_range_bit_exact(oracle, kind, H, W, args, ns):
    for rule in (0, 2):
        check_case(oracle, kind, H, W, args, nstripes=ns, uniq_rule=rule, seed=H + W)


def test_wide_disparity_batch_and_colour(oracle):
    """D = 320 on a batch of 3 CV_8UC3 frames: the colour operand sets through the two-pass cost."""
    dev = torch.device("cuda", 0)
    args = (0, 320, 5, 600, 2400, 1, 31, 10, 0, 2, 0)
    frames = [S.make_pair(30, 400, 320, seed=90 + i)[:2] for i in range(3)]
    Lc = np.stack([np.stack([f[0], np.roll(f[0], 1, 1), 255 - f[0]], -1) for f in frames])
    Rc = np.stack([np.stack([f[1], np.roll(f[1], 1, 1), 255 - f[1]], -1) for f in frames])
    m = sdr.StereoSGBM.create(*args)
    got = m.compute(torch.from_numpy(Lc).to(dev), torch.from_numpy(Rc).to(dev)).cpu().numpy()
    p = oracle.make_params(*args)
    for i in range(3):
        assert np.array_equal(got[i], oracle.sgbm_compute(Lc[i], Rc[i], p)), i


def test_disparity_range_past_512_is_refused():
    L = np.zeros((10, 700), np.uint8)
    with pytest.raises(sdr.SDRError) as e:
        sdr.StereoSGBM.create(0, 528, 5, 10, 100, 1, 63).compute(L, L)
    assert e.value.code == -8
