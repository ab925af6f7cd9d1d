"""Batched MODE_HH through the row-synchronous sweeps (k_sweep: N/NE/NW up, SE/SW down, one
record each) against the oracle, frame by frame.  Batches of >= 8 frames take the sweep path;
single frames take k_paths' per-direction chains, so the two formulations are also compared with
each other.  Shapes cover one tile and partial last tiles (kSweepTile = 32 columns), padded
disparity lanes (D < 64 * DPL at both lane widths) and the int16 extremes (binary / noise pairs:
saturated sums)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import stereo_depth_ruler_amd as sdr  # noqa: E402
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402


def _batch(kind, F, H, W, D, seed):
    Ls = np.empty((F, H, W), np.uint8)
    Rs = np.empty((F, H, W), np.uint8)
    for i in range(F):
        if kind == "textured":
            Ls[i], Rs[i], _ = S.make_pair(H, W, D, seed + i)
        else:
            Ls[i], Rs[i] = S.adversarial_pair(kind, H, W, D, seed=seed + i)
    return Ls, Rs


@pytest.mark.parametrize("kind,F,H,W,D,speckle,seed", [
    ("textured", 8, 40, 200, 64, 30, 1),    # 5 tiles, the last partial (W1 = 136)
    ("textured", 9, 33, 90, 48, 0, 2),      # one tile + 10 columns, D padded (DPL 2)
    ("noise", 8, 24, 60, 32, 0, 3),         # W1 = 28: a single partial tile
    ("binary", 8, 30, 120, 16, 0, 4),       # saturated S sums
    ("textured", 8, 26, 260, 160, 20, 5),   # DPL 4 with padded lanes
    ("steps", 10, 20, 100, 32, 0, 6),
    ("textured", 8, 18, 192, 32, 0, 7),     # W1 = 160: whole tiles only (80 columns)
    ("textured", 8, 24, 300, 128, 0, 8),    # DPL 2 without padded lanes
    ("noise", 8, 20, 400, 256, 10, 9),      # DPL 4 without padded lanes (C3 / C5's D)
    ("binary", 8, 16, 380, 256, 0, 10),     # the same at the int16 extremes
])
def test_hh_sweep_batch_bit_exact(oracle, kind, F, H, W, D, speckle, seed):
    args = (0, D, 5, 600, 2400, 1, 63, 10, speckle, 2, sdr.MODE_HH)
    Ls, Rs = _batch(kind, F, H, W, D, seed)
    dev = torch.device("cuda", 0)
    m = sdr.StereoSGBM.create(*args)
    out = m.compute(torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)).cpu().numpy()
    p = oracle.make_params(*args)
    for i in range(F):
        ref = oracle.sgbm_compute(Ls[i], Rs[i], p)
        assert np.array_equal(out[i], ref), f"frame {i}: {(out[i] != ref).sum()} px differ"
    # the same frames one at a time (k_paths' chains) and again as a batch on the same handle
    # (the sweep's counters and edge rings start over every call)
    for i in (0, F - 1):
        assert np.array_equal(m.compute(Ls[i], Rs[i]), out[i])
    again = m.compute(torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)).cpu().numpy()
    assert np.array_equal(again, out)
    m.close()


def test_hh_sweep_frames_per_slot_and_negative_min_disparity(oracle):
    """Wide frames (W1 = 1652: 21 tiles of 80 columns, so about 12 frames fit the resident grid)
    in a batch of 16: the slots take a second frame each (the edge counters run on across frames,
    the frame-start waits), with minDisparity < 0 and the uniqueness / LR variations."""
    F, H, W, D = 16, 12, 1700, 48
    args = (-8, D, 5, 200, 1600, 2, 63, 5, 0, 2, sdr.MODE_HH)
    Ls, Rs = _batch("noise", F // 2, H, W, D, 11)
    L2, R2 = _batch("textured", F // 2, H, W, D, 30)
    Ls, Rs = np.concatenate([Ls, L2]), np.concatenate([Rs, R2])
    dev = torch.device("cuda", 0)
    m = sdr.StereoSGBM.create(*args)
    out = m.compute(torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)).cpu().numpy()
    p = oracle.make_params(*args)
    for i in range(F):
        ref = oracle.sgbm_compute(Ls[i], Rs[i], p)
        assert np.array_equal(out[i], ref), f"frame {i}: {(out[i] != ref).sum()} px differ"
    m.close()


def test_sweep_timeout_poisons_batch_and_reports(oracle):
    """The failure contract of the row sweeps: with the neighbour waits cut to one
    poll (debug knob), waits give up; the batch's frames then come back INVALID ((minD-1)*16 on
    every pixel, never silently wrong values) and the handle's status reports SDR_ERR_DEVICE once.
    The next batch with the default budget is bit-exact again and the status is clean."""
    F, H, W, D = 16, 96, 1700, 48
    args = (0, D, 5, 600, 2400, 1, 63, 10, 0, 2, sdr.MODE_HH)
    Ls, Rs = _batch("textured", F, H, W, D, 40)
    dev = torch.device("cuda", 0)
    Ld, Rd = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    m = sdr.StereoSGBM.create(*args)
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 1)
    bad = m.compute(Ld, Rd).cpu().numpy()
    with pytest.raises(sdr.SDRError) as ei:
        m.check_status()
    assert ei.value.code == -6
    assert (bad == -16).all(), "a timed-out sweep must leave no frame values behind"
    m.check_status()  # reported once
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 0)
    good = m.compute(Ld, Rd).cpu().numpy()
    m.check_status()
    p = oracle.make_params(*args)
    for i in (0, F - 1):
        assert np.array_equal(good[i], oracle.sgbm_compute(Ls[i], Rs[i], p)), i
    m.close()


def test_sweep_timeout_reported_by_next_call(oracle):
    """A caller that never polls sdr_sgbm_last_status still hears of a timed-out sweep:
    the next compute call on the handle returns SDR_ERR_DEVICE without running, the status is then
    clean, and the call after is bit-exact."""
    F, H, W, D = 16, 96, 1700, 48
    args = (0, D, 5, 600, 2400, 1, 63, 10, 0, 2, sdr.MODE_HH)
    Ls, Rs = _batch("textured", F, H, W, D, 41)
    dev = torch.device("cuda", 0)
    Ld, Rd = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    m = sdr.StereoSGBM.create(*args)
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 1)
    bad = m.compute(Ld, Rd).cpu().numpy()  # synchronises: the status copy has landed
    assert (bad == -16).all()
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 0)
    with pytest.raises(sdr.SDRError) as ei:
        m.compute(Ld, Rd)
    assert ei.value.code == -6
    m.check_status()  # reported by the call: clean
    good = m.compute(Ld, Rd).cpu().numpy()
    m.check_status()
    p = oracle.make_params(*args)
    assert np.array_equal(good[F - 1], oracle.sgbm_compute(Ls[F - 1], Rs[F - 1], p))
    m.close()


def test_sweep_timeout_reported_once_unsynchronised(oracle):
    """a timeout is reported exactly once even when later batches are queued before its
    status copy lands.  The device word counts timed-out batches and the host remembers the count
    it reported (no clear of the device word that a copy still in flight could undo): one forced
    timeout, then four calls queued back to back with no synchronisation, then the status --
    SDR_ERR_DEVICE exactly once over all of them, and the frames after it bit-exact."""
    F, H, W, D = 16, 96, 1700, 48
    args = (0, D, 5, 600, 2400, 1, 63, 10, 0, 2, sdr.MODE_HH)
    Ls, Rs = _batch("textured", F, H, W, D, 42)
    dev = torch.device("cuda", 0)
    Ld, Rd = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    m = sdr.StereoSGBM.create(*args)
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 1)
    bad = torch.empty((F, H, W), dtype=torch.int16, device=dev)
    m.compute(Ld, Rd, disp=bad)  # queued, not synchronised
    m.set_debug_knob(sdr.sgbm.DEBUG_SWEEP_SPIN, 0)
    errors = 0
    outs = []
    for _ in range(4):
        o = torch.empty((F, H, W), dtype=torch.int16, device=dev)
        try:
            m.compute(Ld, Rd, disp=o)
            outs.append(o)
        except sdr.SDRError as e:
            assert e.code == -6
            errors += 1
    try:
        m.check_status()
    except sdr.SDRError as e:
        assert e.code == -6
        errors += 1
    assert errors == 1, errors
    assert (bad.cpu().numpy() == -16).all()
    m.check_status()
    good = m.compute(Ld, Rd).cpu().numpy()
    m.check_status()
    p = oracle.make_params(*args)
    ref = oracle.sgbm_compute(Ls[F - 1], Rs[F - 1], p)
    assert np.array_equal(good[F - 1], ref)
    # calls queued after the timed-out batch in the same stream ran with the default budget
    for o in outs[1:]:
        assert np.array_equal(o[F - 1].cpu().numpy(), ref)
    m.close()


def test_two_handles_two_streams_concurrent_sweeps(oracle):
    """Two matchers on two streams each enqueue 8-frame MODE_HH batches back to back without a
    synchronisation in between: their sweeps are chained per device (never two in flight), and
    every frame equals its single-frame k_paths run."""
    F, H, W, D = 8, 40, 600, 64
    args = (0, D, 5, 600, 2400, 1, 63, 10, 20, 2, sdr.MODE_HH)
    dev = torch.device("cuda", 0)
    batches = [_batch("textured", F, H, W, D, 100 + 10 * k) for k in range(4)]
    dev_in = [(torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)) for L, R in batches]
    ms = [sdr.StereoSGBM.create(*args) for _ in range(2)]
    ss = [torch.cuda.Stream(dev) for _ in range(2)]
    torch.cuda.synchronize(dev)
    outs = []
    for k, (Ld, Rd) in enumerate(dev_in):
        with torch.cuda.stream(ss[k % 2]):
            outs.append(ms[k % 2].compute(Ld, Rd))
    torch.cuda.synchronize(dev)
    for m in ms:
        m.check_status()
    one = sdr.StereoSGBM.create(*args)
    for k, (L, R) in enumerate(batches):
        got = outs[k].cpu().numpy()
        for i in range(F):
            assert np.array_equal(got[i], one.compute(L[i], R[i])), f"batch {k} frame {i}"
    p = oracle.make_params(*args)
    assert np.array_equal(outs[3][F - 1].cpu().numpy(), oracle.sgbm_compute(batches[3][0][F - 1], batches[3][1][F - 1], p))
    for m in ms + [one]:
        m.close()


hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from conftest import hyp_examples  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@st.composite
def sweep_cases(draw):
    D = 16 * draw(st.integers(1, 16))  # both lane widths, padded and full
    bs = draw(st.sampled_from([1, 3, 5, 7]))
    return dict(kind=draw(st.sampled_from(["textured", "noise", "binary", "steps"])),
                F=draw(st.integers(8, 11)), H=draw(st.integers(4, 28)),
                W=D + bs // 2 + 1 + draw(st.integers(0, 258)), D=D,  # W1 > blockSize / 2
                bs=bs, P1=draw(st.integers(1, 400)),
                P2x=draw(st.integers(2, 8)), uniq=draw(st.sampled_from([0, 5, 15])),
                ws=draw(st.sampled_from([0, 0, 20])), seed=draw(st.integers(0, 10**6)))


@settings(max_examples=hyp_examples(12), deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(case=sweep_cases())
def test_hh_sweep_hypothesis_bit_exact(oracle, case):
    """Random batched MODE_HH shapes through the row sweeps (every lane width, partial tiles,
    block sizes, penalties), each frame against the oracle."""
    c = case
    args = (0, c["D"], c["bs"], c["P1"], c["P1"] * c["P2x"], 1, 63, c["uniq"], c["ws"], 2, sdr.MODE_HH)
    Ls, Rs = _batch(c["kind"], c["F"], c["H"], c["W"], c["D"], c["seed"])
    dev = torch.device("cuda", 0)
    m = sdr.StereoSGBM.create(*args)
    out = m.compute(torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)).cpu().numpy()
    p = oracle.make_params(*args)
    for i in range(c["F"]):
        ref = oracle.sgbm_compute(Ls[i], Rs[i], p)
        assert np.array_equal(out[i], ref), f"frame {i}: {(out[i] != ref).sum()} px differ"
    m.close()
