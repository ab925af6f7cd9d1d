"""One matcher moved between HIP streams while its earlier calls are still queued.

A handle's scratch (cost volume, path records, ...) is reused by every call, so a call on a new
stream must not start before the handle's work on the old stream is done.  The engine records its
retire event on the old stream only at the switch (sdr_engine.hip use_stream; recording one per
call was a queue barrier): these tests queue calls back to back across switches with
no host synchronisation in between, and every output must equal the same call made alone.
"""
import numpy as np
import pytest

import stereo_depth_ruler_amd as sdr
from stereo_depth_ruler_amd import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _refs(m, L, R, F, n):
    out = []
    for k in range(n):
        out.append(m.compute(L[k * F:(k + 1) * F], R[k * F:(k + 1) * F]).clone())
        torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("mode,D,F", [(sdr.MODE_SGBM, 128, 4), (sdr.MODE_HH, 64, 8)])
def test_stream_switch_with_pending_work(mode, D, F, oracle):
    """C2-sized frames (a few ms of queued work per call) through streams a, b, a, then the
    handle's own stream: each call's disparity equals the synchronised one-at-a-time run (and the
    first frame equals the oracle).  MODE_HH with 8 frames takes the row-sweep path."""
    H, W = (720, 1280) if mode == sdr.MODE_SGBM else (240, 640)
    n = 4
    Ls, Rs = S.make_batch(n * F, H, W, D, seed0=900)
    dev = torch.device("cuda", 0)
    L, R = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    args = (0, D, 5, 600, 2400, 1, 63, 12, 200, 2, mode)
    m = sdr.StereoSGBM.create(*args)
    refs = _refs(m, L, R, F, n)
    a, b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = [torch.empty((F, H, W), dtype=torch.int16, device=dev) for _ in range(n)]
    torch.cuda.synchronize()
    for k, s in enumerate((a, b, a, None)):
        if s is None:
            m.compute(L[k * F:(k + 1) * F], R[k * F:(k + 1) * F], disp=outs[k])
        else:
            with torch.cuda.stream(s):
                m.compute(L[k * F:(k + 1) * F], R[k * F:(k + 1) * F], disp=outs[k])
    torch.cuda.synchronize()
    for k in range(n):
        assert torch.equal(outs[k], refs[k]), k
    p = oracle.make_params(*args)
    assert np.array_equal(refs[0][0].cpu().numpy(), oracle.sgbm_compute(Ls[0], Rs[0], p))
    m.close()


def test_caller_stream_destroyed_after_switching_away(oracle):
    """ADVICE r4 / sdr.h: a caller's stream must outlive the handle's use of it (HIP does not
    validate a destroyed stream's handle: an event recorded on one, or waited on after being
    recorded there, crashes the process -- measured on MI355X in round 5, so no engine-side check
    can catch the misuse).  The supported order: work on a caller's stream, move the handle off it
    (another stream, or reset_stream), destroy the stream, keep using the handle -- bit-exact, and
    close() works."""
    import ctypes

    from stereo_depth_ruler_amd._lib import check, lib

    hip = ctypes.CDLL("libamdhip64.so")
    H, W, D = 120, 320, 64
    Ls, Rs = S.make_batch(1, H, W, D, seed0=77)
    dev = torch.device("cuda", 0)
    L, R = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    args = (0, D, 5, 600, 2400, 1, 63, 12, 0, 2, sdr.MODE_SGBM)
    ref = oracle.sgbm_compute(Ls[0], Rs[0], oracle.make_params(*args))
    m = sdr.StereoSGBM.create(*args)
    for leave in ("set_stream", "reset_stream"):
        raw = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
        with torch.cuda.stream(torch.cuda.ExternalStream(raw.value, device=dev)):
            out = m.compute(L, R)
        if leave == "set_stream":  # the caller's next stream, as compute() on it would
            check(lib().sdr_sgbm_set_stream(m._h, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        else:
            check(lib().sdr_sgbm_reset_stream(m._h))
        assert hip.hipStreamDestroy(raw) == 0
        assert np.array_equal(out[0].cpu().numpy(), ref)
        for _ in range(2):
            assert np.array_equal(m.compute(L, R)[0].cpu().numpy(), ref)
    m.close()


def test_switch_off_a_destroyed_stream(oracle):
    """VERDICT r5 item 4 (the crash in gpurun_out/r5b/tests.log): a caller's external stream is
    destroyed right after a call on it, WITHOUT moving the handle off it first; the next call
    (on another stream), last_status and close() must not touch the dead stream.  An external
    stream is bound transient (sgbm.set_handle_stream: sdr_sgbm_set_stream_ex without
    SDR_STREAM_PERSISTENT), so the handle relays its retire event through its own stream at the
    end of each call.  Bit-exact throughout; also through the raw C ABI's set_stream."""
    import ctypes

    from stereo_depth_ruler_amd._lib import check, lib

    hip = ctypes.CDLL("libamdhip64.so")
    H, W, D = 120, 320, 64
    Ls, Rs = S.make_batch(1, H, W, D, seed0=78)
    dev = torch.device("cuda", 0)
    L, R = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    args = (0, D, 5, 600, 2400, 1, 63, 12, 0, 2, sdr.MODE_SGBM)
    ref = oracle.sgbm_compute(Ls[0], Rs[0], oracle.make_params(*args))
    for how in ("torch_external", "c_abi", "close_on_dead_stream"):
        m = sdr.StereoSGBM.create(*args)
        raw = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
        out = torch.empty((1, H, W), dtype=torch.int16, device=dev)
        if how == "torch_external":
            with torch.cuda.stream(torch.cuda.ExternalStream(raw.value, device=dev)):
                m.compute(L, R, disp=out)
        else:
            check(lib().sdr_sgbm_set_stream(m._h, raw))
            check(lib().sdr_sgbm_compute_device(m._h, ctypes.c_void_p(L.data_ptr()), ctypes.c_void_p(R.data_ptr()),
                                                W, H, W, H * W, 1, ctypes.c_void_p(out.data_ptr()), W, H * W))
        assert hip.hipStreamSynchronize(raw) == 0
        assert hip.hipStreamDestroy(raw) == 0  # the handle is still bound to it
        assert np.array_equal(out[0].cpu().numpy(), ref)
        if how == "close_on_dead_stream":
            check(lib().sdr_sgbm_last_status(m._h))
            m.close()
            continue
        for _ in range(2):  # compute() moves the handle to torch's current stream
            assert np.array_equal(m.compute(L, R)[0].cpu().numpy(), ref)
        m.close()


def test_transient_stream_orders_next_stream(oracle):
    """A transient stream's calls are ordered before the next stream's without a host sync: C2-size
    frames queued on an external stream, then on torch's stream, back to back; every output equals
    the one-at-a-time run."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    H, W, D, F = 720, 1280, 128, 2
    Ls, Rs = S.make_batch(2 * F, H, W, D, seed0=910)
    dev = torch.device("cuda", 0)
    L, R = torch.from_numpy(Ls).to(dev), torch.from_numpy(Rs).to(dev)
    args = (0, D, 5, 600, 2400, 1, 63, 12, 200, 2, sdr.MODE_SGBM)
    m = sdr.StereoSGBM.create(*args)
    refs = _refs(m, L, R, F, 2)
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
    outs = [torch.empty((F, H, W), dtype=torch.int16, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    with torch.cuda.stream(torch.cuda.ExternalStream(raw.value, device=dev)):
        m.compute(L[:F], R[:F], disp=outs[0])
    m.compute(L[F:], R[F:], disp=outs[1])
    torch.cuda.synchronize()
    assert hip.hipStreamSynchronize(raw) == 0
    assert hip.hipStreamDestroy(raw) == 0
    for k in range(2):
        assert torch.equal(outs[k], refs[k]), k
    m.close()
