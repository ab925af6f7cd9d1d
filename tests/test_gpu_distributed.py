"""The N>1 path on the HIP engine, world size 2 on the box's one GPU: two fresh
spawned processes (gloo, both ranks on cuda:0) each run the engine on their frame shard.

  - gather_frames: rank 0's gathered disparities equal a single-process run of all frames on the
    same engine, bit for bit (and the oracle on two of them);
  - bench.py's own step/async-gather loop under torch.distributed.run (--dist-backend gloo): the
    JSON line reports 2 ranks and its end-to-end gather check passes;
  - the failure path: a rank whose engine call returns SDR_ERR_* makes BOTH processes
    exit non-zero promptly (gather_frames and bench.py), no rank blocks in a collective.

Scaling is not measured here (both ranks share one GPU); the RCCL path is the same code with
backend "nccl" and one GPU per rank.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = (0, 64, 5, 600, 2400, 1, 63, 12, 50, 2, 0)
H, W, N = 96, 320, 7


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames():
    from stereo_depth_ruler_amd import synthetic as S
    return S.make_batch(N, H, W, 64, seed0=300)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import stereo_depth_ruler_amd as sdr
    from stereo_depth_ruler_amd.distributed import gather_frames, init_process_group, shard_frames

    init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    Ls, Rs = _frames()
    mine = shard_frames(N, world, rank)
    m = sdr.StereoSGBM.create(*ARGS)
    Ld = torch.from_numpy(Ls[mine]).cuda()
    Rd = torch.from_numpy(Rs[mine]).cuda()
    local = m.compute(Ld, Rd).cpu()  # gloo gathers host tensors
    out = gather_frames(local, N, world, rank)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    m.close()
    dist.destroy_process_group()


def test_world2_gather_frames_hip_engine(oracle):
    import torch.multiprocessing as mp

    import stereo_depth_ruler_amd as sdr

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Ls, Rs = _frames()
    m = sdr.StereoSGBM.create(*ARGS)
    single = m.compute(torch.from_numpy(Ls).cuda(), torch.from_numpy(Rs).cuda()).cpu().numpy()
    assert got.shape == single.shape == (N, H, W)
    assert np.array_equal(got, single)
    p = oracle.make_params(*ARGS)
    for i in (0, N - 1):
        assert np.array_equal(got[i], oracle.sgbm_compute(Ls[i], Rs[i], p)), i


def test_world2_bench_step_gather_loop():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "6", "--warmup", "2", "--dist-backend", "gloo", "--streams", "2",
           "--frames", "4", "--no-cpu-baseline", "--no-kernel-timing"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["steps"] == 6
    assert out["gather_check"] == {"step": 7, "ranks": 2, "gather_every": 8, "ok": True}


def test_bench_gpus2_self_launch():
    """`python bench.py --gpus 2` with NO external launcher (the driver's N-GPU command minus
    torch.distributed.run): bench.py starts both ranks itself (here over gloo, both on the box's one
    GPU) and prints one line with n_gpus 2, both ranks' times and a good gather check."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--dist-backend", "gloo", "--streams", "2", "--frames", "4", "--no-cpu-baseline", "--no-kernel-timing"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["gather_check"]["ok"] and out["gather_check"]["ranks"] == 2
    assert out["ranks"]["world_size_seen"] == 2 and len(out["ranks"]["per_rank"]) == 2
    assert out["ranks"]["launcher"].startswith("bench.py --gpus")
    assert {r["rank"] for r in out["ranks"]["per_rank"]} == {0, 1}
    worst = max(r["ms_per_step"] for r in out["ranks"]["per_rank"])
    assert abs(out["ms_per_step"] - worst) < 1e-3 + 1e-3 * worst


def test_bench_gpus2_nccl_needs_two_gpus():
    """Over RCCL every rank needs its own GPU: on a one-GPU box --gpus 2 fails loudly instead of
    printing an N=1 number."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU: the RCCL path can run")
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-kernel-timing"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode != 0
    assert "need 2 GPUs" in res.stderr
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("config", ["c2", "c4"])
def test_bench_rccl_world1(config):
    """The RCCL data path executed on the one-GPU box: bench.py under
    torch.distributed.run --nproc-per-node 1 with --dist-world1 initialises the nccl (RCCL)
    process group on the GPU, runs the per-step dist.gather of device tensors to rank 0, the
    status exchanges and the end-to-end gather check -- the same calls the 8-GPU run makes."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--dist-world1", "--config", config, "--steps", "20", "--warmup", "3", "--status-every", "4",
           "--no-cpu-baseline", "--no-kernel-timing"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert out["ranks"]["backend"] == "nccl (RCCL)" and out["ranks"]["world_size_seen"] == 1
    assert out["gather_check"]["ok"] and out["gather_check"]["ranks"] == 1
    assert "RCCL gather" in out["config"]["parallelism"]


def _failing_worker(rank, world, port, q):
    """Rank 1 asks the real engine for numDisparities = 20 (SDR_ERR_NUMDISP, OpenCV's assert)."""
    import sys
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import stereo_depth_ruler_amd as sdr
    from stereo_depth_ruler_amd.distributed import RankFailure, gather_frames, init_process_group, shard_frames

    init_process_group("gloo", rank=rank, world_size=world, timeout=60)
    torch.cuda.set_device(0)
    Ls, Rs = _frames()
    mine = shard_frames(N, world, rank)
    args = ARGS if rank == 0 else (0, 20) + ARGS[2:]
    local, err = None, None
    t0 = time.time()
    try:
        m = sdr.StereoSGBM.create(*args)
        local = m.compute(torch.from_numpy(Ls[mine]).cuda(), torch.from_numpy(Rs[mine]).cuda()).cpu()
    except sdr.SDRError as e:
        err = e
    try:
        gather_frames(local, N, world, rank, error=err)
    except RankFailure as f:
        q.put((rank, f.codes, time.time() - t0))
        dist.destroy_process_group()
        sys.exit(3)
    q.put((rank, None, time.time() - t0))


def test_world2_engine_error_aborts_gather():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank hung"
    assert [p.exitcode for p in procs] == [3, 3]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, codes, dt in res:
        assert codes == [0, -2], codes  # SDR_ERR_NUMDISP on rank 1
        assert dt < 60


def test_world2_bench_rank_failure_exits_nonzero():
    """bench.py with rank 1's step 5 failing: both ranks raise RankFailure at the next status
    check (every 4 steps here) and torch.distributed.run exits non-zero, well inside the timeout."""
    env = dict(os.environ, PYTHONUNBUFFERED="1", SDR_DIST_TIMEOUT="60")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "8", "--warmup", "2", "--dist-backend", "gloo", "--streams", "2",
           "--frames", "4", "--no-cpu-baseline", "--no-kernel-timing", "--status-every", "4",
           "--inject-failure", "1:5"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode != 0
    assert "RankFailure" in res.stderr and "injected failure at rank 1 step 5" in res.stderr, res.stderr[-3000:]
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
