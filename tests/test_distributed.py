"""Multi-rank logic on CPU (gloo, world_size 2): frame sharding + gather to rank 0 reproduce the
single-process result.  The per-rank compute here is the oracle (the CPU tests' stand-in for
the HIP engine, which the -m gpu tests and bench.py exercise)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from stereo_depth_ruler_amd.distributed import (RankFailure, check_ranks, frames_per_rank, gather_frames,
                                                shard_frames)


def test_shard_round_robin_covers_all():
    for n in (0, 1, 7, 8, 33):
        for world in (1, 2, 4, 8):
            seen = sorted(i for r in range(world) for i in shard_frames(n, world, r))
            assert seen == list(range(n))
            assert max((len(shard_frames(n, world, r)) for r in range(world)), default=0) <= frames_per_rank(n, world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_frames, q):
    import torch.distributed as dist

    from oracle import oracle as O
    from stereo_depth_ruler_amd import synthetic as S

    from stereo_depth_ruler_amd.distributed import init_process_group

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    init_process_group("gloo", rank=rank, world_size=world)
    p = O.make_params(0, 16, 5, 600, 2400, 1, 63, 12, 20, 2, 0)
    mine = shard_frames(n_frames, world, rank)
    res = []
    for i in mine:
        L, R, _ = S.make_pair(24, 64, 16, seed=i)
        res.append(torch.from_numpy(O.sgbm_compute(L, R, p)))
    local = torch.stack(res) if res else torch.empty((0, 24, 64), dtype=torch.int16)
    out = gather_frames(local, n_frames, world, rank)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [5, 6])
def test_gloo_world2_gather_matches_single(n_frames):
    from oracle import oracle as O
    from stereo_depth_ruler_amd import synthetic as S

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    p = O.make_params(0, 16, 5, 600, 2400, 1, 63, 12, 20, 2, 0)
    for i in range(n_frames):
        L, R, _ = S.make_pair(24, 64, 16, seed=i)
        assert np.array_equal(got[i], O.sgbm_compute(L, R, p)), i


def _failing_worker(rank, world, port, fail_rank, q):
    """Rank `fail_rank` fails its step with an engine-style error; every rank must raise
    RankFailure from gather_frames (none may block in the gather) and exit non-zero."""
    import sys
    import time

    import torch.distributed as dist

    from stereo_depth_ruler_amd._lib import SDRError
    from stereo_depth_ruler_amd.distributed import init_process_group

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    init_process_group("gloo", rank=rank, world_size=world, timeout=30)
    local, err = torch.zeros((2, 8, 8), dtype=torch.int16), None
    if rank == fail_rank:
        err = SDRError(-2, "numDisparities must be positive and divisible by 16")
        local = None
    t0 = time.time()
    try:
        gather_frames(local, 4, world, rank, error=err)
    except RankFailure as f:
        q.put((rank, f.codes, time.time() - t0))
        dist.destroy_process_group()
        sys.exit(3)
    q.put((rank, None, time.time() - t0))


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_gloo_world2_rank_failure_aborts_gather(fail_rank):
    """SURVEY.md 5 failure detection: one rank's SDR_ERR_* makes BOTH processes exit non-zero
    quickly (well inside the collective timeout), with the failing rank's code reported."""
    import time

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t0 = time.time()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=90)
    alive = [pr for pr in procs if pr.is_alive()]
    for pr in alive:
        pr.kill()
    assert not alive, "a rank hung"
    assert all(pr.exitcode == 3 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, codes, dt in res:
        assert codes is not None and codes[fail_rank] == -2 and codes[1 - fail_rank] == 0
        assert dt < 20
    assert time.time() - t0 < 90


def test_check_ranks_single_process():
    """world 1: the status exchange is a no-op on success and raises on failure."""
    import torch.distributed as dist

    from stereo_depth_ruler_amd.distributed import init_process_group

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    init_process_group("gloo", rank=0, world_size=1, timeout=30)
    try:
        check_ranks(0)
        with pytest.raises(RankFailure):
            check_ranks(-4)
    finally:
        dist.destroy_process_group()


def _group_worker(rank, world, port, direct, q):
    """world 3; ranks 0 and 1 gather over a subgroup {0, 1} while rank 2 stays out of it, or
    (direct) the world is set up by torch.distributed.init_process_group itself, without the
    wrapper's status group."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if direct:
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
    else:
        from stereo_depth_ruler_amd.distributed import init_process_group
        init_process_group("gloo", rank=rank, world_size=world, timeout=30)
    local = torch.full((2, 4, 4), rank + 1, dtype=torch.int16)
    out = None
    if direct:
        out = gather_frames(local, 2 * world, world, rank)
    else:
        g = dist.new_group([0, 1])
        if rank < 2:
            out = gather_frames(local, 4, 2, rank, group=g)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("direct", [False, True])
def test_gather_frames_subgroup_and_direct_init(direct):
    """gather_frames' status exchange runs on the caller's group (a subgroup's ranks only) and works
    on a world that init_process_group set up without the wrapper."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, direct, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=90)
    for pr in procs:
        pr.join(timeout=60)
    alive = [pr for pr in procs if pr.is_alive()]
    for pr in alive:
        pr.kill()
    assert not alive and all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    nr = world if direct else 2
    # frame i came from rank i mod nr, its (i // nr)-th local frame
    assert got.shape[0] == 2 * nr
    for i in range(2 * nr):
        assert (got[i] == (i % nr) + 1).all(), i
