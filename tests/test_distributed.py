"""Multi-rank logic on CPU (gloo, world_size 2): frame sharding + gather to rank 0 reproduce the
single-process result.  The per-rank compute here is the oracle (the CPU tests' stand-in for
the HIP engine, which the -m gpu tests and bench.py exercise)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from stereo_depth_ruler_amd.distributed import frames_per_rank, gather_frames, shard_frames


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

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
