"""Frame sharding across ranks and the gather of disparity maps to rank 0.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm, "gloo" for CPU
tests).  Frames are independent, so the path shards by frame with no exchange during compute;
the only collective is the gather of results to rank 0.

Failure handling ("per-rank failure aborts the gather cleanly").  The reference's
only failure behaviour is to stop (stereo_displayer.cpp:149-152: an empty frame ends the loop).
Sharded, a rank whose compute raises (an SDR_ERR_* from the engine, a bad frame) must not leave
the others blocked in a collective:
  * ``init_process_group`` bounds every collective with a timeout (SDR_DIST_TIMEOUT seconds,
    default 120), so a rank that dies outright (segfault, killed) ends the others' waits;
  * ``check_ranks(code)`` exchanges one status code per rank over a host-side (gloo) group, and
    raises ``RankFailure`` on EVERY rank if any code is non-zero, so all processes exit non-zero
    together instead of one blocking in ``dist.gather``;
  * ``gather_frames(..., error=e)`` runs that exchange before its gather: a rank that failed
    passes its exception instead of results.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

DEFAULT_TIMEOUT_S = 120.0
_status_group = None


class RankFailure(RuntimeError):
    """Raised on every rank when any rank reported a failed step."""

    def __init__(self, codes):
        self.codes = list(codes)
        bad = {r: c for r, c in enumerate(self.codes) if c != 0}
        super().__init__(f"rank(s) failed, status codes by rank: {bad}")


def timeout_s() -> float:
    return float(os.environ.get("SDR_DIST_TIMEOUT", DEFAULT_TIMEOUT_S))


def init_process_group(backend: str, device_id=None, timeout: Optional[float] = None, **kw):
    """torch.distributed.init_process_group with a bounded collective timeout (seconds) and the
    host-side status group used by check_ranks."""
    import torch.distributed as dist

    global _status_group
    t = datetime.timedelta(seconds=timeout if timeout is not None else timeout_s())
    if device_id is not None:
        kw["device_id"] = device_id
    dist.init_process_group(backend, timeout=t, **kw)
    _status_group = dist.new_group(backend="gloo", timeout=t) if backend != "gloo" else None
    return _status_group


def error_code(err) -> int:
    """Status code of a failed step: the engine's SDR_ERR_* code, -1000 for anything else."""
    if err is None:
        return 0
    c = getattr(err, "code", None)
    return int(c) if isinstance(c, int) and c != 0 else -1000


def check_ranks(code: int = 0, group=None) -> None:
    """All ranks of `group` (default: the world) exchange their status (0 = ok); raises
    RankFailure on every rank if any is not 0.  Over the host-side gloo status group when the world
    is meant (it never waits on a GPU stream); over `group` itself otherwise, with the codes in
    device memory when that group's backend is nccl (RCCL has no host tensors).  A world set up
    by torch.distributed.init_process_group directly (no status group) is treated the same way."""
    import torch
    import torch.distributed as dist

    g = group if group is not None else _status_group
    dev = "cpu"
    if dist.get_backend(g) != "gloo":
        dev = torch.device("cuda", torch.cuda.current_device())
    world = dist.get_world_size(g)
    mine = torch.tensor([int(code)], dtype=torch.int64, device=dev)
    codes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(codes, mine, group=g)
    vals = [int(c.item()) for c in codes]
    if any(vals):
        raise RankFailure(vals)


def shard_frames(n_frames: int, world: int, rank: int) -> List[int]:
    """Frame i -> rank i mod world (round robin, as frames arrive from a stream)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return list(range(rank, n_frames, world))


def frames_per_rank(n_frames: int, world: int) -> int:
    return (n_frames + world - 1) // world


def gather_frames(local, n_frames: int, world: int, rank: int, group=None, error=None):
    """Gathers each rank's results (tensor [n_local, ...] in shard_frames order) to rank 0.

    Returns a tensor [n_frames, ...] in global frame order on rank 0, None elsewhere.  Ranks pad
    to the same count so a single collective gather suffices.  A rank whose compute failed passes
    the exception as `error` (local may then be None): every rank raises RankFailure before the
    gather, none blocks in it.
    """
    import torch
    import torch.distributed as dist

    try:
        check_ranks(error_code(error), group=group)
    except RankFailure as f:
        if error is not None:
            raise f from error
        raise

    per = frames_per_rank(n_frames, world)
    if local.shape[0] > per:
        raise ValueError("local shard larger than frames_per_rank")
    padded = local
    if local.shape[0] < per:
        pad = torch.zeros((per - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        padded = torch.cat([local, pad], 0)
    # collectives move bytes: neither gloo nor RCCL has an int16 type
    raw = as_bytes(padded.contiguous())
    bufs: Optional[list] = None
    if rank == 0:
        bufs = [torch.empty_like(raw) for _ in range(world)]
    dist.gather(raw, bufs, dst=0, group=group)
    if rank != 0:
        return None
    got = [b.view(local.dtype).view(padded.shape) for b in bufs]
    out = torch.empty((n_frames,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for i in range(n_frames):
        out[i] = got[i % world][i // world]
    return out


def as_bytes(t):
    """Flat uint8 view of a contiguous tensor (for collectives on dtypes RCCL/gloo lack)."""
    return t.contiguous().view(-1).view(__import__("torch").uint8)
