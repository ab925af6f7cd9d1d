"""Frame sharding across ranks and the gather of disparity maps to rank 0.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm, "gloo" for CPU
tests).  Frames are independent, so the path shards by frame with no exchange during compute;
the only collective is the gather of results to rank 0.
"""
from __future__ import annotations

from typing import List, Optional


def shard_frames(n_frames: int, world: int, rank: int) -> List[int]:
    """Frame i -> rank i mod world (round robin, as frames arrive from a stream)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return list(range(rank, n_frames, world))


def frames_per_rank(n_frames: int, world: int) -> int:
    return (n_frames + world - 1) // world


def gather_frames(local, n_frames: int, world: int, rank: int, group=None):
    """Gathers each rank's results (tensor [n_local, ...] in shard_frames order) to rank 0.

    Returns a tensor [n_frames, ...] in global frame order on rank 0, None elsewhere.  Ranks pad
    to the same count so a single collective gather suffices.
    """
    import torch
    import torch.distributed as dist

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
