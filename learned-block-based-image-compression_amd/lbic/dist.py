"""Multi-GPU: images shard over ranks (one process per GPU); the only collective gathers the per-image
rate/distortion summary.  The closed-loop state never crosses images, so the codec itself
has no data-path collective.  Backend "nccl" is RCCL over xGMI on ROCm; tests use "gloo" on the CPU.
"""
from __future__ import annotations

import os

import torch


def rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def shard(items, rank, world):
    """Image i -> rank i mod world (deterministic, balanced to within one image)."""
    return list(items)[rank::world]


def gather_records(rec: torch.Tensor) -> torch.Tensor:
    """All-gather a [n_local, k] float64 summary from every rank (n_local may differ per rank) and return
    the [n_total, k] concatenation ordered by rank.  No-op without an initialised process group."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return rec
    world = dist.get_world_size()
    n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=rec.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    nmax = int(max(int(x.item()) for x in ns))
    pad = torch.full((nmax, rec.shape[1]), float("nan"), dtype=rec.dtype, device=rec.device)
    pad[: rec.shape[0]] = rec
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad)
    return torch.cat([o[: int(k.item())] for o, k in zip(out, ns)])
