"""Env sharding across ranks (one process per GPU), SURVEY.md §8(e).

Envs are independent (model/ffm_core.py:16-21 holds all per-env state), so a
node-wide run is a partition of the global env range into contiguous blocks,
one per rank, with every random draw keyed by the *global* env id (the
engine's ``env_base``).  The data path has no collective; the only exchange is
the end-of-run reduction of counters (sum) and elapsed time (max).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_global: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of the global env range owned by ``rank``: (env_base, count).

    Blocks differ in size by at most one env (the first ``n_global % world``
    ranks take one extra), so any ``n_global >= world`` is valid.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if n_global < world:
        raise ValueError(f"{n_global} envs cannot be split over {world} ranks")
    q, r = divmod(n_global, world)
    count = q + (1 if rank < r else 0)
    base = rank * q + min(rank, r)
    return base, count


def weak_shard(envs_per_rank: int, rank: int) -> int:
    """env_base of ``rank`` when every rank steps ``envs_per_rank`` envs (weak scaling)."""
    return rank * envs_per_rank


_KEYS = ("agent_steps", "exits", "resets", "steps")


def reduce_counters(counters: dict, device=None, group=None) -> dict:
    """Sum the engine counters over ranks (``steps`` is per-launch, so max)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return dict(counters)
    t = torch.tensor([int(counters[k]) for k in _KEYS[:3]], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    s = torch.tensor([int(counters["steps"])], dtype=torch.int64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.MAX, group=group)
    out = {k: int(v) for k, v in zip(_KEYS[:3], t.tolist())}
    out["steps"] = int(s.item())
    return out


def reduce_max(x: float, device=None, group=None) -> float:
    """Max of a float over ranks (the bench's elapsed time)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
