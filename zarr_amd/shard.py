"""Multi-GPU partition of independent chunks.

Chunks carry no cross-chunk state (each read_chunk builds a fresh decoder,
chunk.rs:282,297), so N GPUs split a batch round-robin — chunk i goes to GPU
i mod N — with no collective on the data path.  The only collectives are the
timing ones the benchmark contract needs (a barrier and the max over ranks).
"""
from __future__ import annotations

from typing import List


def round_robin_ids(rank: int, world: int, n_per_rank: int) -> List[int]:
    """Global chunk ids of `rank` when every rank decodes `n_per_rank` chunks
    (weak scaling): ids rank, rank + world, rank + 2*world, ..."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return [i * world + rank for i in range(n_per_rank)]


def split_round_robin(n_total: int, rank: int, world: int) -> List[int]:
    """Global chunk ids of `rank` for a fixed batch of n_total chunks (strong
    scaling, e.g. C4's 65 536 chunks over 8 GPUs)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return list(range(rank, n_total, world))


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar over the default process group (RCCL on GPU
    ranks, gloo in the CPU tests); the identity without a group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(bytes_per_rank: int, seconds_local: float, device=None) -> float:
    """Whole-job throughput: bytes of ALL ranks / the slowest rank's time."""
    import torch.distributed as dist
    world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    t = max_over_ranks(seconds_local, device)
    return world * bytes_per_rank / t
