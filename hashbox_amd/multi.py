"""Multi-GPU: one process per GPU, files sharded by LPT on bytes.

Files are independent, so ranks never exchange data on the
hot path: each rank chunks+hashes its shard on its own GPU/stream and only
the (tiny) results — cut lists and 16-byte IDs — are gathered at the end.
torch.distributed carries that gather and the timing barrier (gloo on CPU
in tests; nccl = RCCL on the GPU box).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence

from .shard import lpt_assign


def shard_for_rank(lens: Sequence[int], rank: int, world: int) -> List[int]:
    return lpt_assign(lens, world)[rank]


def run_sharded(lens: Sequence[int], process: Callable[[List[int]], Dict[int, object]],
                rank: int, world: int, group=None) -> Dict[int, object]:
    """Run ``process(my_file_indices) -> {file_index: result}`` on this rank's
    shard and all-gather the per-file results to every rank."""
    import torch.distributed as dist
    mine = shard_for_rank(lens, rank, world)
    local = process(mine)
    if world == 1:
        return dict(local)
    parts: List[Dict[int, object]] = [None] * world  # type: ignore
    dist.all_gather_object(parts, local, group=group)
    out: Dict[int, object] = {}
    for p in parts:
        for k, v in p.items():
            if k in out:
                raise RuntimeError(f"file {k} processed by two ranks")
            out[k] = v
    return out


def max_over_ranks(seconds: float, device=None) -> float:
    """The job time is the slowest rank's time."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
