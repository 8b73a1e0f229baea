"""Pair-list sharding across ranks (one process per GPU) and the contact all-gather.

Pairs are independent, so a job of P pairs splits into contiguous shards with no data-path
exchange; the only collective is the all-gather of fixed-size contact records (RCCL over xGMI on
MI355X, gloo in the CPU tests) when every rank needs every contact (config C3).
"""
from __future__ import annotations


def shard_range(total_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """[first, first + count) of the pair list owned by `rank`; shards differ by at most one pair."""
    if world < 1 or not 0 <= rank < world or total_pairs < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total_pairs, world)
    first = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return first, count


def allgather_records(local, world: int, group=None):
    """All-gather equal-size uint8 record shards (torch tensors) into rank order.
    `local` must hold the same number of bytes on every rank (use equal shards)."""
    import torch
    import torch.distributed as dist

    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out
