"""Multi-GPU sharding of a packet batch.

Packets are independent, so each rank takes a contiguous index range and runs the codec on it
with no data-path collective.  The only cross-rank step is bookkeeping on the host side: the
per-rank VALID counts are summed and the per-rank (order-stable) valid-index lists are
concatenated with each rank's global offset — what an RConn-style caller needs to deliver the
surviving packets in input order.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n packets for `rank` of `world` (floor split, covers n)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return (n * rank) // world, (n * (rank + 1)) // world


def to_global(local_valid_idx, lo: int):
    """Local compacted indices of shard [lo, hi) -> global packet indices."""
    return local_valid_idx + lo


def gather_valid(local_valid_idx, lo: int, group=None):
    """All-gather every rank's VALID list (global indices, input order) and its count over
    torch.distributed (gloo for host tensors).  Returns (global_list, per_rank_counts).  Used
    only for result delivery/bookkeeping; the codec itself never communicates."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    g = to_global(local_valid_idx.to(torch.int64), lo)
    cnt = torch.tensor([g.numel()], dtype=torch.int64)
    counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    padded = torch.full((m,), -1, dtype=torch.int64)
    padded[: g.numel()] = g
    outs = [torch.empty(m, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, padded, group=group)
    return torch.cat([o[:c] for o, c in zip(outs, counts)]), counts
