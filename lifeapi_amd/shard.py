"""Data-parallel sharding of a universe batch across ranks (one process per GPU).

Universes are independent (no halo, no exchange: SURVEY.md 8(e)), so a batch
shards into contiguous ranges with no collective on the data path.  The only
collective is result collection after the kernels: an all-gather of the
per-universe 64-bit hashes (RCCL over xGMI on GPUs, gloo on CPU tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def weak_shard(rank: int, n_per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns universes [r*n, (r+1)*n) of the global array."""
    return rank * n_per_rank, n_per_rank


def strong_shard(rank: int, world: int, n_total: int) -> tuple[int, int]:
    """Strong scaling: near-equal contiguous slices of a fixed n_total."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi - lo


def gather_hashes(h: torch.Tensor, world: int, counts: list[int] | None = None) -> torch.Tensor:
    """All-gather per-universe hashes (int64) in rank order.

    Equal shard sizes use one all_gather_into_tensor; ragged shards (strong
    scaling with n_total % world != 0) pad to the largest shard and trim.
    With a process group the collective runs at every world size (one rank
    under the launcher included); without one, world 1 returns `h`.
    """
    if world == 1 and not dist.is_initialized():
        return h
    n = h.numel()
    if counts is None:
        counts = [n] * world
    m = max(counts)
    src = h if n == m else torch.cat([h, h.new_zeros(m - n)])
    if dist.get_backend() == "gloo":
        parts = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(parts, src)
        out = torch.cat(parts)
    else:
        out = torch.empty(world * m, dtype=h.dtype, device=h.device)
        dist.all_gather_into_tensor(out, src)
    if all(c == m for c in counts):
        return out
    return torch.cat([out[r * m: r * m + counts[r]] for r in range(world)])
