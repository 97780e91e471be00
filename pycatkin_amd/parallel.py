"""Sharding of condition grids over ranks (one process per GPU).

The MK solves are independent, so the only multi-GPU structure is the split of
the grid and one gather of the results after the solve: no data-path
collective.  With torch.distributed on ROCm the 'nccl' backend is RCCL over
xGMI; the unit tests run the same code on 'gloo'.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n_total, rank, world):
    """Contiguous [start, stop) of `n_total` items owned by `rank` (sizes differ by at most 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError('bad rank/world %d/%d' % (rank, world))
    base, extra = divmod(int(n_total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def weak_grid_rows(rows_per_rank, rank, world, lo=-2.5, hi=0.5, cyclic=True):
    """The bench's weak-scaling grid axis: world*rows_per_rank points on
    [lo, hi].  cyclic (default): `rank` owns rows rank, rank+world, ... -- every
    rank samples the whole descriptor range, so the per-rank cost matches the
    one-GPU grid instead of depending on which band of the volcano a rank got;
    contiguous: rows [rank*rows_per_rank, (rank+1)*rows_per_rank)."""
    axis = np.linspace(lo, hi, rows_per_rank * world)
    if cyclic:
        return axis[rank::world]
    return axis[rank * rows_per_rank:(rank + 1) * rows_per_rank]


def weak_grid_row_index(rows_per_rank, rank, world, cyclic=True):
    """Global row numbers of weak_grid_rows(rows_per_rank, rank, world)."""
    rows = np.arange(rows_per_rank * world)
    return rows[rank::world] if cyclic else rows[rank * rows_per_rank:(rank + 1) * rows_per_rank]


def gather_shards(local, n_total, dist=None, group=None):
    """All-gather every rank's 1-D shard (torch tensor) into the full array on
    each rank (shards may differ in length by one; they are padded to the
    largest for the collective and trimmed afterwards)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    world = dist.get_world_size(group)
    sizes = [shard_bounds(n_total, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    buf = torch.zeros(width, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return torch.cat([o[:b - a] for o, (a, b) in zip(out, sizes)])


def assemble_weak_grid(shards, rows_per_rank, n_cols, perm=None, cyclic=True):
    """Global (world*rows_per_rank, n_cols) map from every rank's flat result
    (the list an all_gather returns, rank order).  `perm` is the device order
    of the local conditions (functions/volcano.py: tile_order), undone first."""
    import torch
    world = len(shards)
    out = torch.empty((rows_per_rank * world, n_cols), dtype=shards[0].dtype, device=shards[0].device)
    inv = None
    if perm is not None:
        inv = np.empty_like(perm)
        inv[perm] = np.arange(perm.size)
        inv = torch.from_numpy(inv).to(shards[0].device)
    for r, s in enumerate(shards):
        local = (s[inv] if inv is not None else s).reshape(rows_per_rank, n_cols)
        out[torch.from_numpy(weak_grid_row_index(rows_per_rank, r, world, cyclic)).to(out.device)] = local
    return out
