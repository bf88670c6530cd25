"""Patch sharding across the GPUs of one node (BASELINE config 4).

Eval-mode descriptor extraction is embarrassingly parallel: input_norm is per patch and
BatchNorm uses running statistics, so rank r owns the contiguous patch range
``shard_range(n, world, r)`` and runs the forward with no data-path collective.  The only
exchange is the optional all-gather that reassembles the [N,128] descriptor matrix for
the pairwise-distance step (the reference's ``nn.DataParallel`` gather,
hardnetNAS/supernet_main_file.py:60).  One process per GPU; backend "nccl" (= RCCL on
ROCm, over xGMI) on GPUs, "gloo" for the CPU tests.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, end) of n patches for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(x: torch.Tensor, group=None) -> torch.Tensor:
    """This rank's slice of a batch that every rank holds (or can index lazily)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    s, e = shard_range(x.shape[0], world, rank)
    return x[s:e]


def gather_descriptors(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather per-rank [n_r,128] descriptors into the full [n_total,128] matrix in
    patch order.  Uses one all_gather_into_tensor when the shards are equal-sized (the
    benchmark configuration), else pads to the largest shard."""
    world = dist.get_world_size(group)
    sizes = [shard_range(n_total, world, r) for r in range(world)]
    counts = [e - s for s, e in sizes]
    d = local.shape[1]
    m = max(counts)
    if local.shape[0] != counts[dist.get_rank(group)]:
        raise ValueError("local shard size does not match shard_range")
    if all(c == m for c in counts):
        out = torch.empty((n_total, d), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    buf = torch.zeros((m, d), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    full = torch.empty((m * world, d), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        parts = list(full.chunk(world))
        dist.all_gather(parts, buf, group=group)
    else:
        dist.all_gather_into_tensor(full, buf, group=group)
    return torch.cat([full[r * m: r * m + counts[r]] for r in range(world)])


@torch.no_grad()
def sharded_forward(model: torch.nn.Module, x_all: torch.Tensor, gather: bool = True,
                    group=None) -> torch.Tensor:
    """Each rank describes its shard of `x_all` with `model` (the HIP path when the model
    is in eval mode on a GPU), then optionally all-gathers the descriptor matrix."""
    n = x_all.shape[0]
    local = model(shard(x_all, group))
    return gather_descriptors(local, n, group) if gather else local
