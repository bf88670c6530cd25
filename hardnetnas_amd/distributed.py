"""Patch sharding across the GPUs of one node (BASELINE config 4).

Eval-mode descriptor extraction is embarrassingly parallel: input_norm is per patch and
BatchNorm uses running statistics, so rank r owns the contiguous patch range
``shard_range(n, world, r)`` and runs the forward with no data-path collective.  The only
exchange is the optional all-gather that reassembles the [N,128] descriptor matrix for
the pairwise-distance step (the reference's ``nn.DataParallel`` gather,
hardnetNAS/supernet_main_file.py:60).  One process per GPU; backend "nccl" (= RCCL on
ROCm, over xGMI) on GPUs, "gloo" for the CPU tests.

The triplet-mining step at scale (``sharded_hardnet_loss``, BASELINE config 5 over N GPUs):
rank r owns anchor/positive pairs [s_r, e_r); the positives are all-gathered once, each rank
computes its row block of the B x B masked distance matrix (hn_pairdist_rows), anchor_swap's
column minima are combined with one all-reduce(MIN) of [B] floats, and the loss is the
all-reduced sum of per-rank partial sums scaled by 1/B -- loss_HardNet (hardnet/Losses.py:87-154)
without any rank holding more than its row block.
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


def _rows_torch(a_rows, row0, p_all, col_min):
    """CPU-tensor restatement of hn_pairdist_rows (the module-level CPU path; HIP tensors always
    take the kernel): loss_HardNet's masked matrix rows [row0, row0 + n) (Losses.py:95-108)."""
    d1 = torch.sum(a_rows * a_rows, dim=1).unsqueeze(-1)
    d2 = torch.sum(p_all * p_all, dim=1).unsqueeze(0)
    dm = torch.sqrt(d1 + d2 - 2.0 * a_rows @ p_all.t() + 1e-6) + 1e-8
    n = a_rows.shape[0]
    idx = torch.arange(n)
    pos = dm[idx, row0 + idx]
    d = dm.clone()
    d[idx, row0 + idx] += 10
    d = d + (d < 0.008).to(d.dtype) * 10
    return pos, d.min(dim=1)[0], (d.min(dim=0)[0] if col_min else None)


_LOSS = {"triplet_margin", "softmax", "contrastive"}


def _loss_torch(pos, mn, margin, loss_type):
    if loss_type == "triplet_margin":
        return torch.clamp(margin + pos - mn, min=0.0)
    if loss_type == "softmax":
        ep = torch.exp(2.0 - pos)
        return -torch.log(ep / (ep + torch.exp(2.0 - mn) + 1e-8))
    return torch.clamp(margin - mn, min=0.0) + pos


def sharded_hardnet_loss(a_local: torch.Tensor, p_local: torch.Tensor, n_total: int,
                         anchor_swap: bool = False, margin: float = 1.0,
                         loss_type: str = "triplet_margin", group=None):
    """loss_HardNet (batch_reduce='min') over a pair batch sharded by ``shard_range``:
    returns (loss [1] -- the same on every rank, this rank's pos [n_r], this rank's min_neg
    [n_r]).  Collectives: one all-gather of the positives, one all-reduce(MIN) of the [B]
    column minima (anchor_swap only), one all-reduce(SUM) of the scalar loss."""
    if loss_type not in _LOSS:
        raise ValueError(f"loss_type must be one of {sorted(_LOSS)}")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    s, e = shard_range(n_total, world, rank)
    if a_local.shape != p_local.shape or a_local.shape[0] != e - s:
        raise ValueError("local anchors/positives must be this rank's shard_range slice")
    p_all = gather_descriptors(p_local, n_total, group)
    if a_local.is_cuda:
        from . import _native
        pos, rmin, cmin = _native.pairdist_rows(a_local, s, p_all, col_min=anchor_swap)
    else:
        pos, rmin, cmin = _rows_torch(a_local, s, p_all, anchor_swap)
    if anchor_swap:
        dist.all_reduce(cmin, op=dist.ReduceOp.MIN, group=group)
        cmin = cmin[s:e]
    if a_local.is_cuda:
        loss, mn = _native.hardnet_loss(pos, rmin, cmin, margin, loss_type, scale=1.0 / n_total)
    else:
        mn = torch.minimum(rmin, cmin) if anchor_swap else rmin
        loss = (_loss_torch(pos, mn, margin, loss_type).sum() / n_total).reshape(1)
    dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=group)
    return loss, pos, mn
