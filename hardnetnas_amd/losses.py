"""Differentiable ``loss_HardNet`` for training loops (hardnet/Losses.py:87-154, batch_reduce
'min'), with ``distance_matrix_vector`` (Losses.py:5-13) in the reference's formulation.

This is the autograd form the reference training loop calls (HardNet.py:392-397): the B x B
distance matrix is materialised (1024 pairs = 1 M entries), so gradients flow to both inputs
through the selected hardest negatives exactly as in the reference.  For inference-time mining
at large B (65,536 pairs: a 17 GB matrix) use ``hardnetnas_amd._native.pairdist_rows`` /
``hardnet_loss`` and ``hardnetnas_amd.distributed.sharded_hardnet_loss``, the fused MFMA kernel
that never materialises it (forward only).
"""
from __future__ import annotations

import torch

__all__ = ["distance_matrix_vector", "loss_HardNet", "SupernetLoss"]


def distance_matrix_vector(anchor: torch.Tensor, positive: torch.Tensor) -> torch.Tensor:
    """sqrt(|a_i|^2 + |p_j|^2 - 2 a_i . p_j + 1e-6) (Losses.py:5-13)."""
    a2 = (anchor * anchor).sum(dim=1, keepdim=True)
    p2 = (positive * positive).sum(dim=1, keepdim=True)
    return torch.sqrt(a2 + p2.t() - 2.0 * anchor @ positive.t() + 1e-6)


def loss_HardNet(anchor: torch.Tensor, positive: torch.Tensor, anchor_swap: bool = False,
                 anchor_ave: bool = False, margin: float = 1.0, batch_reduce: str = "min",
                 loss_type: str = "triplet_margin") -> torch.Tensor:
    """Hardest-in-batch margin loss (Losses.py:87-154); batch_reduce 'min' only (the reference
    training default, HardNet.py:392-397); anchor_ave is accepted and unused, as there."""
    if anchor.size() != positive.size() or anchor.dim() != 2:
        raise ValueError("anchor and positive must be 2-D tensors of the same shape")
    if batch_reduce != "min":
        raise ValueError(f"batch_reduce {batch_reduce!r} is not supported (only 'min')")
    eps = 1e-8
    d = distance_matrix_vector(anchor, positive) + eps
    eye = torch.eye(d.size(1), device=d.device, dtype=d.dtype)
    pos = torch.diagonal(d)
    dn = d + 10.0 * eye
    dn = dn + 10.0 * (dn < 0.008).to(dn.dtype)  # near-duplicate "negatives" pushed out
    min_neg = dn.min(dim=1)[0]
    if anchor_swap:
        min_neg = torch.minimum(min_neg, dn.min(dim=0)[0])
    if loss_type == "triplet_margin":
        loss = torch.clamp(margin + pos - min_neg, min=0.0)
    elif loss_type == "softmax":
        e_pos = torch.exp(2.0 - pos)
        loss = -torch.log(e_pos / (e_pos + torch.exp(2.0 - min_neg) + eps))
    elif loss_type == "contrastive":
        loss = torch.clamp(margin - min_neg, min=0.0) + pos
    else:
        raise ValueError(f"unknown loss_type {loss_type!r}")
    return loss.mean()


class SupernetLoss(torch.nn.Module):
    """The supernet search loss (hardnetNAS/supernet_functions/model_supernet.py:88-110):
    alpha * (loss_HardNet(outs, targets) + clamp(log(latency^beta) * (log(((sample_latency - target)
    / target)^2) + 5) * 0.2, 0)), with the hardnetNAS loss_HardNet (general_functions/Losses.py:27-51:
    anchor swap always on, margin 1).  alpha 0.2, beta 0.6 (config_for_supernet.py)."""

    def __init__(self, alpha: float = 0.2, beta: float = 0.6):
        super().__init__()
        self.alpha, self.beta = alpha, beta

    def forward(self, outs, targets, latency, sample_latency, target):
        ce = loss_HardNet(outs, targets, anchor_swap=True)
        lat = torch.clamp(torch.log(latency ** self.beta) * (torch.log(((sample_latency - target) / target) ** 2) + 5)
                          * 0.2, 0)
        loss = self.alpha * (ce + lat)
        return loss, ce, lat
