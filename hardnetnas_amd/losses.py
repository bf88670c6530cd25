"""Differentiable ``loss_HardNet`` for training loops (hardnet/Losses.py:87-154, batch_reduce
'min'), with ``distance_matrix_vector`` (Losses.py:5-13) in the reference's formulation.

The training loop calls it as HardNet.py:408-413.  With batch_reduce 'min' on HIP fp32 [B,128]
descriptors it runs the fused kernels of hn_loss.hip (forward and backward, no B x B matrix); the
autograd formulation below (the B x B matrix materialised, as in the reference) serves CPU / fp64
tensors, the 'average' and 'random' reductions and ``fused=False``.  For inference-time mining at
large B (65,536 pairs) ``hardnetnas_amd._native.pairdist_rows`` / ``hardnet_loss`` and
``hardnetnas_amd.distributed.sharded_hardnet_loss`` run the bf16x3 MFMA pair kernel (forward only).
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
                 loss_type: str = "triplet_margin", fused: bool = True) -> torch.Tensor:
    """Hardest-in-batch margin loss (Losses.py:87-154); anchor_ave is accepted and unused, as there.

    batch_reduce 'min' (the training default, HardNet.py:74) on [B,128] fp32 HIP tensors runs the
    fused kernels (``_native.HardNetLossFunction``: forward and backward without the B x B matrix);
    ``fused=False``, CPU / fp64 tensors and the other reductions run the reference's autograd
    formulation here.  'average' (:124-130) takes every masked entry as a negative, paired -- as in
    the reference -- with the positive distance of its column; 'random' (:131-138) one negative per
    row at torch.randperm(B) drawn from the CPU generator as the reference draws it."""
    if anchor.size() != positive.size() or anchor.dim() != 2:
        raise ValueError("anchor and positive must be 2-D tensors of the same shape")
    if batch_reduce not in ("min", "average", "random"):
        raise ValueError(f"unknown batch_reduce {batch_reduce!r} (min, average or random)")
    if loss_type not in ("triplet_margin", "softmax", "contrastive"):
        raise ValueError(f"unknown loss_type {loss_type!r}")
    if (fused and batch_reduce == "min" and anchor.is_cuda and positive.is_cuda
            and anchor.dtype == torch.float32 and positive.dtype == torch.float32 and anchor.shape[1] == 128):
        from . import _native
        return _native.HardNetLossFunction.apply(anchor, positive, anchor_swap, margin, loss_type)
    eps = 1e-8
    d = distance_matrix_vector(anchor, positive) + eps
    b = d.size(1)
    eye = torch.eye(b, device=d.device, dtype=d.dtype)
    pos1 = torch.diagonal(d)
    dn = d + 10.0 * eye
    dn = dn + 10.0 * (dn < 0.008).to(dn.dtype)  # near-duplicate "negatives" pushed out
    if batch_reduce == "min":
        pos = pos1
        min_neg = dn.min(dim=1)[0]
        if anchor_swap:
            min_neg = torch.minimum(min_neg, dn.min(dim=0)[0])
    elif batch_reduce == "average":
        pos = pos1.repeat(anchor.size(0))          # entry k pairs with pos1[k % B]
        min_neg = dn.reshape(-1)                   # entry k = dn[k // B][k % B]
        if anchor_swap:
            min_neg = torch.minimum(min_neg, dn.t().contiguous().reshape(-1))
    else:
        idxs = torch.randperm(anchor.size(0)).long().to(d.device)
        min_neg = dn.gather(1, idxs.view(-1, 1)).reshape(-1)
        if anchor_swap:
            min_neg = torch.minimum(min_neg, dn.t().gather(1, idxs.view(-1, 1)).reshape(-1))
        pos = pos1
    if loss_type == "triplet_margin":
        loss = torch.clamp(margin + pos - min_neg, min=0.0)
    elif loss_type == "softmax":
        e_pos = torch.exp(2.0 - pos)
        loss = -torch.log(e_pos / (e_pos + torch.exp(2.0 - min_neg) + eps))
    else:
        loss = torch.clamp(margin - min_neg, min=0.0) + pos
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
