"""hardnetnas_amd.losses (the autograd loss_HardNet for training loops) against the oracle's
restatement and the committed golden loss vectors (hardnet/Losses.py:87-154)."""
import numpy as np
import pytest
import torch

from hardnetnas_amd.losses import distance_matrix_vector, loss_HardNet
from oracle import hardnet_oracle as O


@pytest.mark.parametrize("swap", [False, True])
@pytest.mark.parametrize("loss_type", ["triplet_margin", "softmax", "contrastive"])
def test_matches_oracle_with_duplicates(swap, loss_type):
    g = torch.Generator().manual_seed(3)
    a = torch.nn.functional.normalize(torch.randn(96, 128, generator=g, dtype=torch.float64), dim=1)
    p = torch.nn.functional.normalize(a + 0.05 * torch.randn(96, 128, generator=g, dtype=torch.float64), dim=1)
    p[7] = a[9]  # a near-duplicate negative (masked by the 0.008 rule)
    got = loss_HardNet(a, p, anchor_swap=swap, loss_type=loss_type)
    ref = O.loss_hardnet(a, p, anchor_swap=swap, loss_type=loss_type)
    assert abs(got.item() - ref.item()) <= 1e-12


def test_gradients_flow_and_match_autograd_of_oracle():
    g = torch.Generator().manual_seed(4)
    a0 = torch.randn(64, 128, generator=g, dtype=torch.float64)
    p0 = torch.randn(64, 128, generator=g, dtype=torch.float64)
    a1, p1 = a0.clone().requires_grad_(True), p0.clone().requires_grad_(True)
    a2, p2 = a0.clone().requires_grad_(True), p0.clone().requires_grad_(True)
    loss_HardNet(a1, p1, anchor_swap=True).backward()
    O.loss_hardnet(a2, p2, anchor_swap=True).backward()
    assert torch.allclose(a1.grad, a2.grad, atol=1e-12) and torch.allclose(p1.grad, p2.grad, atol=1e-12)


def test_distance_matrix_and_errors():
    a = torch.eye(4, 128, dtype=torch.float64)
    d = distance_matrix_vector(a, a)
    assert np.allclose(torch.diagonal(d).numpy(), 1e-3)
    with pytest.raises(ValueError):
        loss_HardNet(a, a[:3])
    with pytest.raises(ValueError):
        loss_HardNet(a, a, batch_reduce="average")
