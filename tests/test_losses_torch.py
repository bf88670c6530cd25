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
        loss_HardNet(a, a, batch_reduce="L2Net")


LT = ["triplet_margin", "softmax", "contrastive"]


@pytest.mark.parametrize("swap", [False, True])
@pytest.mark.parametrize("loss_type", LT)
def test_average_and_random_reductions_match_reference(swap, loss_type):
    """batch_reduce 'average' / 'random' (Losses.py:124-138) against the reference's own values
    (tests/golden/loss_modes.npz; 'random' draws torch.randperm after torch.manual_seed(23))."""
    from fixtures import load
    fx = load("loss_modes")
    a, p = torch.from_numpy(fx["a"]).double(), torch.from_numpy(fx["p"]).double()
    tag = f"{int(swap)}_{loss_type}"
    got = loss_HardNet(a, p, anchor_swap=swap, batch_reduce="average", loss_type=loss_type).item()
    assert abs(got - float(fx[f"average_{tag}"])) <= 1e-12
    torch.manual_seed(fx["meta"]["random_seed"])
    got = loss_HardNet(a, p, anchor_swap=swap, batch_reduce="random", loss_type=loss_type).item()
    assert abs(got - float(fx[f"random_{tag}"])) <= 1e-12


@pytest.mark.parametrize("swap", [False, True])
@pytest.mark.parametrize("loss_type", LT)
def test_min_gradients_match_reference(swap, loss_type):
    """The autograd formulation's gradients (the CPU path) against the reference's fp64 backward."""
    from fixtures import load
    fx = load("loss_modes")
    a = torch.from_numpy(fx["a"]).double().requires_grad_(True)
    p = torch.from_numpy(fx["p"]).double().requires_grad_(True)
    tag = f"{int(swap)}_{loss_type}"
    loss = loss_HardNet(a, p, anchor_swap=swap, loss_type=loss_type)
    loss.backward()
    assert abs(loss.item() - float(fx[f"min_{tag}_64"])) <= 1e-12
    g = torch.cat([a.grad, p.grad]).numpy()
    ref = fx[f"g_{tag}"].astype(np.float64)
    assert np.linalg.norm(g - ref) / np.linalg.norm(ref) <= 1e-6
