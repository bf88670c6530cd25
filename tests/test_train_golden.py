"""Train mode against the reference's own training step (tests/golden/train_hardnet.npz, made by
tests/golden/make_train_golden.py from hardnet/HardNet.py:379-423): two model calls (anchors,
positives), loss_HardNet(anchor_swap=True), backward.  CPU: the oracle's functional train-mode
restatement and the module's torch path.  The HIP train path is checked against the same
fixture in tests/test_gpu_train.py::test_reference_train_step."""
import numpy as np
import pytest
import torch

from fixtures import TRAIN_BN_IDX, TRAIN_CONV_IDX, grad_errors, train_start
from oracle import hardnet_oracle as O


def _check(fx, init, tag, out_a, out_p, loss, rm, rv, grads, out_tol, stat_tol, grad_tol):
    pre = f"{init}/"
    assert np.abs(out_a - fx[f"{pre}out_a_{tag}"]).max() <= out_tol
    assert np.abs(out_p - fx[f"{pre}out_p_{tag}"]).max() <= out_tol
    assert abs(loss - float(fx[f"{pre}loss_64"])) <= max(out_tol, 1e-6)
    for i in TRAIN_BN_IDX:
        for got, key in ((rm[i], "rm"), (rv[i], "rv")):
            ref = fx[f"{pre}{key}{i}_{tag}"]
            assert np.abs(got - ref).max() / max(1e-12, np.abs(ref).max()) <= stat_tol, (key, i)
        assert int(fx[f"{pre}nbt{i}"]) == 2
    for i in TRAIN_CONV_IDX:
        e = grad_errors(grads[i], fx, pre, i)
        assert max(e.values()) <= grad_tol, (i, e)


@pytest.mark.parametrize("init", ["golden", "fresh"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_oracle_train_step_matches_reference(init, dtype):
    m, fx, a, p = train_start(init)
    params = {f"features.{i}.weight": m.features[i].weight.detach().to(dtype).clone().requires_grad_(True)
              for i in TRAIN_CONV_IDX}
    running = {}
    for i in TRAIN_BN_IDX:
        running[f"features.{i}.running_mean"] = m.features[i].running_mean.clone().to(dtype)
        running[f"features.{i}.running_var"] = m.features[i].running_var.clone().to(dtype)
    out_a = O.hardnet_train_forward(params, torch.from_numpy(a), running, 0.1, dtype)
    out_p = O.hardnet_train_forward(params, torch.from_numpy(p), running, 0.1, dtype)
    loss = O.loss_hardnet(out_a, out_p, anchor_swap=True)
    loss.backward()
    tag = "32" if dtype == torch.float32 else "64"
    tol = (1e-5, 1e-5, 5e-3) if tag == "32" else (1e-12, 1e-12, 1e-7)  # sampled entries are stored as fp32
    _check(fx, init, tag, out_a.detach().numpy(), out_p.detach().numpy(), loss.item(),
           {i: running[f"features.{i}.running_mean"].numpy() for i in TRAIN_BN_IDX},
           {i: running[f"features.{i}.running_var"].numpy() for i in TRAIN_BN_IDX},
           {i: params[f"features.{i}.weight"].grad.numpy() for i in TRAIN_CONV_IDX}, *tol)


@pytest.mark.parametrize("init", ["golden", "fresh"])
def test_module_torch_train_step_matches_reference(init):
    """hardnetnas_amd.model.HardNet's torch layers (the CPU path of train()) in the loop's shape."""
    from hardnetnas_amd.losses import loss_HardNet
    m, fx, a, p = train_start(init)
    out_a = m(torch.from_numpy(a))
    out_p = m(torch.from_numpy(p))
    loss = loss_HardNet(out_a, out_p, anchor_swap=True)
    loss.backward()
    _check(fx, init, "32", out_a.detach().numpy(), out_p.detach().numpy(), loss.item(),
           {i: m.features[i].running_mean.numpy() for i in TRAIN_BN_IDX},
           {i: m.features[i].running_var.numpy() for i in TRAIN_BN_IDX},
           {i: m.features[i].weight.grad.numpy() for i in TRAIN_CONV_IDX}, 1e-5, 1e-5, 5e-3)


def test_fixture_fp32_reference_gradient_error_is_recorded():
    """The reference's own fp32 step sits well inside the 5e-3 L2 bar the HIP path is held to."""
    from fixtures import load
    meta = load("train_hardnet")["meta"]
    for init in ("golden", "fresh"):
        errs = meta["inits"][init]["fp32_grad_l2rel_vs_fp64"]
        assert len(errs) == 7 and max(errs.values()) < 2.5e-3



# ---- hardnetNAS: the sampled descriptors and the supernet ------------------------------------
@pytest.mark.parametrize("name", ["wang2", "cov_b"])
def test_module_torch_nas_train_step_matches_reference(name):
    """HardNetNAS's torch layers (the CPU path of train()) in the supernet training loop's shape
    (two calls, hardnetNAS loss_HardNet = anchor swap, backward) against the reference's step."""
    from fixtures import nas_grad_check, nas_train_start
    from hardnetnas_amd.losses import loss_HardNet
    m, fx, a, p = nas_train_start(name)
    oa, op_ = m(torch.from_numpy(a)), m(torch.from_numpy(p))
    loss = loss_HardNet(oa, op_, anchor_swap=True)
    loss.backward()
    pre = f"nas_{name}/"
    assert np.abs(oa.detach().numpy() - fx[pre + "out_a_32"]).max() <= 1e-5
    assert np.abs(op_.detach().numpy() - fx[pre + "out_p_32"]).max() <= 1e-5
    assert abs(loss.item() - float(fx[pre + "loss_64"])) <= 1e-5
    for k, v in m.state_dict().items():
        if "running" in k:
            ref = fx[f"{pre}stat/{k}_32"]
            assert np.abs(v.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), k
    glob, worst, where = nas_grad_check([(k, t.grad.numpy()) for k, t in m.named_parameters()], fx, pre)
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)


@pytest.mark.parametrize("variant", ["NASNet", "NASNet_0.1"])
def test_module_torch_fdl_train_step_matches_reference(variant):
    """HardNetNeiMask's torch layers (the CPU path of train()) against the reference FDLNet module's
    train step (tests/golden/train_fdl.npz: two calls, hardnetNAS loss_HardNet, backward)."""
    from fixtures import fdl_train_start, nas_grad_check
    from hardnetnas_amd.losses import loss_HardNet
    m, fx, a, p = fdl_train_start(variant)
    oa, op_ = m(torch.from_numpy(a)), m(torch.from_numpy(p))
    loss = loss_HardNet(oa, op_, anchor_swap=True)
    loss.backward()
    pre = f"fdl_{variant.replace('.', '')}/"
    assert np.abs(oa.detach().numpy() - fx[pre + "out_a_32"]).max() <= 1e-5
    assert np.abs(op_.detach().numpy() - fx[pre + "out_p_32"]).max() <= 1e-5
    assert abs(loss.item() - float(fx[pre + "loss_64"])) <= 1e-5
    for k, v in m.state_dict().items():
        if "running" in k:
            ref = fx[f"{pre}stat/{k}_32"]
            assert np.abs(v.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), k
    glob, worst, where = nas_grad_check([(k, t.grad.numpy()) for k, t in m.named_parameters()], fx, pre)
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)


def test_supernet_module_torch_step_matches_reference():
    """HardNetNASSupernet (torch layers) with the recorded Gumbel noise reproduces the reference
    supernet's training step (FBNet_Stochastic_SuperNet + SupernetLoss): descriptors, the loss and
    its latency term, the thetas gradient and every weight gradient."""
    from fixtures import nas_grad_check, supernet_start, supernet_step
    m, fx, x, y = supernet_start()
    ox, oy, loss, ce, lat = supernet_step(m, fx, x, y)
    assert np.abs(ox.detach().numpy() - fx["super/out_x_32"]).max() <= 1e-5
    assert np.abs(oy.detach().numpy() - fx["super/out_y_32"]).max() <= 1e-5
    for k in ("loss", "ce", "lat"):
        assert abs(float({"loss": loss, "ce": ce, "lat": lat}[k].item()) - float(fx[f"super/{k}_64"])) <= 1e-5, k
    tg = torch.stack([st.thetas.grad for st in m.stages_to_search]).numpy()
    ref = fx["super/thetas_grad_64"]
    assert np.linalg.norm(tg - ref) / np.linalg.norm(ref) <= 5e-3
    named = [(k, t.grad.numpy()) for k, t in m.named_parameters() if not k.endswith("thetas")]
    glob, worst, where = nas_grad_check(named, fx, "super/", cap=fx["meta"]["supernet"]["sample"])
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)
