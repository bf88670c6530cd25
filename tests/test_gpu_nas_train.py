"""Train-mode hardnetNAS on MI355X (second half): hn_nas_train_* through
HardNetNAS.train() and HardNetNASSupernet.train(), against the reference's own training steps
(tests/golden/train_nas.npz, made by tests/golden/make_train_golden.py from
hardnetNAS/supernet_functions/model_supernet.py + training_functions_supernet.py:88-103).

Bars: descriptors 1e-4 max abs (north_star), running statistics 1e-5 relative, the loss 1e-5; the
gradients of all parameters together L2-relative 5e-3 against the reference's fp64 step, and every
single tensor's within 2e-2 (or 3x the reference's own fp32 error on it): a ReLU kink moves one
small tensor (an SE / BN bias summing few entries) by percent in any fp32 implementation
(tests/fixtures.py::nas_grad_check; wang2 measures 1.5e-5 on every tensor)."""
import numpy as np
import pytest
import torch

from fixtures import nas_grad_check, nas_train_start, supernet_start, supernet_step

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["wang2", "cov_b"])
def test_nas_train_step_matches_reference(name, cuda_device):
    """A sampled descriptor (wang2; cov_b: SE and ChannelShuffle in every layer) in the loop's shape:
    two train() calls, the hardnetNAS loss_HardNet (anchor swap), backward."""
    from hardnetnas_amd.losses import loss_HardNet
    m, fx, a, p = nas_train_start(name)
    m = m.to(cuda_device)
    oa = m(torch.from_numpy(a).to(cuda_device))
    op_ = m(torch.from_numpy(p).to(cuda_device))
    assert "NasTrainFunction" in type(oa.grad_fn).__name__
    loss = loss_HardNet(oa, op_, anchor_swap=True)
    loss.backward()
    pre = f"nas_{name}/"
    ea = np.abs(oa.detach().cpu().numpy() - fx[pre + "out_a_32"]).max()
    ep = np.abs(op_.detach().cpu().numpy() - fx[pre + "out_p_32"]).max()
    el = abs(loss.item() - float(fx[pre + "loss_64"]))
    print(f"{name}: out_a {ea:.2e} out_p {ep:.2e} loss {el:.2e}")
    assert ea <= 1e-4 and ep <= 1e-4 and el <= 1e-5
    worst_stat = 0.0
    for k, v in m.state_dict().items():
        if "running" in k:
            ref = fx[f"{pre}stat/{k}_32"]
            worst_stat = max(worst_stat, float(np.abs(v.cpu().numpy() - ref).max() / max(1.0, np.abs(ref).max())))
        if k.endswith("num_batches_tracked"):
            assert int(v) == 2, k
    print(f"{name}: running stats worst rel {worst_stat:.2e}")
    assert worst_stat <= 1e-5
    glob, worst, where = nas_grad_check([(k, t.grad.cpu().numpy()) for k, t in m.named_parameters()], fx, pre)
    print(f"{name}: gradients L2-rel (all) {glob:.2e}, worst tensor {worst:.2e} at {where}")
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)


def test_supernet_step_matches_reference(cuda_device):
    """The supernet search step itself: every layer runs all 17 CANDIDATE_BLOCKS (so every op at
    every layer is exercised, forward and backward), the soft weights come from the fixture's
    recorded Gumbel noise, outs_Y runs under no_grad, the SupernetLoss latency term and the thetas
    gradient flow through the HIP op's soft-weight gradient."""
    m, fx, x, y = supernet_start()
    m = m.to(cuda_device)
    ox, oy, loss, ce, lat = supernet_step(m, fx, x, y, device=cuda_device)
    assert "NasTrainFunction" in type(ox.grad_fn).__name__
    ex = np.abs(ox.detach().cpu().numpy() - fx["super/out_x_32"]).max()
    ey = np.abs(oy.detach().cpu().numpy() - fx["super/out_y_32"]).max()
    print(f"supernet: out_x {ex:.2e} out_y {ey:.2e} loss {loss.item():.6f} vs {float(fx['super/loss_64']):.6f}")
    assert ex <= 1e-4 and ey <= 1e-4
    for k, v in (("loss", loss), ("ce", ce), ("lat", lat)):
        assert abs(float(v.item()) - float(fx[f"super/{k}_64"])) <= 1e-5, k
    tg = torch.stack([st.thetas.grad for st in m.stages_to_search]).cpu().numpy()
    ref = fx["super/thetas_grad_64"]
    et = np.linalg.norm(tg - ref) / np.linalg.norm(ref)
    print(f"supernet: thetas grad L2-rel {et:.2e}")
    assert et <= 5e-3
    named = [(k, t.grad.cpu().numpy()) for k, t in m.named_parameters() if not k.endswith("thetas")]
    glob, worst, where = nas_grad_check(named, fx, "super/", cap=fx["meta"]["supernet"]["sample"])
    print(f"supernet: gradients L2-rel (all) {glob:.2e}, worst tensor {worst:.2e} at {where}")
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)
    names = [str(n) for n in fx["super/stat_names"]]
    sd = m.state_dict()
    for n, ref in zip(names, fx["super/stat_norms_64"]):
        got = float(sd[n].double().norm())
        assert abs(got - ref) <= 1e-5 * max(1.0, ref), n


def test_nas_train_eligibility(cuda_device):
    """Input gradients, CPU tensors and eval mode take the module's torch layers."""
    m, fx, a, _ = nas_train_start("wang2")
    m = m.to(cuda_device)
    x = torch.from_numpy(a[:8]).to(cuda_device)
    assert "NasTrainFunction" in type(m(x).grad_fn).__name__
    xr = x.clone().requires_grad_(True)
    assert "NasTrainFunction" not in type(m(xr).grad_fn).__name__
    m.native_train = False
    assert "NasTrainFunction" not in type(m(x).grad_fn).__name__


def test_nas_train_matches_torch_layers_on_gpu(cuda_device):
    """The HIP train path against the same module's torch layers on the GPU (MIOpen) over wang3
    (maxpool + 1x1 skip ops) at 96 patches: descriptors and gradients."""
    from fixtures import build_module
    from hardnetnas_amd.losses import loss_HardNet
    from hardnetnas_amd import synth
    res = {}
    x = torch.from_numpy(synth.synth_patches(96, seed=41)).to(cuda_device)
    for native in (True, False):
        m, _, _ = build_module("wang3")
        m = m.to(cuda_device).train()
        m.native_train = native
        torch.backends.cudnn.allow_tf32 = False
        y = m(x)
        loss_HardNet(y[:48], y[48:], anchor_swap=True).backward()
        res[native] = (y.detach(), {k: t.grad.detach().clone() for k, t in m.named_parameters()})
    assert (res[True][0] - res[False][0]).abs().max().item() <= 1e-4
    for k, g in res[False][1].items():
        n = g.norm().item()
        if n > 1e-6:
            assert (res[True][1][k] - g).norm().item() / n <= 2e-2, k


@pytest.mark.parametrize("variant", ["NASNet", "NASNet_0.1"])
def test_fdl_train_step_matches_reference(variant, cuda_device):
    """FDLNet HardNetNeiMask.train() on hn_nas_train_* (input_norm, conv0 + bias, the NASNet front's
    BN(affine=False) and stride-2 1x1 convs or the NASNet_0.1 max-pool front, three IRF blocks, the
    4x4 head) against the reference FDLNet module's step (tests/golden/train_fdl.npz)."""
    from fixtures import fdl_train_start
    from hardnetnas_amd.losses import loss_HardNet
    m, fx, a, p = fdl_train_start(variant)
    m = m.to(cuda_device)
    oa = m(torch.from_numpy(a).to(cuda_device))
    op_ = m(torch.from_numpy(p).to(cuda_device))
    assert "NasTrainFunction" in type(oa.grad_fn).__name__
    loss = loss_HardNet(oa, op_, anchor_swap=True)
    loss.backward()
    pre = f"fdl_{variant.replace('.', '')}/"
    ea = np.abs(oa.detach().cpu().numpy() - fx[pre + "out_a_32"]).max()
    ep = np.abs(op_.detach().cpu().numpy() - fx[pre + "out_p_32"]).max()
    el = abs(loss.item() - float(fx[pre + "loss_64"]))
    print(f"{variant}: out_a {ea:.2e} out_p {ep:.2e} loss {el:.2e}")
    assert ea <= 1e-4 and ep <= 1e-4 and el <= 1e-5
    worst_stat = 0.0
    for k, v in m.state_dict().items():
        if "running" in k:
            ref = fx[f"{pre}stat/{k}_32"]
            worst_stat = max(worst_stat, float(np.abs(v.cpu().numpy() - ref).max() / max(1.0, np.abs(ref).max())))
        if k.endswith("num_batches_tracked"):
            assert int(v) == 2, k
    print(f"{variant}: running stats worst rel {worst_stat:.2e}")
    assert worst_stat <= 1e-5
    glob, worst, where = nas_grad_check([(k, t.grad.cpu().numpy()) for k, t in m.named_parameters()], fx, pre)
    print(f"{variant}: gradients L2-rel (all) {glob:.2e}, worst tensor {worst:.2e} at {where}")
    assert glob <= 5e-3 and worst <= 2e-2, (glob, where, worst)


def _native_vs_torch(m_factory, x, cuda_device, freeze=()):
    """One loss_HardNet train step of a fresh module on the HIP train path and on its torch layers
    (MIOpen): (descriptors, {name: grad}) for each."""
    from hardnetnas_amd.losses import loss_HardNet
    res = {}
    h = x.shape[0] // 2
    for native in (True, False):
        m = m_factory().to(cuda_device).train()
        m.native_train = native
        for k, t in m.named_parameters():
            if k in freeze:
                t.requires_grad_(False)
        y = m(x)
        assert ("NasTrainFunction" in type(y.grad_fn).__name__) == native
        loss_HardNet(y[:h], y[h:], anchor_swap=True).backward()
        res[native] = (y.detach(), {k: (t.grad.detach().clone() if t.grad is not None else None)
                                    for k, t in m.named_parameters()})
    return res


def _compare(res, bar=2e-2):
    e = (res[True][0] - res[False][0]).abs().max().item()
    assert e <= 1e-4, e
    worst = 0.0
    for k, g in res[False][1].items():
        gn = res[True][1][k]
        assert (g is None) == (gn is None), k
        if g is None:
            continue
        n = g.norm().item()
        if n > 1e-6:
            r = (gn - g).norm().item() / n
            worst = max(worst, r)
            assert r <= bar, (k, r)
    return e, worst


def test_frozen_parameters_train_natively(cuda_device):
    """Frozen parameters (requires_grad False: the stem conv and an SE conv of cov_b) keep the native
    train path (their gradient slots get throwaway buffers: the kernels write every weight
    gradient) and the other gradients match the torch layers; frozen ones stay None."""
    from fixtures import build_module
    from hardnetnas_amd import synth
    x = torch.from_numpy(synth.synth_patches(64, seed=5)).to(cuda_device)
    freeze = ("first.conv.weight", "stages.2.se4.op.1.weight", "stages.2.se4.op.1.bias")
    res = _native_vs_torch(lambda: build_module("cov_b")[0], x, cuda_device, freeze)
    for k in freeze:
        assert res[True][1][k] is None
    e, worst = _compare(res)
    print(f"frozen: fwd {e:.2e}, worst grad L2-rel {worst:.2e}")


@pytest.mark.parametrize("name,b", [("fdl_NASNet", 1024), ("cov_b", 4096)])
def test_large_batch_train_matches_torch_layers(name, b, cuda_device):
    """Batches whose elementwise kernels cover > 2^24 elements (FDL conv0 bias over 32 x B x 1024;
    SE scale / pool over C x B x 256 at 16 x 16): grid-stride loops, so every element is touched."""
    from fixtures import build_module
    from hardnetnas_amd import synth
    x = torch.from_numpy(synth.synth_patches(b, seed=9)).to(cuda_device)
    e, worst = _compare(_native_vs_torch(lambda: build_module(name)[0], x, cuda_device))
    print(f"{name} B={b}: fwd {e:.2e}, worst grad L2-rel {worst:.2e}")


def test_bn_in_eval_inside_a_train_module_takes_torch_layers(cuda_device):
    """A BatchNorm switched to eval() inside a train() module uses running statistics in the
    reference's layers; the native train path (batch statistics everywhere) must not take it."""
    m, fx, a, _ = nas_train_start("wang2")
    m = m.to(cuda_device)
    x = torch.from_numpy(a[:8]).to(cuda_device)
    m.stages[1].pw.bn.eval()
    assert "NasTrainFunction" not in type(m(x).grad_fn).__name__
