"""The triplet-mining step on MI355X (BASELINE config 5): the fused
masked distance + hardest negative (hardnet/Losses.py:5-13, 87-154) against the fp64 oracle --
row blocks of a sharded batch, descriptors that are not unit-norm (dm > 10, where the +10 mask
must not win), the full 65,536-pair batch on a row sample, and the three margin losses."""
import numpy as np
import pytest
import torch

from oracle import hardnet_oracle as O

pytestmark = pytest.mark.gpu


def _pairs(b, seed, scale=1.0, dup=()):
    g = torch.Generator().manual_seed(seed)
    a = torch.nn.functional.normalize(torch.randn(b, 128, generator=g), dim=1)
    p = torch.nn.functional.normalize(a + 0.3 * torch.randn(b, 128, generator=g), dim=1)
    for i, j in dup:  # positive i is (almost) anchor j: dm < 0.008 off the diagonal
        p[i] = a[j] + 1e-4 * torch.randn(128, generator=g)
    return a * scale, p * scale


@pytest.mark.parametrize("swap", [False, True])
@pytest.mark.parametrize("scale", [1.0, 9.0])
def test_pairdist_unnormalised_and_duplicates(swap, scale, cuda_device):
    from hardnetnas_amd._native import pairdist_hardneg
    # near-duplicates only at unit norm: at |a| = 9 the fp32 form |a|^2 + |p|^2 - 2 a.p loses
    # ~1e-5 absolute to cancellation, which a distance of ~0.008 cannot absorb (the reference's
    # fp32 arithmetic has the same conditioning)
    a, p = _pairs(1000, 3, scale, dup=[(5, 9), (700, 12), (13, 13)] if scale == 1.0 else [])
    pos, mn = pairdist_hardneg(a.to(cuda_device), p.to(cuda_device), swap)
    rpos, rmn = O.hardest_negative(a.double(), p.double(), swap)
    tol = 1e-4 * scale
    assert (pos.cpu().double() - rpos).abs().max().item() < tol
    assert (mn.cpu().double() - rmn).abs().max().item() < tol


@pytest.mark.parametrize("swap", [False, True])
def test_row_shards_reassemble_the_full_result(swap, cuda_device):
    """Three uneven row blocks (hn_pairdist_rows) + min over their column minima == the
    single-call result, bit for bit (same kernel, same per-element arithmetic)."""
    from hardnetnas_amd._native import hardnet_loss, pairdist_hardneg, pairdist_rows
    a, p = _pairs(3001, 4, dup=[(100, 2000)])
    a, p = a.to(cuda_device), p.to(cuda_device)
    pos_f, mn_f = pairdist_hardneg(a, p, swap)
    cuts = [0, 1000, 2200, 3001]
    parts, cmins = [], []
    for s, e in zip(cuts, cuts[1:]):
        pos, rmin, cmin = pairdist_rows(a[s:e], s, p, col_min=swap)
        parts.append((pos, rmin))
        cmins.append(cmin)
    pos = torch.cat([x[0] for x in parts])
    if swap:
        cm = torch.stack(cmins).min(dim=0)[0]
        mn = torch.cat([hardnet_loss(x[0], x[1], cm[s:e])[1] for x, s, e in zip(parts, cuts, cuts[1:])])
    else:
        mn = torch.cat([x[1] for x in parts])
    assert torch.equal(pos, pos_f)
    assert torch.equal(mn, mn_f)


def test_full_config5_batch_on_a_row_sample(cuda_device):
    """65,536 pairs with anchor_swap (BASELINE config 5's distance step): 256 sampled rows of
    pos / min_neg against the fp64 oracle restricted to those rows and columns."""
    from hardnetnas_amd._native import pairdist_hardneg
    b = 65536
    a, p = _pairs(b, 6, dup=[(17, 40000)])
    pos, mn = pairdist_hardneg(a.to(cuda_device), p.to(cuda_device), True)
    rows = torch.cat([torch.arange(0, b, b // 254)[:254], torch.tensor([17, b - 1])])
    rpos, rmn = O.hardest_negative_rows(a.double(), p.double(), rows, True)
    assert (pos.cpu()[rows].double() - rpos).abs().max().item() < 1e-4
    assert (mn.cpu()[rows].double() - rmn).abs().max().item() < 1e-4


@pytest.mark.parametrize("loss_type", ["triplet_margin", "softmax", "contrastive"])
@pytest.mark.parametrize("swap", [False, True])
def test_hardnet_loss_matches_reference(loss_type, swap, cuda_device):
    from hardnetnas_amd._native import hardnet_loss, pairdist_rows
    a, p = _pairs(777, 8, dup=[(1, 2)])
    ad, pd = a.to(cuda_device), p.to(cuda_device)
    pos, rmin, cmin = pairdist_rows(ad, 0, pd, col_min=swap)
    loss, mn = hardnet_loss(pos, rmin, cmin, margin=1.0, loss_type=loss_type)
    ref = O.loss_hardnet(a.double(), p.double(), swap, loss_type=loss_type).item()
    assert abs(loss.item() - ref) < 1e-5
    _, rmn = O.hardest_negative(a.double(), p.double(), swap)
    assert (mn.cpu().double() - rmn).abs().max().item() < 1e-4


_REG_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from test_gpu_pairs import _pairs
from hardnetnas_amd._native import pairdist_rows
dev = torch.device("cuda:0")
out = {}
for b, swap in ((1000, True), (65536 + 37, True), (4097, False)):
    a, p = _pairs(b, 11, dup=[(3, 9)])
    pos, rmin, cmin = pairdist_rows(a.to(dev), 0, p.to(dev), col_min=swap)
    out[f"{b}_{swap}"] = [pos.cpu(), rmin.cpu()] + ([cmin.cpu()] if cmin is not None else [])
torch.save(out, sys.argv[2])
"""


def test_lds_dma_ring_equals_register_staged_form(tmp_path, cuda_device):
    """The LDS-DMA ring pair kernel (default) and the register-staged one (HN_PAIRDIST_REG=1, read
    once per process: a child process) stage the same bf16 hi / lo values and run the same MFMA
    chains: pos, row minima and column minima agree bit for bit, including a batch that is not a
    multiple of the 64-column tile and the 8-wave (>= 65,536 anchors) form.  The same for the ring kernel
    with the next-but-one tile's DMA issued at once instead of spread over the first sub-tile's chain
    (HN_PAIRDIST_SPREAD=0)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for tag, env in (("ring", {}), ("reg", {"HN_PAIRDIST_REG": "1"}), ("nospread", {"HN_PAIRDIST_SPREAD": "0"})):
        f = str(tmp_path / f"{tag}.pt")
        r = subprocess.run([sys.executable, "-c", _REG_CHILD, here, f], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-3000:]
        res[tag] = torch.load(f, weights_only=True)
    for other in ("reg", "nospread"):  # nospread: the ring kernel without the spread next-but-one tile DMA
        for k in res["ring"]:
            for x, y in zip(res["ring"][k], res[other][k]):
                if x is not None:
                    assert torch.equal(x, y), (other, k)


LOSS_TYPES = ["triplet_margin", "softmax", "contrastive"]


@pytest.mark.parametrize("swap", [False, True])
@pytest.mark.parametrize("loss_type", LOSS_TYPES)
def test_fused_train_loss_matches_reference_backward(swap, loss_type, cuda_device):
    """loss_HardNet 'min' on HIP tensors runs hn_hardnet_loss_train_forward / hn_hardnet_loss_backward
    (no B x B matrix): loss and d loss / d (anchor, positive) against the reference's fp64 step
    (tests/golden/loss_modes.npz: a masked near-duplicate and a zero positive distance included);
    loss <= max(1e-6, the reference's own fp32 error) and gradients L2-relative <= 1e-5 (or 3x the
    reference's own fp32 error).  Run twice: bit-identical -- the backward's atomicAdds only count each
    target's sources (k_lmin_bwd_count / _fill); the gather sorts every target's source list before it
    sums, so the summation order does not depend on the order the atomics land in."""
    from fixtures import load
    from hardnetnas_amd.losses import loss_HardNet
    fx = load("loss_modes")
    tag = f"{int(swap)}_{loss_type}"
    res = []
    for _ in range(2):
        a = torch.from_numpy(fx["a"]).to(cuda_device).requires_grad_(True)
        p = torch.from_numpy(fx["p"]).to(cuda_device).requires_grad_(True)
        loss = loss_HardNet(a, p, anchor_swap=swap, loss_type=loss_type)
        assert "HardNetLossFunction" in type(loss.grad_fn).__name__
        loss.backward()
        res.append((loss.item(), torch.cat([a.grad, p.grad]).cpu().numpy()))
    assert res[0][0] == res[1][0] and np.array_equal(res[0][1], res[1][1])
    el = abs(res[0][0] - float(fx[f"min_{tag}_64"]))
    ref = fx[f"g_{tag}"].astype(np.float64)
    eg = np.linalg.norm(res[0][1] - ref) / np.linalg.norm(ref)
    print(f"{tag}: loss {el:.2e}, grad L2-rel {eg:.2e} (reference fp32: {float(fx[f'g32err_{tag}']):.2e})")
    # the per-row losses are fp32 as the reference's, their mean is summed in fp64: the loss must be as
    # close to the fp64 reference as the reference's own fp32 step is (2e-6 for 'contrastive', a mean of
    # distances)
    assert el <= max(1e-6, 1.0 * abs(float(fx[f"min_{tag}_32"]) - float(fx[f"min_{tag}_64"])))
    assert eg <= max(1e-5, 3 * float(fx[f"g32err_{tag}"]))


@pytest.mark.parametrize("b", [512, 4096])
def test_fused_train_loss_matches_autograd_on_gpu(b, cuda_device):
    """The fused loss against the autograd formulation on the same GPU (fused=False) at the training
    loop's batch (512, HardNet.py:98) and 4,096 pairs of unit descriptors, anchor_swap on."""
    from hardnetnas_amd.losses import loss_HardNet
    g = torch.Generator(device=cuda_device).manual_seed(b)
    a0 = torch.nn.functional.normalize(torch.randn(b, 128, device=cuda_device, generator=g), dim=1)
    p0 = torch.nn.functional.normalize(a0 + 0.4 * torch.randn(b, 128, device=cuda_device, generator=g), dim=1)
    out = {}
    for fused in (True, False):
        a, p = a0.clone().requires_grad_(True), p0.clone().requires_grad_(True)
        loss = loss_HardNet(a, p, anchor_swap=True, fused=fused)
        loss.backward()
        out[fused] = (loss.item(), torch.cat([a.grad, p.grad]))
    el = abs(out[True][0] - out[False][0]) / abs(out[False][0])
    eg = ((out[True][1] - out[False][1]).norm() / out[False][1].norm()).item()
    print(f"B={b}: loss rel {el:.2e}, grad L2-rel {eg:.2e}")
    assert el <= 1e-5 and eg <= 1e-4


@pytest.mark.parametrize("swap", [True, False])
@pytest.mark.parametrize("loss_type", ["triplet_margin", "contrastive"])
def test_fused_train_loss_ties(swap, loss_type, cuda_device):
    """Hand-built ties: duplicated positives make two columns of a row exactly equal, and
    duplicated anchors make a column's minimum appear in two rows of different 64-row workgroups (B = 200),
    so the first-index rule of the u64 atomicMin keys is exercised across workgroups; duplicated pairs also
    make the row and the column minimum of a row equal (anchor_swap's 0.5 / 0.5 split).  Loss and
    gradients against the module formulation in fp64 (hardnetnas_amd.losses, fused=False); a heavily
    selected target (one positive picked by every row) exercises the gather's long-list path."""
    from hardnetnas_amd.losses import loss_HardNet
    g = torch.Generator().manual_seed(7)
    b = 200
    unit = lambda v: torch.nn.functional.normalize(v, dim=-1)  # noqa: E731
    c = unit(torch.randn(128, generator=g))
    a = unit(c + 0.5 * unit(torch.randn(b, 128, generator=g)))   # anchors clustered around c
    p = unit(a + 0.3 * unit(torch.randn(b, 128, generator=g)))
    p[150] = p[20]          # equal columns 20 / 150 for every row (tie across column tiles)
    a[130] = a[10]          # equal rows 10 / 130 (different 64-row workgroups)
    a[77], p[77] = a[5].clone(), p[5].clone()  # a duplicated pair: row / column minima tie
    a2, p2 = a.clone(), p.clone()
    p2[3] = c               # case 2: the cluster centre is every anchor's hardest negative (long list)
    for aa, pp in ((a, p), (a2, p2)):
        x = aa.to(cuda_device).requires_grad_(True)
        y = pp.to(cuda_device).requires_grad_(True)
        loss = loss_HardNet(x, y, anchor_swap=swap, loss_type=loss_type)
        loss.backward()
        x64 = aa.double().requires_grad_(True)
        y64 = pp.double().requires_grad_(True)
        ref = loss_HardNet(x64, y64, anchor_swap=swap, loss_type=loss_type, fused=False)
        ref.backward()
        assert abs(loss.item() - ref.item()) <= 1e-5
        gr = torch.cat([x64.grad, y64.grad]).float()
        gg = torch.cat([x.grad, y.grad]).cpu()
        assert (gg - gr).norm() / gr.norm() <= 1e-4, float((gg - gr).norm() / gr.norm())
