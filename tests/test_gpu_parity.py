"""Parity of the HIP path (through the C ABI) with the reference vectors and the oracle.

Tolerances (BASELINE.json north_star: <= 1e-4 max abs on the 128-D descriptor):
  HardNet  -- bf16x3 split-precision MFMA: 1e-4 max abs vs the reference fp32 forward.
  NAS      -- fp16x3 MFMA 1x1 convs/head + fp32 depthwise: 2e-5 max abs (the old exact-fp32 budget).
  FDL      -- FDLNet HardNetNeiMask: fp32 VALU front + the NAS kernels: 2e-5 max abs.
"""
import os

import numpy as np
import pytest

from hardnetnas_amd import arch as A
import torch

from fixtures import FDL_NAMES, NAS_NAMES, build_module, load, golden_inputs
from oracle import hardnet_oracle as O

pytestmark = pytest.mark.gpu

TOL = {"hardnet": 1e-4}
NAS_TOL = 2e-5


def _tol(name):
    return TOL.get(name, NAS_TOL)


def _native_lib_loaded():
    maps = open("/proc/self/maps").read()
    return "libhardnet_mi355x.so" in maps


@pytest.mark.parametrize("name", ["hardnet"] + NAS_NAMES + FDL_NAMES)
def test_forward_matches_reference_vectors(name, cuda_device):
    m, fx, _ = build_module(name)
    m = m.to(cuda_device)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    with torch.no_grad():
        y = m(x).cpu().numpy()
    assert _native_lib_loaded()
    err = np.abs(y - fx["y"]).max()
    err64 = np.abs(y - fx["y64"]).max()
    print(f"{name}: max|hip - ref32| = {err:.3e}, max|hip - ref64| = {err64:.3e}")
    assert err <= _tol(name)
    xe = torch.from_numpy(fx["x_edge"]).to(cuda_device)
    with torch.no_grad():
        ye = m(xe).cpu().numpy()
    assert np.abs(ye - fx["y_edge"]).max() <= _tol(name)


@pytest.mark.parametrize("name", ["hardnet", "wang2", "wang3", "fdl_NASNet", "fdl_NASNet_01"])
@pytest.mark.parametrize("b", [1, 3, 63, 65, 130, 255])
def test_ragged_batches(name, b, cuda_device):
    m, fx, _ = build_module(name)
    m = m.to(cuda_device)
    x = torch.from_numpy(golden_inputs(fx)[:b]).to(cuda_device)
    with torch.no_grad():
        y = m(x).cpu().numpy()
    assert y.shape == (b, 128)
    assert np.abs(y - fx["y"][:b]).max() <= _tol(name)


def test_empty_batch(cuda_device):
    m, _, _ = build_module("hardnet")
    m = m.to(cuda_device)
    with torch.no_grad():
        y = m(torch.empty(0, 1, 32, 32, device=cuda_device))
    assert tuple(y.shape) == (0, 128)


@pytest.mark.parametrize("name", ["hardnet", "cov_a"])
def test_chunked_forward_equals_unchunked(name, cuda_device, monkeypatch):
    """HN_CHUNK splits the batch inside hn_forward; results must be identical."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    full = NativeModel.from_module(m, cuda_device)(x)
    monkeypatch.setenv("HN_CHUNK", "100")
    chunked = NativeModel.from_module(m, cuda_device)(x)
    assert torch.equal(full, chunked)


@pytest.mark.parametrize("variant", ["000000", "505000", "606000", "6050f0", "605g0g", "605gfg", "605gig"])
def test_tiling_variants_match_reference(variant, cuda_device, monkeypatch):
    """The product library's fallback tilings (HN_VARIANT digits per conv layer; the defaults are 6 0 5 q i l):
    0 = k_conv3x3 everywhere, 5 / 6 = warp-specialised stem+conv1 / conv2, f / i = conv4 on the 64-byte window
    (MFMA-wave / producer-wave stores), g = direct conv3 / conv5 -- against the reference vectors."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    monkeypatch.setenv("HN_VARIANT", variant)
    monkeypatch.setenv("HN_NO_C12", "1")  # the per-layer conv1 / conv2 kernels
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    y = NativeModel.from_module(m, cuda_device)(x).cpu().numpy()
    assert np.abs(y - fx["y"]).max() <= TOL["hardnet"]


@pytest.mark.parametrize("variant", ["605lil", "605qiq", "605qil", "605gil", "605qig"])
def test_winograd_1d_conv3_conv5_match_reference(variant, cuda_device, monkeypatch):
    """conv3 / conv5 as 1-D Winograd F(2,3) (hn_wino1.hip, HN_VARIANT digits l / q = weight ring depth 6 / 8;
    the shallower rings j / k and the F(4,3) conv3 w / x are experiments-library only) against the reference's
    fp32 and fp64 vectors (edge patches included) and against the direct kernels on ragged batches whose last
    two-patch conv5 tile is half empty.  605qil is the default."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    xe = torch.from_numpy(fx["x_edge"]).to(cuda_device)
    monkeypatch.setenv("HN_VARIANT", "605gig")  # the direct conv3 / conv5 kernels
    direct = NativeModel.from_module(m, cuda_device)
    monkeypatch.setenv("HN_VARIANT", variant)
    nm = NativeModel.from_module(m, cuda_device)
    y = nm(x).cpu().numpy()
    ye = nm(xe).cpu().numpy()
    e32 = max(np.abs(y - fx["y"]).max(), np.abs(ye - fx["y_edge"]).max())
    e64 = max(np.abs(y - fx["y64"]).max(), np.abs(ye - fx["y_edge64"]).max())
    print(f"{variant}: max abs vs reference fp32 {e32:.2e}, fp64 {e64:.2e}")
    assert e32 <= TOL["hardnet"] and e64 <= TOL["hardnet"]
    for b in (1, 3, 255):
        assert (nm(x[:b]) - direct(x[:b])).abs().max().item() <= 5e-5


def test_conv4_producer_stores_are_bit_identical(cuda_device, monkeypatch):
    """conv4 with its outputs staged in LDS and stored by the producer waves (HN_VARIANT digit i)
    against the MFMA waves' own stores (digit f): same arithmetic, so identical bits, including
    ragged batches whose last two-patch tile is half empty."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    out = {}
    for v in ("605gfg", "605gig"):
        monkeypatch.setenv("HN_VARIANT", v)
        nm = NativeModel.from_module(m, cuda_device)
        out[v] = [nm(x[:b]) for b in (1, 3, 255, x.shape[0])]
    for a, b in zip(out["605gfg"], out["605gig"]):
        assert torch.equal(a, b)


def test_fused_c12_is_default_and_matches_layerwise(cuda_device, monkeypatch):
    """k_c12 (input_norm + conv0 + conv1 + conv2 in one kernel) runs by default; it matches the
    reference vectors and the layer-by-layer kernels (HN_NO_C12=1) on ragged batches that end
    mid-workgroup-range."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x).cpu().numpy()
    assert "stem+conv1+conv2" in nm.stage_times()
    assert np.abs(y - fx["y"]).max() <= TOL["hardnet"]
    xe = torch.from_numpy(fx["x_edge"]).to(cuda_device)
    assert np.abs(nm(xe).cpu().numpy() - fx["y_edge"]).max() <= TOL["hardnet"]
    monkeypatch.setenv("HN_NO_C12", "1")
    lw = NativeModel.from_module(m, cuda_device)
    for b in (1, 5, 255):
        assert np.abs(nm(x[:b]).cpu().numpy() - lw(x[:b]).cpu().numpy()).max() <= 2e-5


def test_c12_winograd_conv1_matches_reference(cuda_device, monkeypatch):
    """The default k_c12s (HN_C12_CFG=15: conv1 as a 1-D Winograd F(4,3), conv1 and conv2 + stem waves per SIMD,
    bands software-pipelined, hn_c12w.hip) against the reference vectors (edge patches included) at the 1e-4 bar,
    and within 5e-5 of the direct k_c12 (HN_C12_CFG=12, the product library's fallback) -- the transform changes
    the rounding: tests/precision/wino1d_precision.py puts it at 1.7e-5 from fp64 vs 1.0e-5 direct; bit-identical
    to itself on ragged batches and on a persistent run of several patches per workgroup."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    xe = torch.from_numpy(fx["x_edge"]).to(cuda_device)
    monkeypatch.setenv("HN_C12_CFG", "12")  # read once, by hn_create
    direct = NativeModel.from_module(m, cuda_device)
    y0 = direct(x).cpu().numpy()
    assert np.abs(y0 - fx["y"]).max() <= TOL["hardnet"]
    assert np.abs(direct(xe).cpu().numpy() - fx["y_edge"]).max() <= TOL["hardnet"]
    monkeypatch.setenv("HN_C12_CFG", "15")
    nm = NativeModel.from_module(m, cuda_device)
    y = nm(x).cpu().numpy()
    err, err64 = np.abs(y - fx["y"]).max(), np.abs(y - fx["y64"]).max()
    print(f"k_c12s: max|hip - ref32| = {err:.3e}, max|hip - ref64| = {err64:.3e}, vs direct {np.abs(y - y0).max():.3e}")
    assert err <= TOL["hardnet"]
    assert np.abs(y - y0).max() <= 5e-5
    assert np.abs(nm(xe).cpu().numpy() - fx["y_edge"]).max() <= TOL["hardnet"]
    for b in (1, 3, 130):
        assert np.abs(nm(x[:b]).cpu().numpy() - y[:b]).max() == 0.0
        assert np.abs(nm(x[:b]).cpu().numpy() - direct(x[:b]).cpu().numpy()).max() <= 5e-5
    xr = x.repeat(12, 1, 1, 1)[:3001]
    yr = nm(xr).cpu().numpy()
    assert np.abs(yr - np.tile(y, (12, 1))[:3001]).max() == 0.0
    assert np.abs(yr - direct(xr).cpu().numpy()).max() <= 5e-5


def test_unfused_stem_matches(cuda_device, monkeypatch):
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    monkeypatch.setenv("HN_UNFUSED_STEM", "1")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    y = NativeModel.from_module(m, cuda_device)(x).cpu().numpy()
    assert np.abs(y - fx["y"]).max() <= TOL["hardnet"]


def test_deterministic_and_batch_independent(cuda_device):
    m, fx, _ = build_module("hardnet")
    m = m.to(cuda_device)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    with torch.no_grad():
        y1 = m(x)
        y2 = m(x)
        perm = torch.randperm(x.shape[0], device=cuda_device)
        y3 = m(x[perm])
        y4 = torch.cat([m(x[:100]), m(x[100:])])
    assert torch.equal(y1, y2)
    assert torch.equal(y3, y1[perm])
    assert torch.equal(y4, y1)


@pytest.mark.parametrize("name", ["hardnet", "wang2"])
def test_large_batch_properties(name, cuda_device):
    """Full-size path (65,536 patches): unit norm, finite, and a 512-row sample equals the
    oracle on the same rows."""
    from hardnetnas_amd import synth
    m, fx, p = build_module(name)
    m = m.to(cuda_device)
    b = 65536
    x = torch.from_numpy(synth.synth_patches(b, seed=3)).to(cuda_device)
    with torch.no_grad():
        y = m(x)
    assert torch.isfinite(y).all()
    nrm = y.norm(dim=1)
    assert (nrm - 1).abs().max().item() < 1e-5
    idx = torch.randint(0, b, (512,), generator=torch.Generator().manual_seed(0))
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    xs = x[idx.to(cuda_device)].cpu()
    if name == "hardnet":
        ref = O.hardnet_forward(t, xs)
    else:
        ref = O.nas_forward(t, load("nas_" + name)["meta"]["ops"], xs)
    assert (y[idx.to(cuda_device)].cpu() - ref).abs().max().item() <= _tol(name)


def _oracle_rows(name, p, xs):
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    if name == "hardnet":
        return O.hardnet_forward(t, xs)
    if name.startswith("fdl_"):
        return O.fdl_forward(t, load(name)["meta"]["variant"], xs)
    return O.nas_forward(t, load("nas_" + name)["meta"]["ops"], xs)


@pytest.mark.parametrize("name", ["wang2", "wang3", "wang4", "fdl_NASNet", "fdl_NASNet_01"])
def test_persistent_kernels_past_one_round(name, cuda_device):
    """65,537 patches: every persistent NAS / FDL kernel (grid = min(tiles, resident)) runs
    several rounds per workgroup and ends on a ragged tile; a strided 256-row sample (incl.
    the last row) equals the oracle and every row has unit norm."""
    from hardnetnas_amd import synth
    m, fx, p = build_module(name)
    m = m.to(cuda_device)
    b = 65537
    x = torch.from_numpy(synth.synth_patches(b, seed=21)).to(cuda_device)
    with torch.no_grad():
        y = m(x)
    assert (y.norm(dim=1) - 1).abs().max().item() < 1e-5
    idx = torch.cat([torch.arange(0, b, b // 255)[:255], torch.tensor([b - 1])])
    ref = _oracle_rows(name, p, x[idx.to(cuda_device)].cpu())
    assert (y[idx.to(cuda_device)].cpu() - ref).abs().max().item() <= _tol(name)


@pytest.mark.parametrize("name", ["wang2", "wang3", "wang4"])
def test_nas_at_the_timed_size(name, cuda_device):
    """BASELINE config 3's exact launch (262,144 patches: four 65,536-patch chunks, the bench's grids)
    for each searched net: a strided 1,024-row sample (away from the chunk starts, plus the last row)
    equals the oracle to 2e-5 and every row has unit norm."""
    from hardnetnas_amd import synth
    m, fx, p = build_module(name)
    m = m.to(cuda_device)
    b = 262144
    x = torch.from_numpy(synth.synth_patches(b, seed=1003)).to(cuda_device)
    with torch.no_grad():
        y = m(x)
    assert torch.isfinite(y).all()
    assert (y.norm(dim=1) - 1).abs().max().item() < 1e-5
    idx = torch.cat([torch.arange(0, b, b // 1023)[:1023] + 127, torch.tensor([b - 1])])
    ref = _oracle_rows(name, p, x[idx.to(cuda_device)].cpu())
    assert (y[idx.to(cuda_device)].cpu() - ref).abs().max().item() <= _tol(name)


@pytest.mark.parametrize("u8", [False, True])
def test_c12_group_and_subchunk_sizes_are_bitwise_neutral(u8, cuda_device, monkeypatch):
    """k_c12 over groups (HN_C12_GROUP) and conv3..conv5 over sub-chunks of them (HN_SUBCHUNK): odd
    group / sub-chunk sizes that leave ragged tails give the same descriptors, bit for bit, as one
    launch per chunk (every patch's arithmetic is the same; only the launch boundaries move)."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    b = 2 * 16384 + 77
    g = torch.Generator().manual_seed(7)
    if u8:
        x = torch.randint(0, 256, (b, 32, 32), generator=g, dtype=torch.uint8).to(cuda_device)
    else:
        x = torch.from_numpy(golden_inputs(fx)).repeat(b // 129 + 1, 1, 1, 1)[:b].to(cuda_device)
        x = x + 0.01 * torch.randn(x.shape, generator=g).to(cuda_device)
    out = {}
    for tag, grp, sub in (("one", 65536, 65536), ("odd", 20000, 7000)):
        monkeypatch.setenv("HN_C12_GROUP", str(grp))
        monkeypatch.setenv("HN_SUBCHUNK", str(sub))
        nm = NativeModel.from_module(m, cuda_device)
        out[tag] = nm.forward_u8(x, resize="none") if u8 else nm(x)
    assert torch.equal(out["one"], out["odd"])


def test_hardnet_at_the_timed_size(cuda_device):
    """BASELINE config 2's exact launch (262,144 patches, the bench's chunking and grids): a
    strided 1,024-row sample equals the oracle to 1e-4 and every row has unit norm."""
    from hardnetnas_amd import synth
    m, fx, p = build_module("hardnet")
    m = m.to(cuda_device)
    b = 262144
    x = torch.from_numpy(synth.synth_patches(b, seed=1000)).to(cuda_device)
    with torch.no_grad():
        y = m(x)
    assert torch.isfinite(y).all()
    assert (y.norm(dim=1) - 1).abs().max().item() < 1e-5
    idx = torch.arange(0, b, b // 1024) + 255  # offset: rows away from chunk starts too
    ref = _oracle_rows("hardnet", p, x[idx.to(cuda_device)].cpu())
    err = (y[idx.to(cuda_device)].cpu() - ref).abs().max().item()
    assert err <= TOL["hardnet"]
    # the precision margin: bf16x3 products with conv1, conv3 and conv5 in 1-D Winograd
    # form measure 1.9e-5 here (tests/precision/wino1d_precision.py predicts 1.7-2.0e-5); a further transformed
    # or narrower layer that eats more than half of the 1e-4 bar fails this guard before it can fail the bar
    assert err <= 5e-5, err


def test_weights_update_triggers_repack(cuda_device):
    m, fx, _ = build_module("hardnet")
    m = m.to(cuda_device)
    x = torch.from_numpy(golden_inputs(fx)[:16]).to(cuda_device)
    with torch.no_grad():
        y1 = m(x)
        m.features[3].weight.mul_(2.0)
        y2 = m(x)
        m.features[3].weight.mul_(0.5)
        y3 = m(x)
    assert not torch.allclose(y1, y2)
    assert torch.equal(y1, y3)


def test_train_mode_uses_autograd_path(cuda_device):
    m, fx, _ = build_module("hardnet")
    m = m.to(cuda_device).train()
    x = torch.from_numpy(golden_inputs(fx)[:32]).to(cuda_device)
    y = m(x)
    y.sum().backward()
    assert m.features[0].weight.grad is not None


@pytest.mark.parametrize("b", [2, 64, 300, 4097])
@pytest.mark.parametrize("swap", [False, True])
def test_pairdist_hardneg_matches_oracle(b, swap, cuda_device):
    from hardnetnas_amd._native import pairdist_hardneg
    fx = load("losses")
    if b in (64, 300):
        a, p = torch.from_numpy(fx[f"a{b}"]), torch.from_numpy(fx[f"p{b}"])
    else:
        g = torch.Generator().manual_seed(b)
        a = torch.nn.functional.normalize(torch.randn(b, 128, generator=g), dim=1)
        p = torch.nn.functional.normalize(a + 0.3 * torch.randn(b, 128, generator=g), dim=1)
    pos, mn = pairdist_hardneg(a.to(cuda_device), p.to(cuda_device), swap)
    rpos, rmn = O.hardest_negative(a.double(), p.double(), swap)
    assert (pos.cpu().double() - rpos).abs().max().item() < 1e-4
    assert (mn.cpu().double() - rmn).abs().max().item() < 1e-4


def test_fpr95_matches_reference_vectors(cuda_device):
    """Device FPR95 vs ErrorRateAt95Recall (reference-generated values, tests/golden/losses.npz)
    using descriptors whose pair distances equal the fixture distances."""
    from hardnetnas_amd._native import fpr95
    fx = load("losses")
    for lab_k, dist_k, want_k in (("fpr_kat_labels", "fpr_kat_dists", "fpr_kat"),
                                  ("fpr_labels", "fpr_dists", "fpr")):
        labels = torch.from_numpy(fx[lab_k].astype(np.int32))
        d = torch.from_numpy(fx[dist_k].astype(np.float32))
        a = torch.zeros(len(d), 128)
        p = torch.zeros(len(d), 128)
        p[:, 0] = d                       # |a - p| = d exactly
        got, dd = fpr95(a.to(cuda_device), p.to(cuda_device), labels.to(cuda_device))
        assert torch.allclose(dd.cpu(), d, rtol=1e-6, atol=0)
        # fp32 keys vs the reference's float64: an adjacent swap could move one sample
        assert got == pytest.approx(float(fx[want_k]), abs=2.0 / len(d))


def test_fpr95_on_descriptors_matches_oracle(cuda_device):
    from hardnetnas_amd._native import fpr95
    g = torch.Generator().manual_seed(7)
    n = 20000
    a = torch.nn.functional.normalize(torch.randn(n, 128, generator=g), dim=1)
    lab = (torch.rand(n, generator=g) > 0.5).int()
    noise = torch.where(lab[:, None] == 1, 0.4, 1.5) * torch.randn(n, 128, generator=g)
    p = torch.nn.functional.normalize(a + noise, dim=1)
    got, dd = fpr95(a.to(cuda_device), p.to(cuda_device), lab.to(cuda_device))
    d_ref = torch.sqrt(torch.sum((a - p) ** 2, 1)).numpy()
    ref = O.error_rate_at_95_recall(lab.numpy(), 1.0 / (d_ref + 1e-8))
    assert np.abs(dd.cpu().numpy() - d_ref).max() < 1e-6
    assert got == pytest.approx(ref, abs=2.0 / n)   # tie order may move one sample


@pytest.mark.parametrize("name", ["wang2", "wang3", "wang4", "cov_a"])
def test_nas_unfused_front_matches(name, cuda_device, monkeypatch):
    """HN_NO_FRONT=1 keeps the layer-by-layer stem + layer-0 kernels reachable and exact."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    monkeypatch.setenv("HN_NO_FRONT", "1")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x).cpu().numpy()
    assert "front" not in nm.stage_times()
    assert np.abs(y - fx["y"]).max() <= NAS_TOL


def _synth_nas(ops, seed=99):
    from hardnetnas_amd import synth
    from hardnetnas_amd.model import HardNetNAS
    m = HardNetNAS(list(ops))
    sd = m.state_dict()
    w = synth.synth_state_dict({k: tuple(v.shape) for k, v in sd.items()}, seed)
    for k in w:
        sd[k] = torch.from_numpy(w[k])
    m.load_state_dict(sd)
    return m.eval(), {k: torch.from_numpy(v) for k, v in w.items()}


@pytest.mark.parametrize("op", ["skip", "ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3",
                                "ir_k5_s4", "ir_k3_e1_se", "ir_k3_e3_se", "ir_k3_s4_se",
                                "ir_k5_e1_se", "ir_k5_e3_se", "ir_k5_s4_se", "ir_k3_s2",
                                "ir_k5_s2", "ir_k3_s2_se", "ir_k5_s2_se"])
def test_every_candidate_op_at_layer0_fused_front(op, cuda_device):
    """Each of the 17 CANDIDATE_BLOCKS as layer 0 (the fused stem+layer-0 kernel) against the
    fp32 oracle on synthetic weights; ragged batch exercises the last workgroup."""
    from hardnetnas_amd import synth
    from hardnetnas_amd._native import NativeModel
    ops = [op, "ir_k3_e1", "skip", "ir_k5_s2", "skip", "ir_k3_e1"]
    m, p = _synth_nas(ops)
    x = torch.from_numpy(synth.synth_patches(77, seed=5))
    ref = O.nas_forward(p, ops, x).numpy()
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x.to(cuda_device)).cpu().numpy()
    assert "front" in nm.stage_times()
    assert np.abs(y - ref).max() <= NAS_TOL


ALL_OPS = ["skip", "ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3", "ir_k5_s4",
           "ir_k3_e1_se", "ir_k3_e3_se", "ir_k3_s4_se", "ir_k5_e1_se", "ir_k5_e3_se",
           "ir_k5_s4_se", "ir_k3_s2", "ir_k5_s2", "ir_k3_s2_se", "ir_k5_s2_se"]


@pytest.mark.parametrize("op", ALL_OPS[1:])
@pytest.mark.parametrize("pairs", [True, False])
def test_every_candidate_op_at_every_layer_fused_irf(op, pairs, cuda_device, monkeypatch):
    """The op at all six slots: layer 0 through the fused front, layers 1..5 through the
    fused IRF block kernel (every SEARCH_SPACE2 shape incl. 16/8/4 px and e3/e4 MID) -- with the
    two-block kernel k_irf2 for layers 1+2 and 3+4 where the op qualifies, and without
    (HN_NO_IRF2=1); ragged batch 37 exercises partial tiles (NPB = 1/4/8 patches per workgroup)."""
    from hardnetnas_amd import synth
    from hardnetnas_amd._native import NativeModel
    if not pairs:
        monkeypatch.setenv("HN_NO_IRF2", "1")
    ops = [op] * 6
    m, p = _synth_nas(ops, seed=7)
    x = torch.from_numpy(synth.synth_patches(37, seed=9))
    ref = O.nas_forward(p, ops, x).numpy()
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x.to(cuda_device)).cpu().numpy()
    st = nm.stage_times()
    n1, n2 = st.get("irf", (0, 0))[1], st.get("irf2", (0, 0))[1]
    assert n1 + 2 * n2 == 5 and "pw" not in st
    spec = A.OP_SPECS[op]
    fusable = pairs and not spec.se and A.ir_mid(32, spec.expansion) == 32 and A.ir_mid(64, spec.expansion) == 64
    assert n2 == (2 if fusable else 0), (op, st)
    assert np.abs(y - ref).max() <= NAS_TOL


@pytest.mark.parametrize("name", ["hardnet", "wang2", "fdl_NASNet"])
def test_head_forms_are_bit_identical(name, cuda_device, monkeypatch):
    """k_head3 (LDS-DMA ring, 128-patch workgroups) accumulates the K-chunks in the same order as
    k_head2 (HN_HEAD=2): bit-identical descriptors for the HardNet (bf16x3, K = 8192) and the NAS /
    FDL (fp16x3, K = 2048) heads, at a ragged batch whose last workgroup is partial."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    xr = torch.from_numpy(np.concatenate([golden_inputs(fx)] * 40)[:301]).to(cuda_device)
    monkeypatch.setenv("HN_HEAD", "3")  # k_head3 unsplit (the default splits K at these batch sizes)
    nm = NativeModel.from_module(m, cuda_device)
    y, yr = nm(x), nm(xr)
    for form in ("2", "1"):  # k_head2; k_head (no LDS staging)
        monkeypatch.setenv("HN_HEAD", form)
        nm2 = NativeModel.from_module(m, cuda_device)
        assert torch.equal(y, nm2(x)), form
        assert torch.equal(yr, nm2(xr)), form
    assert np.abs(y.cpu().numpy() - fx["y"]).max() <= _tol(name)


@pytest.mark.parametrize("name", ["hardnet", "wang2"])
def test_split_k_head_for_small_batches(name, cuda_device, monkeypatch):
    """Batches of up to 16,384 patches run the head as split-K k_head3 (64 / 16 K ranges, one workgroup per
    128 patches x range) + k_head_fin (the partials summed in range order, bias, L2): against the reference
    vectors; within 2e-6 of the unsplit k_head3 (a reassociated K sum); bit for bit the same descriptors for a
    patch whatever batch of <= 16,384 it comes in (the reference eval loop's 512, a ragged 37, the largest
    split batch); and the first unsplit batch size (16,385) stays within 2e-6 of it."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    g = golden_inputs(fx)
    xb = torch.from_numpy(np.concatenate([g] * (16_385 // len(g) + 1))[:16_385]).to(cuda_device)
    xb = xb + 0.01 * torch.randn(xb.shape, generator=torch.Generator().manual_seed(3)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y512, y37, y16k = nm(xb[:512]), nm(xb[:37]), nm(xb[:16_384])
    launches = nm.stage_times()["head"][1]
    assert launches == 3, launches  # three split-K heads (stage records count the calls)
    assert torch.equal(y37, y512[:37]) and torch.equal(y512, y16k[:512])
    assert torch.equal(nm(xb[100:612]), y16k[100:612])
    y_unsplit = nm(xb)  # 16,385: k_head3
    assert (y_unsplit[:16_384] - y16k).abs().max().item() <= 2e-6
    monkeypatch.setenv("HN_HEAD", "3")
    n3 = NativeModel.from_module(m, cuda_device)
    assert (n3(xb[:512]) - y512).abs().max().item() <= 2e-6
    x = torch.from_numpy(g).to(cuda_device)
    assert np.abs(nm(x).cpu().numpy() - fx["y"]).max() <= _tol(name)


@pytest.mark.parametrize("name", ["hardnet", "wang2"])
def test_head4_is_bit_identical(name, cuda_device, monkeypatch):
    """k_head4 (HN_HEAD=4: 256-patch workgroups, every wave all 128 columns, chunks of 65,536) keeps
    k_head3's K-chunk order and L2 summation order: bit-identical descriptors at a ragged batch above
    its 61,440-patch launch threshold (partial last workgroup), and at a small one (k_head3 runs)."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    g = golden_inputs(fx)
    xb = torch.from_numpy(np.concatenate([g] * (61_517 // len(g) + 1))[:61_517]).to(cuda_device)
    xs = torch.from_numpy(g[:37]).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    yb, ys = nm(xb), nm(xs)
    monkeypatch.setenv("HN_HEAD", "4")
    nm4 = NativeModel.from_module(m, cuda_device)
    nm4.set_profiling(True)
    assert torch.equal(yb, nm4(xb))
    assert torch.equal(ys, nm4(xs))
    assert np.abs(yb[: len(g)].cpu().numpy() - fx["y"]).max() <= _tol(name)
    if name == "hardnet":  # the prefetching head form (HN_HEAD_PF, default on) against the plain k_head4
        monkeypatch.setenv("HN_HEAD_PF", "0")
        assert torch.equal(yb, NativeModel.from_module(m, cuda_device)(xb))


@pytest.mark.parametrize("name", ["wang2", "wang4"])
def test_two_block_kernel_is_bit_identical(name, cuda_device, monkeypatch):
    """k_irf2 (layers 1+2 / 3+4 in one kernel, the activation between them in LDS) computes exactly
    what the two k_irf launches do (the same fp32 values are split and multiplied): bit-identical
    descriptors, on the golden patches and a ragged batch."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x)
    assert "irf2" in nm.stage_times()
    monkeypatch.setenv("HN_NO_IRF2", "1")
    nm1 = NativeModel.from_module(m, cuda_device)
    assert torch.equal(y, nm1(x))
    assert torch.equal(nm(x[:37]), nm1(x[:37]))
    assert np.abs(y.cpu().numpy() - fx["y"]).max() <= NAS_TOL


@pytest.mark.parametrize("name", ["wang2", "wang4"])
def test_nas_unfused_irf_matches(name, cuda_device, monkeypatch):
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    monkeypatch.setenv("HN_NO_IRF", "1")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x).cpu().numpy()
    assert "irf" not in nm.stage_times()
    assert np.abs(y - fx["y"]).max() <= NAS_TOL


@pytest.mark.parametrize("name", FDL_NAMES)
def test_fdl_runs_front_irf_head_and_matches_layerwise(name, cuda_device, monkeypatch):
    """The FDL descriptor runs its fused front, the fused IRF blocks and the MFMA head; the
    layer-by-layer pw/dw/pwl kernels (HN_NO_IRF=1) agree; a 3 000-patch run matches the
    oracle on a sample."""
    from hardnetnas_amd._native import NativeModel
    m, fx, p = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x).cpu().numpy()
    assert set(nm.stage_times()) == {"front", "irf", "head"}
    assert np.abs(y - fx["y"]).max() <= NAS_TOL
    monkeypatch.setenv("HN_NO_IRF", "1")
    lw = NativeModel.from_module(m, cuda_device)
    assert np.abs(lw(x).cpu().numpy() - y).max() <= NAS_TOL
    from hardnetnas_amd import synth
    xb = torch.from_numpy(synth.synth_patches(3000, 11))
    yb = nm(xb.to(cuda_device)).cpu()
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    ref = O.fdl_forward(t, fx["meta"]["variant"], xb[-200:])
    assert float((yb[-200:] - ref).abs().max()) <= NAS_TOL



@pytest.mark.parametrize("name,model", [("hardnet", "hardnet"), ("fdl_NASNet", "fdl_nasnet"),
                                        ("wang2", "nas:1,4,14,13,4,0")])
def test_c_abi_demo_program(name, model, tmp_path):
    """hardnetnas_amd/lib/hn_cabi_demo (built by `make`): the forward driven through the C ABI
    alone (hn_param_count / hn_create / hn_workspace_bytes / hn_forward + hipMalloc), in a
    child process with no Python or torch -- the boundary a non-Python host would bind."""
    import subprocess
    from hardnetnas_amd import _native as N
    exe = os.path.join(os.path.dirname(N.lib_path()), "hn_cabi_demo")
    assert os.path.exists(exe), "build the library first (make -C hardnetnas_amd/csrc)"
    m, fx, _ = build_module(name)
    x = golden_inputs(fx)[:100]
    N.state_dict_blob(m.state_dict()).tofile(tmp_path / "p.f32")
    np.ascontiguousarray(x, dtype=np.float32).tofile(tmp_path / "x.f32")
    r = subprocess.run([exe, model, str(tmp_path / "p.f32"), str(tmp_path / "x.f32"), "100",
                        str(tmp_path / "y.f32")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    y = np.fromfile(tmp_path / "y.f32", dtype=np.float32).reshape(100, 128)
    assert np.abs(y - fx["y"][:100]).max() <= _tol(name)


def test_forward_is_graph_capturable(cuda_device):
    """The header's promise: hn_forward neither allocates nor synchronises, so a whole forward
    (several chunks) can be captured once into a HIP graph and replayed on new inputs."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    ref = nm(x).clone()
    static_x = torch.zeros_like(x)
    out = torch.empty((x.shape[0], 128), device=cuda_device)
    ws = torch.empty(nm.workspace_bytes(x.shape[0]), device=cuda_device, dtype=torch.uint8)
    nm.forward(static_x, out=out, workspace=ws)  # warm-up: one-time launch attributes
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=cuda_device)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            nm.forward(static_x, out=out, workspace=ws)
    static_x.copy_(x)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_chunk_pipeline_is_bit_identical(cuda_device, monkeypatch):
    """forward_hardnet_pipe (opt-in, HN_PIPELINE=1): a HardNet batch of several chunks runs chunk k + 1's k_c12s on
    a second stream (into
    the other of two k_c12 output buffers) beside chunk k's conv3 .. head.  The kernels and their inputs are the
    sequential path's, so the descriptors are bit-identical to HN_PIPELINE=0 -- here 6 chunks of 4,096 (the
    buffer alternation and both event waits) with a ragged last one -- the workspace grows by one k_c12 output
    (64 KiB per chunk patch) only for batches of more than one chunk, and the two-stream forward is captured
    into a HIP graph (fork and join through events) and replayed."""
    from hardnetnas_amd import synth
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module("hardnet")
    g = golden_inputs(fx)
    n = 5 * 4096 + 37
    x = torch.from_numpy(np.concatenate([g, synth.synth_patches(n - len(g), seed=41)])).to(cuda_device)
    monkeypatch.setenv("HN_CHUNK", "4096")
    monkeypatch.setenv("HN_PIPELINE", "1")
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x)
    assert nm.stage_times()["stem+conv1+conv2"][1] == 6
    assert np.abs(y[: len(g)].cpu().numpy() - fx["y"]).max() <= _tol("hardnet")
    monkeypatch.setenv("HN_PIPELINE", "0")
    n0 = NativeModel.from_module(m, cuda_device)
    assert torch.equal(y, n0(x))
    assert nm.workspace_bytes(n) == n0.workspace_bytes(n) + 4096 * 16384 * 4
    assert nm.workspace_bytes(4096) == n0.workspace_bytes(4096)
    nm.set_profiling(False)
    static_x = torch.zeros_like(x)
    out = torch.empty((n, 128), device=cuda_device)
    ws = torch.empty(nm.workspace_bytes(n), device=cuda_device, dtype=torch.uint8)
    nm.forward(static_x, out=out, workspace=ws)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=cuda_device)
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            nm.forward(static_x, out=out, workspace=ws)
    static_x.copy_(x)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y)


@pytest.mark.parametrize("name", ["wang3", "cov_c"])
def test_nas_fused_skip_s2_matches_unfused(name, cuda_device, monkeypatch):
    """The channel-changing stride-2 "skip" (MaxPool2d(3, 2, 1) + ConvBNRelu 1x1,
    fbnet_builder.py:202-228) runs as one kernel (stage "skip", fp16x3 MFMA); it matches the
    reference vectors, and the maxpool + fp32 pw kernels (HN_NO_SKIPFUSE=1) on ragged batches."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x).cpu().numpy()
    st = nm.stage_times()
    # (wang3's skip runs inside k_irf_skip with the layer-2 block, stage "irf+skip")
    assert ("skip" in st or "irf+skip" in st) and "maxpool" not in st
    assert np.abs(y - fx["y"]).max() <= NAS_TOL
    monkeypatch.setenv("HN_NO_SKIPFUSE", "1")
    lw = NativeModel.from_module(m, cuda_device)
    lw.set_profiling(True)
    for b in (1, 3, 37, 256):
        assert np.abs(lw(x[:b]).cpu().numpy() - y[:b]).max() <= NAS_TOL
    assert "maxpool" in lw.stage_times() and "skip" not in lw.stage_times()


@pytest.mark.parametrize("op", ["ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3", "ir_k5_s4", "ir_k5_s2",
                                "wang3"])
def test_irf_skip_kernel_is_bit_identical(op, cuda_device, monkeypatch):
    """k_irf_skip: the 16x16 stride-2 block of layer 2 and the 8x8 64 -> 128 stride-2 skip after the
    identity skip of layer 3 (wang3's layers 2-4) in one kernel, the block's output kept in LDS.  It
    repeats k_skip_s2's arithmetic step for step, so its descriptors equal the two-kernel path
    (HN_NO_IRFSKIP=1) bit for bit -- every MID (e1 / e3 / e4 + groups) and kernel size, ragged batches --
    and match the reference restatement (wang3: the golden vectors)."""
    from hardnetnas_amd import synth
    from hardnetnas_amd._native import NativeModel
    if op == "wang3":
        m, fx, _ = build_module("wang3")
        x = torch.from_numpy(golden_inputs(fx))
        ref = fx["y"]
    else:
        ops = ["ir_k3_e1", "skip", op, "skip", "skip", "skip"]
        m, p = _synth_nas(ops, seed=13)
        x = torch.from_numpy(synth.synth_patches(301, seed=17))
        ref = O.nas_forward(p, ops, x).numpy()
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x.to(cuda_device))
    st = nm.stage_times()
    assert "irf+skip" in st and "skip" not in st and "irf" not in st, st
    assert np.abs(y.cpu().numpy() - ref).max() <= NAS_TOL
    monkeypatch.setenv("HN_NO_IRFSKIP", "1")
    n2 = NativeModel.from_module(m, cuda_device)
    n2.set_profiling(True)
    assert torch.equal(y, n2(x.to(cuda_device)))
    assert "irf+skip" not in n2.stage_times() and "skip" in n2.stage_times()
    for b in (1, 37):
        assert torch.equal(nm(x[:b].to(cuda_device)), n2(x[:b].to(cuda_device)))


@pytest.mark.parametrize("op", ["ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3", "ir_k5_s4", "ir_k3_s2",
                                "wang4"])
def test_maxpool_front_irf_kernel_is_bit_identical(op, cuda_device, monkeypatch):
    """k_mpfront_irf: the max-pool front (layer 0 "skip" at stride 2), the identity layer 1 and the 16x16 stride-2
    layer-2 block in one persistent kernel, the 16x16x32 front output kept on chip.  It repeats k_front's stem /
    max-pool and k_irf's block arithmetic step for step, so its descriptors equal the two-kernel path
    (HN_NO_MPFRONT=1) bit for bit -- every MID (e1 / e3 / e4, groups + shuffle) and kernel size, ragged batches,
    several patches per persistent workgroup -- and match the reference restatement (wang4: the golden vectors)."""
    from hardnetnas_amd import synth
    from hardnetnas_amd._native import NativeModel
    if op == "wang4":
        m, fx, _ = build_module("wang4")
        x = torch.from_numpy(golden_inputs(fx))
        ref = fx["y"]
    else:
        ops = ["skip", "skip", op, "ir_k3_e1", "ir_k5_e1", "skip"]
        m, p = _synth_nas(ops, seed=19)
        x = torch.from_numpy(synth.synth_patches(301, seed=23))
        ref = O.nas_forward(p, ops, x).numpy()
    nm = NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    y = nm(x.to(cuda_device))
    st = nm.stage_times()
    assert "front+irf" in st and "front" not in st, st
    assert np.abs(y.cpu().numpy() - ref).max() <= NAS_TOL
    monkeypatch.setenv("HN_NO_MPFRONT", "1")
    n2 = NativeModel.from_module(m, cuda_device)
    n2.set_profiling(True)
    assert torch.equal(y, n2(x.to(cuda_device)))
    assert "front+irf" not in n2.stage_times() and "front" in n2.stage_times()
    for b in (1, 37):
        assert torch.equal(nm(x[:b].to(cuda_device)), n2(x[:b].to(cuda_device)))
    xr = x.repeat(7, 1, 1, 1)[:2001].to(cuda_device)  # more patches than resident workgroups: several each
    assert torch.equal(nm(xr), n2(xr))


@pytest.mark.parametrize("name", ["wang2", "cov_c"])
def test_front_k3_xch_form_is_bit_identical(name, cuda_device, monkeypatch):
    """The k3 MID-32 front in the XCH form (HN_FRONT_XCH3=1: dw per channel group with SGPR weights,
    results crossed to the pwl layout through s_x, 32-float ring pixels with the swizzled chunks) runs
    the same fp32 FMAs in the same order as the default form: bit-identical descriptors (wang2's k3
    front; cov_c's layer 0 is a k5 front, so there the knob changes nothing), ragged batches included."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    nm = NativeModel.from_module(m, cuda_device)
    y = nm(x)
    monkeypatch.setenv("HN_FRONT_XCH3", "1")
    n3 = NativeModel.from_module(m, cuda_device)
    assert torch.equal(y, n3(x))
    for b in (1, 37):
        assert torch.equal(nm(x[:b]), n3(x[:b]))
    assert np.abs(y.cpu().numpy() - fx["y"]).max() <= NAS_TOL


@pytest.mark.parametrize("name", ["wang2", "wang3", "cov_a", "cov_b", "cov_c"])
def test_front_pwl_forms_match_reference(name, cuda_device, monkeypatch):
    """The NAS front's two pwl forms -- the default 16x16x32 one (wave = band row, no partial-sum
    fold; for k3 and the k5 MID-32 front (wang3) with two stem rows per gathered window) and the
    round-2 32x32x16 one with the fold through LDS (HN_FRONT_FOLD=1) -- both against the reference
    vectors (MID 32 / 96 / 128, k3 / k5, with and without groups and SE), and close to each other
    (they differ only in summation orders)."""
    from hardnetnas_amd._native import NativeModel
    m, fx, _ = build_module(name)
    x = torch.from_numpy(golden_inputs(fx)).to(cuda_device)
    y = NativeModel.from_module(m, cuda_device)(x).cpu().numpy()
    monkeypatch.setenv("HN_FRONT_FOLD", "1")
    yf = NativeModel.from_module(m, cuda_device)(x).cpu().numpy()
    assert np.abs(y - fx["y"]).max() <= NAS_TOL
    assert np.abs(yf - fx["y"]).max() <= NAS_TOL
    assert np.abs(y - yf).max() <= 5e-6
