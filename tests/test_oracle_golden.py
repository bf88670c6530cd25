"""Pin the oracle (CPU restatement) and the drop-in modules' PyTorch path against
the vectors produced by the reference code (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from fixtures import FDL_NAMES, NAS_NAMES, build_module, load, params_for, golden_inputs
from oracle import hardnet_oracle as O

TOL = 1e-5   # fp32 vs fp32 of the same ATen ops: only summation-order noise


def _oracle(name, p, x, dtype=torch.float32):
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    if name == "hardnet":
        return O.hardnet_forward(t, torch.from_numpy(x), dtype).numpy()
    if name.startswith("fdl_"):
        return O.fdl_forward(t, load(name)["meta"]["variant"], torch.from_numpy(x), dtype).numpy()
    ops = load("nas_" + name)["meta"]["ops"]
    return O.nas_forward(t, ops, torch.from_numpy(x), dtype).numpy()


@pytest.mark.parametrize("name", ["hardnet"] + NAS_NAMES + FDL_NAMES)
def test_oracle_matches_reference_vectors(name):
    m, fx, p = build_module(name)
    x = golden_inputs(fx)
    y = _oracle(name, p, x)
    assert y.shape == (fx["meta"]["n_test"], 128)
    assert np.abs(y - fx["y"]).max() <= TOL
    assert np.abs(y - fx["y64"]).max() <= 5e-6
    ye = _oracle(name, p, fx["x_edge"])
    assert np.abs(ye - fx["y_edge"]).max() <= TOL


@pytest.mark.parametrize("name", ["hardnet", "wang2", "cov_b"] + FDL_NAMES)
def test_oracle_fp64_matches_reference_fp64(name):
    m, fx, p = build_module(name)
    y = _oracle(name, p, golden_inputs(fx)[:64], torch.float64)
    assert np.abs(y - fx["y64"][:64]).max() <= 1e-12


@pytest.mark.parametrize("name", ["hardnet"] + NAS_NAMES + FDL_NAMES)
def test_module_torch_path_matches_reference(name):
    m, fx, _ = build_module(name)
    with torch.no_grad():
        y = m(torch.from_numpy(golden_inputs(fx))).numpy()
    assert np.abs(y - fx["y"]).max() <= TOL


def test_state_dict_layout_hardnet():
    from hardnetnas_amd.model import HardNet
    keys = list(HardNet().state_dict().keys())
    conv = [k for k in keys if k.endswith(".weight")]
    assert conv == [f"features.{i}.weight" for i in (0, 3, 6, 9, 12, 15, 19)]
    for i in (1, 4, 7, 10, 13, 16, 20):
        assert f"features.{i}.running_mean" in keys and f"features.{i}.running_var" in keys
    assert sum(v.numel() for k, v in HardNet().state_dict().items()
               if k.endswith("weight")) == 1334560


@pytest.mark.parametrize("name", NAS_NAMES)
def test_supernet_key_mapping(name):
    """The reference supernet keys of the sampled ops map onto HardNetNAS keys."""
    from hardnetnas_amd.model import HardNetNAS
    fx = load("nas_" + name)
    ours = HardNetNAS(fx["meta"]["ops"])
    sk = fx["meta"]["supernet_keys"]
    fake = {("module." + k): torch.zeros(1) for k in sk}
    fake.update({"module.stages_to_search.0.thetas": torch.zeros(17)})
    mapped = set()
    for k in fake:
        kk = k[len("module."):]
        if kk.startswith("stages_to_search.") and ".ops." in kk:
            p = kk.split(".")
            mapped.add(".".join(["stages", p[1]] + p[4:]))
    want = {k for k in ours.state_dict() if k.startswith("stages.")}
    assert mapped == want


def test_supernet_state_dict_loads():
    m, fx, p = build_module("wang2")
    from hardnetnas_amd.arch import CANDIDATE_BLOCKS
    from hardnetnas_amd.model import HardNetNAS
    sd = {}
    for k, v in m.state_dict().items():
        if k.startswith("stages."):
            parts = k.split(".")
            j = CANDIDATE_BLOCKS.index(m.arch_ops[int(parts[1])])
            sd["module." + ".".join(["stages_to_search", parts[1], "ops", str(j)] + parts[2:])] = v
        else:
            sd["module." + k] = v
    sd["module.stages_to_search.0.ops.0.junk"] = torch.zeros(3)   # other op: dropped
    sd["module.stages_to_search.0.thetas"] = torch.zeros(17)
    m2 = HardNetNAS("wang2").eval()
    m2.load_supernet_state_dict(sd)
    x = torch.from_numpy(golden_inputs(fx)[:8])
    with torch.no_grad():
        assert torch.equal(m(x), m2(x))


def test_distance_and_loss_match_reference():
    fx = load("losses")
    for b in (64, 300):
        a, p = torch.from_numpy(fx[f"a{b}"]), torch.from_numpy(fx[f"p{b}"])
        dm = O.distance_matrix_vector(a, p).numpy()
        assert np.abs(dm - fx[f"dm{b}"]).max() <= 2e-6
        for swap in (0, 1):
            for lt in ("triplet_margin", "softmax", "contrastive"):
                v = O.loss_hardnet(a, p, anchor_swap=bool(swap), loss_type=lt).item()
                assert abs(v - float(fx[f"loss{b}_{swap}_{lt}"])) <= 2e-6


def test_fpr95_known_answers():
    fx = load("losses")
    got = O.error_rate_at_95_recall(fx["fpr_kat_labels"], 1.0 / (fx["fpr_kat_dists"] + 1e-8))
    assert got == pytest.approx(1.0 / 3.0) and got == float(fx["fpr_kat"])
    got = O.error_rate_at_95_recall(fx["fpr_labels"], 1.0 / (fx["fpr_dists"] + 1e-8))
    assert got == float(fx["fpr"])


@pytest.mark.parametrize("name", FDL_NAMES)
def test_fdl_edge_outputs_finite(name):
    """Zero / constant patches (std == 0) stay finite through input_norm's eps and the
    eps-free torch.norm (the head's output is never the zero vector)."""
    fx = load(name)
    assert np.isfinite(fx["y_edge"]).all() and np.isfinite(fx["y"]).all()


def test_state_dict_layout_fdl():
    """Index layout of HardNetNeiMask.features (latency/NASNet/model/des.py:13-36,
    latency/NASNet_0.1/model/des.py:17-29)."""
    from hardnetnas_amd.model import HardNetNeiMask
    k1 = list(HardNetNeiMask(variant="NASNet").state_dict().keys())
    assert k1[:4] == ["features.0.weight", "features.0.bias", "features.1.running_mean",
                      "features.1.running_var"]
    assert "features.8.pw.conv.weight" in k1 and "features.11.weight" in k1
    assert "features.12.running_var" in k1 and "features.11.bias" not in k1
    k2 = list(HardNetNeiMask(variant="NASNet_0.1").state_dict().keys())
    assert k2[2] == "features.3.conv.conv.weight" and "features.7.weight" in k2
    assert "features.10.pwl.bn.running_var" not in k2 and "features.6.pwl.bn.running_var" in k2
