"""Generate the golden fixtures from the REFERENCE code (survey container only).

Run from the repo root:  python tests/golden/make_golden.py
Needs /root/reference (read-only, never copied): the reference's own module code is
executed to produce the expected outputs; only data (inputs seeds, BN statistics,
outputs, checksums) is written into tests/golden/*.npz.

* HardNet: ``class HardNet`` + ``def weights_init`` are AST-extracted from
  hardnet/HardNet.py:275-324 and ``class L2Norm`` from hardnet/Utils.py:15-22 (the
  modules themselves import cv2/torchvision and run argparse at import time, which
  this image cannot do -- SURVEY.md 8(c)).
* hardnetNAS: ``FBNet_Stochastic_SuperNet`` (model_supernet.py) and ``PRIMITIVES``
  (fbnet_builder.py) are imported directly; the sampled net is the supernet with
  each MixedOperation replaced by ``ops[CANDIDATE_BLOCKS.index(op)]``.
* FDLNet ``HardNetNeiMask`` (latency/NASNet{,_0.1}/model/des.py) is imported directly with
  the variant's directory as the package root.
* losses/metrics: ``distance_matrix_vector`` / ``loss_HardNet`` (hardnet/Losses.py)
  and ``ErrorRateAt95Recall`` (hardnet/EvalMetrics.py) are AST-extracted.  The
  reference loss calls ``.cuda()`` on an eye matrix; for CPU fixture generation
  ``torch.Tensor.cuda`` is made the identity inside this process only.

Weights come from hardnetnas_amd.synth (splitmix64, seed 1234); BN running stats are
calibrated by a train-mode pass of the reference module (momentum=None, dropout
off) over 2048 synthetic patches, and committed.
"""
from __future__ import annotations

import ast
import json
import os
import sys
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("HN_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from hardnetnas_amd import arch as A          # noqa: E402
from hardnetnas_amd import synth               # noqa: E402
from hardnetnas_amd.model import HardNetNAS    # noqa: E402

WEIGHT_SEED = 1234
CALIB_SEED = 7
TEST_SEED = 0
N_TEST = 256
N_CALIB = 2048


def _extract(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in names]
    assert {n.name for n in keep} == set(names), (path, names)
    return ast.unparse(ast.Module(body=keep, type_ignores=[]))


def _ns():
    return {"torch": torch, "nn": nn, "F": F, "np": np, "sys": sys,
            "Variable": torch.autograd.Variable}


def edge_patches():
    """Edge cases: zero / exactly-representable constant (std == 0),
    low-variance, large-offset, saturated uint8 extremes, single hot pixel."""
    rng_u = synth.uniform(99, 6 * 1024).reshape(6, 1024)
    e = []
    e.append(np.zeros(1024))
    e.append(np.full(1024, 0.25))
    e.append(0.5 + 0.02 * (rng_u[0] - 0.5))
    e.append(1000.0 + 50.0 * rng_u[1])
    e.append(np.where(rng_u[2] > 0.5, (1.0 - synth.MEAN_IMAGE) / synth.STD_IMAGE,
                      (0.0 - synth.MEAN_IMAGE) / synth.STD_IMAGE))
    hot = np.zeros(1024)
    hot[17 * 32 + 5] = 3.0
    e.append(hot)
    return np.stack(e).astype(np.float32).reshape(-1, 1, 32, 32)


def _calibrate(modules, forward, x):
    """Train-mode BN pass with cumulative averaging (momentum=None)."""
    for m in modules.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.reset_running_stats()
            m.momentum = None
        m.train(True)
        if isinstance(m, nn.Dropout):
            m.train(False)
    with torch.no_grad():
        for chunk in torch.split(x, 512):
            forward(chunk)
    modules.eval()


def make_hardnet():
    ns = _ns()
    exec(_extract(os.path.join(REF, "hardnet/Utils.py"), ["L2Norm"]), ns)
    exec(_extract(os.path.join(REF, "hardnet/HardNet.py"), ["HardNet", "weights_init"]), ns)
    torch.manual_seed(0)
    model = ns["HardNet"]()
    sd = model.state_dict()
    tmpl = {k: tuple(v.shape) for k, v in sd.items()}
    w = synth.synth_state_dict(tmpl, WEIGHT_SEED)
    sd.update({k: torch.from_numpy(v) for k, v in w.items()})
    model.load_state_dict(sd)
    xc = torch.from_numpy(synth.synth_patches(N_CALIB, CALIB_SEED))
    _calibrate(model, model, xc)
    x = torch.from_numpy(synth.synth_patches(N_TEST, TEST_SEED))
    xe = torch.from_numpy(edge_patches())
    with torch.no_grad():
        y = model(x).numpy()
        ye = model(xe).numpy()
        m64 = model.double()
        y64 = m64(x.double()).numpy()
        ye64 = m64(xe.double()).numpy()
    sd = {k: v.float().numpy() for k, v in model.state_dict().items()
          if not k.endswith("num_batches_tracked")}
    conv_keys = [k for k in sd if k.endswith(".weight")]
    out = {
        "meta": json.dumps({"model": "hardnet", "weight_seed": WEIGHT_SEED,
                            "test_seed": TEST_SEED, "n_test": N_TEST,
                            "weights_sha256": {k: synth.sha256_f32(sd[k]) for k in conv_keys},
                            "x_sha256": synth.sha256_f32(x.numpy()),
                            "source": "hardnet/HardNet.py:275-324 + hardnet/Utils.py:15-22 "
                                      "(AST-extracted, executed with torch %s CPU)" % torch.__version__}),
        "x_edge": xe.numpy(), "y": y, "y_edge": ye, "y64": y64, "y_edge64": ye64,
    }
    for k, v in sd.items():
        if "running" in k:
            out["bn/" + k] = v
    np.savez_compressed(os.path.join(HERE, "hardnet.npz"), **out)
    print("hardnet", y.shape, float(np.abs(y - y64).max()))


class _StubLUT:
    def __init__(self):
        self.cnt_layers = len(A.SEARCH_SPACE2)
        self.layers_parameters = [(ci, co, -999, s) for ci, co, s in A.SEARCH_SPACE2]
        ns = {}
        self.lookup_table_operations = None
        self.lookup_table_latency = [{op: 1.0 for op in A.CANDIDATE_BLOCKS}
                                     for _ in range(self.cnt_layers)]


def make_nas(name, ops):
    sys.path.insert(0, os.path.join(REF, "hardnetNAS"))
    from fbnet_building_blocks.fbnet_builder import PRIMITIVES
    from supernet_functions.model_supernet import FBNet_Stochastic_SuperNet
    lut = _StubLUT()
    lut.lookup_table_operations = {op: PRIMITIVES[op] for op in A.CANDIDATE_BLOCKS}
    torch.manual_seed(0)
    supernet = FBNet_Stochastic_SuperNet(lut)
    idx = [A.CANDIDATE_BLOCKS.index(op) for op in ops]

    # synthesize weights keyed by OUR module's names, load into the supernet's slots
    ours = HardNetNAS(ops)
    tmpl = {k: tuple(v.shape) for k, v in ours.state_dict().items()}
    w = synth.synth_state_dict(tmpl, WEIGHT_SEED)

    def to_super(k):
        if k.startswith("stages."):
            p = k.split(".")
            i = int(p[1])
            return ".".join(["stages_to_search", str(i), "ops", str(idx[i])] + p[2:])
        return k

    ssd = supernet.state_dict()
    for k, v in w.items():
        sk = to_super(k)
        assert sk in ssd and tuple(ssd[sk].shape) == v.shape, (k, sk)
        ssd[sk] = torch.from_numpy(v)
    supernet.load_state_dict(ssd)

    sampled = nn.ModuleList([supernet.first] +
                            [supernet.stages_to_search[i].ops[j] for i, j in enumerate(idx)] +
                            [supernet.last_stages])

    def fwd(x):  # model_supernet.py:70-85 with argmax ops
        y = supernet.first(x)
        for i, j in enumerate(idx):
            y = supernet.stages_to_search[i].ops[j](y)
        y = supernet.last_stages(y)
        return y / torch.norm(y, p=2, dim=-1, keepdim=True)

    xc = torch.from_numpy(synth.synth_patches(N_CALIB, CALIB_SEED))
    _calibrate(sampled, fwd, xc)
    x = torch.from_numpy(synth.synth_patches(N_TEST, TEST_SEED))
    xe = torch.from_numpy(edge_patches()[[2, 3, 4, 5]])  # no input_norm: keep finite-norm cases
    with torch.no_grad():
        y = fwd(x).numpy()
        ye = fwd(xe).numpy()
        sampled.double()
        y64 = fwd(x.double()).numpy()
        ye64 = fwd(xe.double()).numpy()
        sampled.float()
    ssd = supernet.state_dict()
    bn = {}
    for k in tmpl:
        if "running" in k:
            bn["bn/" + k] = ssd[to_super(k)].float().numpy()
    super_keys = sorted(k for k in ssd if any(k.startswith(f"stages_to_search.{i}.ops.{j}.")
                                              for i, j in enumerate(idx)))
    out = {
        "meta": json.dumps({"model": "nas", "name": name, "ops": ops, "weight_seed": WEIGHT_SEED,
                            "test_seed": TEST_SEED, "n_test": N_TEST,
                            "weights_sha256": {k: synth.sha256_f32(v) for k, v in w.items()
                                               if "running" not in k},
                            "supernet_keys": super_keys,
                            "source": "hardnetNAS FBNet_Stochastic_SuperNet + PRIMITIVES "
                                      "(imported, torch %s CPU)" % torch.__version__}),
        "x_edge": xe.numpy(), "y": y, "y_edge": ye, "y64": y64, "y_edge64": ye64, **bn,
    }
    np.savez_compressed(os.path.join(HERE, f"nas_{name}.npz"), **out)
    print("nas", name, y.shape, float(np.abs(y - y64).max()))


def make_fdl(variant):
    """FDLNet HardNetNeiMask (latency/<variant>/model/des.py), imported from the reference with
    its own package root on sys.path (both variants use the package names model/ and utils/)."""
    from hardnetnas_amd.model import HardNetNeiMask
    for k in [k for k in sys.modules if k.split(".")[0] in ("model", "utils")]:
        del sys.modules[k]
    sys.path.insert(0, os.path.join(REF, "FDLNet-master", "latency", variant))
    try:
        from model.des import HardNetNeiMask as RefNet
    finally:
        sys.path.pop(0)
    torch.manual_seed(0)
    model = RefNet(1.0, 1.0)
    sd = model.state_dict()
    tmpl = {k: tuple(v.shape) for k, v in HardNetNeiMask(variant=variant).state_dict().items()}
    assert tmpl == {k: tuple(v.shape) for k, v in sd.items()}, "state_dict layout differs"
    w = synth.synth_state_dict(tmpl, WEIGHT_SEED)
    sd.update({k: torch.from_numpy(v) for k, v in w.items()})
    model.load_state_dict(sd)
    xc = torch.from_numpy(synth.synth_patches(N_CALIB, CALIB_SEED))
    _calibrate(model, model, xc)
    x = torch.from_numpy(synth.synth_patches(N_TEST, TEST_SEED))
    xe = torch.from_numpy(edge_patches())
    with torch.no_grad():
        y = model(x).numpy()
        ye = model(xe).numpy()
        m64 = model.double()
        y64 = m64(x.double()).numpy()
        ye64 = m64(xe.double()).numpy()
    sd = {k: v.float().numpy() for k, v in model.state_dict().items()
          if not k.endswith("num_batches_tracked")}
    out = {
        "meta": json.dumps({"model": "fdl", "variant": variant, "weight_seed": WEIGHT_SEED,
                            "test_seed": TEST_SEED, "n_test": N_TEST,
                            "weights_sha256": {k: synth.sha256_f32(v) for k, v in w.items()
                                               if "running" not in k},
                            "source": "FDLNet-master/latency/%s/model/des.py HardNetNeiMask "
                                      "(imported, torch %s CPU)" % (variant, torch.__version__)}),
        "x_edge": xe.numpy(), "y": y, "y_edge": ye, "y64": y64, "y_edge64": ye64,
    }
    for k, v in sd.items():
        if "running" in k:
            out["bn/" + k] = v
    tag = variant.replace(".", "")
    np.savez_compressed(os.path.join(HERE, f"fdl_{tag}.npz"), **out)
    print("fdl", variant, y.shape, float(np.abs(y - y64).max()))


def make_losses():
    ns = _ns()
    exec(_extract(os.path.join(REF, "hardnet/Losses.py"),
                  ["distance_matrix_vector", "loss_HardNet"]), ns)
    exec(_extract(os.path.join(REF, "hardnet/EvalMetrics.py"), ["ErrorRateAt95Recall"]), ns)
    torch.Tensor.cuda = lambda self, *a, **k: self  # CPU-only fixture generation
    rs = np.random.RandomState(5)
    out = {}
    for b in (64, 300):
        a = torch.from_numpy(rs.randn(b, 128).astype(np.float32))
        a = a / a.norm(dim=1, keepdim=True)
        p = a + 0.3 * torch.from_numpy(rs.randn(b, 128).astype(np.float32))
        p = p / p.norm(dim=1, keepdim=True)
        if b == 300:   # a duplicated positive exercises the <0.008 mask
            p[7] = a[11]
        out[f"a{b}"], out[f"p{b}"] = a.numpy(), p.numpy()
        out[f"dm{b}"] = ns["distance_matrix_vector"](a, p).numpy()
        for swap in (False, True):
            for lt in ("triplet_margin", "softmax", "contrastive"):
                out[f"loss{b}_{int(swap)}_{lt}"] = np.float32(
                    ns["loss_HardNet"](a, p, anchor_swap=swap, loss_type=lt).item())
    # FPR95 known-answer vectors
    labels = np.array([1, 1, 0, 1, 0, 0])
    dists = np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6])
    out["fpr_kat_labels"], out["fpr_kat_dists"] = labels, dists
    out["fpr_kat"] = np.float64(ns["ErrorRateAt95Recall"](labels, 1.0 / (dists + 1e-8)))
    n = 5000
    labels = (rs.rand(n) > 0.5).astype(np.int64)
    dists = np.where(labels == 1, rs.rand(n) * 0.9, 0.3 + rs.rand(n))
    out["fpr_labels"], out["fpr_dists"] = labels, dists
    out["fpr"] = np.float64(ns["ErrorRateAt95Recall"](labels, 1.0 / (dists + 1e-8)))
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **out)
    print("losses", out["fpr_kat"], out["fpr"])


def make_loss_modes():
    """loss_modes.npz: the reference loss_HardNet's 'average' and 'random' batch reductions
    (Losses.py:124-138; 'random' after torch.manual_seed(seed), so its randperm is reproducible),
    and the gradients of the 'min' reduce w.r.t. anchors and positives (the training step's
    backward, HardNet.py:421-423) in fp64 and fp32, for every loss type and anchor_swap."""
    ns = _ns()
    exec(_extract(os.path.join(REF, "hardnet/Losses.py"), ["distance_matrix_vector", "loss_HardNet"]), ns)
    torch.Tensor.cuda = lambda self, *a, **k: self  # CPU-only fixture generation
    rs = np.random.RandomState(17)
    out = {}
    b = 129
    a = torch.from_numpy(rs.randn(b, 128).astype(np.float32))
    a = a / a.norm(dim=1, keepdim=True)
    p = a + 0.3 * torch.from_numpy(rs.randn(b, 128).astype(np.float32))
    p = p / p.norm(dim=1, keepdim=True)
    p[5] = a[40]   # a masked near-duplicate negative
    p[9] = a[9]    # a zero positive distance
    out["a"], out["p"] = a.numpy(), p.numpy()
    for swap in (False, True):
        for lt in ("triplet_margin", "softmax", "contrastive"):
            tag = f"{int(swap)}_{lt}"
            for br in ("average", "random"):
                torch.manual_seed(23)
                out[f"{br}_{tag}"] = np.float64(ns["loss_HardNet"](a.double(), p.double(), anchor_swap=swap,
                                                                    batch_reduce=br, loss_type=lt).item())
            g = {}
            for dt, sfx in ((torch.float64, "64"), (torch.float32, "32")):
                ag = a.to(dt).clone().requires_grad_(True)
                pg = p.to(dt).clone().requires_grad_(True)
                loss = ns["loss_HardNet"](ag, pg, anchor_swap=swap, loss_type=lt)
                loss.backward()
                out[f"min_{tag}_{sfx}"] = np.float64(loss.item())
                g[sfx] = torch.cat([ag.grad, pg.grad]).double()
            # fp64 gradients (stored fp32) and the reference's own fp32 error on them (L2-relative)
            out[f"g_{tag}"] = g["64"].numpy().astype(np.float32)
            out[f"g32err_{tag}"] = np.float64((g["32"] - g["64"]).norm() / g["64"].norm())
    out["meta"] = json.dumps({"b": b, "random_seed": 23, "source": "hardnet/Losses.py loss_HardNet "
                              "(AST-extracted, torch %s CPU)" % torch.__version__})
    np.savez_compressed(os.path.join(HERE, "loss_modes.npz"), **out)
    print("loss modes", {k: float(v) for k, v in out.items() if k.startswith("average_1")})


NAS_FIXTURES = OrderedDict([
    ("wang2", A.MODEL_ARCH["wang2"]),
    ("wang3", A.MODEL_ARCH["wang3"]),
    ("wang4", A.MODEL_ARCH["wang4"]),
    # coverage archs: every CANDIDATE_BLOCKS op appears at least once
    ("cov_a", ["ir_k3_e3", "ir_k3_s4", "ir_k5_e3", "ir_k5_s4", "ir_k3_e1_se", "ir_k5_s2_se"]),
    ("cov_b", ["ir_k3_s4_se", "ir_k3_e3_se", "ir_k5_e1_se", "ir_k5_e3_se", "ir_k5_s4_se",
               "ir_k3_s2_se"]),
    ("cov_c", ["ir_k5_s2", "ir_k3_s2", "skip", "ir_k5_e1_se", "skip", "ir_k3_e3"]),
])

if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: fixtures can only be regenerated in the survey container")
    if sys.argv[1:] == ["loss_modes"]:
        make_loss_modes()
        sys.exit(0)
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: fixtures can only be regenerated in the survey container")
    torch.set_num_threads(8)
    make_hardnet()
    for name, ops in NAS_FIXTURES.items():
        make_nas(name, ops)
    make_losses()
    make_loss_modes()
    for v in A.FDL_VARIANTS:
        make_fdl(v)
