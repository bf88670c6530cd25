"""Helpers that turn tests/golden/*.npz into parameters + inputs (no /root/reference)."""
from __future__ import annotations

import json
import os
from functools import lru_cache

import numpy as np
import torch

from hardnetnas_amd import synth
from hardnetnas_amd.model import HardNet, HardNetNAS, HardNetNeiMask

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAS_NAMES = ["wang2", "wang3", "wang4", "cov_a", "cov_b", "cov_c"]
FDL_NAMES = ["fdl_NASNet", "fdl_NASNet_01"]  # FDLNet HardNetNeiMask variants NASNet / NASNet_0.1


@lru_cache(maxsize=None)
def load(name: str):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    if "meta" in d:
        d["meta"] = json.loads(str(d["meta"]))
    return d


def params_for(module: torch.nn.Module, fx) -> dict:
    """Full state_dict (numpy) = synthetic weights (seeded) + committed BN stats."""
    meta = fx["meta"]
    tmpl = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    p = synth.synth_state_dict(tmpl, meta["weight_seed"])
    for k, sha in meta["weights_sha256"].items():
        assert synth.sha256_f32(p[k]) == sha, f"synthetic weight drift in {k}"
    for k in list(p):
        if "running" in k:
            p[k] = fx["bn/" + k]
    return p


def golden_inputs(fx) -> np.ndarray:
    meta = fx["meta"]
    return synth.synth_patches(meta["n_test"], meta["test_seed"])


def build_module(name: str):
    """(module in eval mode with fixture weights, fixture dict)."""
    if name.startswith("fdl_"):
        fx = load(name)
        m = HardNetNeiMask(variant=fx["meta"]["variant"])
    else:
        fx = load("hardnet" if name == "hardnet" else "nas_" + name)
        m = HardNet() if name == "hardnet" else HardNetNAS(fx["meta"]["ops"])
    p = params_for(m, fx)
    sd = m.state_dict()
    for k in sd:
        if k in p:
            sd[k] = torch.from_numpy(p[k])
    m.load_state_dict(sd)
    return m.eval(), fx, p


# ---- train-mode fixtures (tests/golden/train_*.npz, tests/golden/make_train_golden.py) -------
GRAD_SAMPLE = 16384   # entries kept per weight gradient (all of them for the smaller layers)
N_PROJ = 8            # +-1 projections of each full gradient (splitmix64 signs, seed 31 + layer)


def train_pairs(n: int, seed_a: int, seed_n: int):
    """Anchors and positives: synthetic patches; a positive is its anchor blended with another
    patch (0.75 / 0.25), so positive distances sit below most negatives as in real pairs."""
    a = synth.synth_patches(n, seed_a)
    o = synth.synth_patches(n, seed_n)
    return a, (0.75 * a + 0.25 * o).astype(np.float32)


def grad_sample_index(n: int) -> np.ndarray:
    """The entries of a flattened gradient a fixture keeps: every k-th, k = ceil(n / 16384)."""
    k = -(-n // GRAD_SAMPLE)
    return np.arange(0, n, k, dtype=np.int64)


def grad_projection_signs(i: int, n: int) -> np.ndarray:
    """[N_PROJ, n] +-1 matrix for gradient number ``i`` (regenerable without torch)."""
    bits = synth.splitmix64(31 + i, N_PROJ * n) >> np.uint64(63)
    return (1.0 - 2.0 * bits.astype(np.float64)).reshape(N_PROJ, n)


def grad_errors(g, fx, prefix: str, i: int) -> dict:
    """Errors of a full gradient ``g`` against a fixture's fp64 summary of the same gradient:
    L2-relative error over the sampled entries, relative error of the L2 norm, and of the +-1
    projections (RMS over the projections relative to the norm: a +-1 projection of an error
    vector e has RMS |e|, so all three estimate the L2-relative error)."""
    flat = np.asarray(g, dtype=np.float64).reshape(-1)
    ref_s = fx[f"{prefix}g{i}_sample"].astype(np.float64)
    got_s = flat[grad_sample_index(flat.size)]
    norm = float(fx[f"{prefix}g{i}_norm"])
    proj = grad_projection_signs(i, flat.size) @ flat
    return {"sample_l2rel": float(np.linalg.norm(got_s - ref_s) / max(1e-30, np.linalg.norm(ref_s))),
            "norm_rel": abs(float(np.linalg.norm(flat)) - norm) / max(1e-30, norm),
            "proj_rel": float(np.linalg.norm(proj - fx[f"{prefix}g{i}_proj"]) / np.sqrt(N_PROJ)
                              / max(1e-30, norm))}


TRAIN_CONV_IDX = (0, 3, 6, 9, 12, 15, 19)
TRAIN_BN_IDX = (1, 4, 7, 10, 13, 16, 20)


def train_start(init: str):
    """(HardNet module in train mode at a train fixture's starting point, fixture, anchors,
    positives): "golden" = synthetic weights + calibrated running stats of hardnet.npz;
    "fresh" = ``torch.manual_seed(0); HardNet()`` (the reference's own init, fresh buffers).
    Dropout is set to p = 0 as in the fixture (tests/golden/make_train_golden.py)."""
    fx = load("train_hardnet")
    meta = fx["meta"]
    if init == "golden":
        m, _, _ = build_module("hardnet")
    else:
        torch.manual_seed(0)
        m = HardNet()
    for i in TRAIN_CONV_IDX:
        w = m.features[i].weight.detach().numpy()
        if init == "golden":  # splitmix64 weights: bit-exact everywhere
            sha = meta["inits"][init]["weights_sha256"][f"features.{i}.weight"]
            assert synth.sha256_f32(w) == sha, f"{init} weight drift at {i}"
        else:  # torch's orthogonal_ (a LAPACK QR) reproduces to rounding on other CPUs
            wf = w.reshape(-1).astype(np.float64)
            ref = fx[f"fresh/w{i}_sample"].astype(np.float64)
            got = wf[grad_sample_index(wf.size)]
            assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max(), f"fresh weight drift at {i}"
            assert abs(np.linalg.norm(wf) - float(fx[f"fresh/w{i}_norm"])) <= 1e-5 * np.linalg.norm(wf)
    m.train()
    m.features[18].p = 0.0
    a, p = train_pairs(meta["n_pairs"], meta["seed_a"], meta["seed_n"])
    assert synth.sha256_f32(a) == meta["a_sha256"] and synth.sha256_f32(p) == meta["p_sha256"]
    return m, fx, a, p
