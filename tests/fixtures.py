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
