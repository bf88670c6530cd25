"""Train-mode fixtures from the REFERENCE code (survey container only).

Run from the repo root:  python tests/golden/make_train_golden.py
Writes tests/golden/train_hardnet.npz (data only; the reference is executed, never copied).

One step of the reference training loop, in its own shape (hardnet/HardNet.py:379-423):

    model.train()
    out_a = model(data_a); out_p = model(data_p)          # two calls: two BN batch statistics,
                                                          # two running-stat updates
    loss = loss_HardNet(out_a, out_p, anchor_swap=True)   # Losses.py:87-154 (batch_reduce 'min')
    loss.backward()

``class HardNet`` + ``weights_init`` (HardNet.py:275-324), ``L2Norm`` (Utils.py:15-22) and
``distance_matrix_vector`` / ``loss_HardNet`` (Losses.py:5-13, 87-154) are AST-extracted and
executed (the modules themselves cannot be imported here).  Dropout is set to
p = 0 (the reference draws its mask from torch's RNG; the HIP path from a counter hash).

Two starting points, both with BatchNorm momentum 0.1 (the module default):
  * "golden": the synthetic weights + calibrated running statistics of tests/golden/hardnet.npz;
  * "fresh":  ``torch.manual_seed(0); HardNet()`` -- the reference's own orthogonal init and fresh
              BatchNorm buffers (the weights are regenerated on the box the same way and checked
              by SHA-256).
For each: out_a / out_p, the loss, every running_mean / running_var after the step and
num_batches_tracked, and the 7 conv weight gradients -- from the fp32 module and from the same
module in fp64.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from hardnetnas_amd import synth       # noqa: E402
import make_golden as G                # noqa: E402
sys.path.insert(0, os.path.dirname(HERE))
import fixtures as F                   # noqa: E402  (tests/fixtures.py: sampling helpers)

N_PAIRS = 128
SEED_A, SEED_N = 21, 22
CONV_IDX = (0, 3, 6, 9, 12, 15, 19)
BN_IDX = (1, 4, 7, 10, 13, 16, 20)


def _ref_ns():
    ns = G._ns()
    exec(G._extract(os.path.join(G.REF, "hardnet/Utils.py"), ["L2Norm"]), ns)
    exec(G._extract(os.path.join(G.REF, "hardnet/HardNet.py"), ["HardNet", "weights_init"]), ns)
    exec(G._extract(os.path.join(G.REF, "hardnet/Losses.py"),
                    ["distance_matrix_vector", "loss_HardNet"]), ns)
    return ns


def _step(model, a, p, loss_fn, dtype):
    model = model.to(dtype).train()
    model.features[18].p = 0.0
    out_a = model(torch.from_numpy(a).to(dtype))
    out_p = model(torch.from_numpy(p).to(dtype))
    loss = loss_fn(out_a, out_p, anchor_swap=True)
    loss.backward()
    sd = model.state_dict()
    r = {"out_a": out_a.detach().numpy(), "out_p": out_p.detach().numpy(),
         "loss": np.float64(loss.item())}
    for i in BN_IDX:
        r[f"rm{i}"] = sd[f"features.{i}.running_mean"].numpy()
        r[f"rv{i}"] = sd[f"features.{i}.running_var"].numpy()
        r[f"nbt{i}"] = np.int64(sd[f"features.{i}.num_batches_tracked"].item())
    for i in CONV_IDX:
        r[f"g{i}"] = model.features[i].weight.grad.numpy()
    return r


def grad_summary(g: np.ndarray, i: int) -> dict:
    flat = g.reshape(-1).astype(np.float64)
    return {"sample": flat[F.grad_sample_index(flat.size)].astype(np.float32),
            "norm": np.float64(np.linalg.norm(flat)),
            "proj": F.grad_projection_signs(i, flat.size) @ flat}


def make_train_hardnet():
    ns = _ref_ns()
    torch.Tensor.cuda = lambda self, *a, **k: self  # the loss's eye().cuda(): CPU fixture generation
    gold = np.load(os.path.join(HERE, "hardnet.npz"), allow_pickle=False)
    a, p = F.train_pairs(N_PAIRS, SEED_A, SEED_N)
    out = {}
    meta = {"n_pairs": N_PAIRS, "seed_a": SEED_A, "seed_n": SEED_N, "blend": [0.75, 0.25],
            "a_sha256": synth.sha256_f32(a), "p_sha256": synth.sha256_f32(p),
            "dropout_p": 0.0, "momentum": 0.1, "anchor_swap": True,
            "source": "hardnet/HardNet.py:275-324,379-423 + Utils.py:15-22 + Losses.py:5-13,87-154 "
                      "(AST-extracted, executed with torch %s CPU)" % torch.__version__,
            "inits": {}}
    for init in ("golden", "fresh"):
        res = {}
        for tag, dtype in (("32", torch.float32), ("64", torch.float64)):
            torch.manual_seed(0)
            model = ns["HardNet"]()
            if init == "golden":
                sd = model.state_dict()
                tmpl = {k: tuple(v.shape) for k, v in sd.items()}
                w = synth.synth_state_dict(tmpl, G.WEIGHT_SEED)
                for k, v in w.items():
                    sd[k] = torch.from_numpy(gold["bn/" + k] if "running" in k else v)
                model.load_state_dict(sd)
            w_sha = {f"features.{i}.weight": synth.sha256_f32(model.features[i].weight.detach().numpy())
                     for i in CONV_IDX}
            if init == "fresh" and tag == "32":
                # orthogonal_ runs a LAPACK QR: other CPUs reproduce it only to rounding, so the
                # box checks these weights against a summary with a tolerance, not the SHA-256
                for i in CONV_IDX:
                    wf = model.features[i].weight.detach().numpy().reshape(-1)
                    out[f"fresh/w{i}_sample"] = wf[F.grad_sample_index(wf.size)]
                    out[f"fresh/w{i}_norm"] = np.float64(np.linalg.norm(wf.astype(np.float64)))
            res[tag] = _step(model, a, p, ns["loss_HardNet"], dtype)
        meta["inits"][init] = {"weights_sha256": w_sha}
        # weight gradients: the fp64 module's, summarised (sampled entries, full L2 norm, +-1
        # projections); the fp32 module's error against it is recorded in meta
        meta["inits"][init]["fp32_grad_l2rel_vs_fp64"] = {}
        for i in CONV_IDX:
            g32, g64 = res["32"].pop(f"g{i}"), res["64"].pop(f"g{i}")
            for k, v in grad_summary(g64, i).items():
                out[f"{init}/g{i}_{k}"] = v
            meta["inits"][init]["fp32_grad_l2rel_vs_fp64"][str(i)] = float(
                np.linalg.norm(g32.astype(np.float64) - g64) / np.linalg.norm(g64))
        for tag in ("32", "64"):
            for k, v in res[tag].items():
                if k.startswith("nbt") and tag == "64":
                    continue
                out[f"{init}/{k}{'' if k.startswith('nbt') else '_' + tag}"] = (
                    v.astype(np.float32) if (tag == "32" and isinstance(v, np.ndarray)
                                             and v.dtype != np.int64) else v)
        print(init, "loss32", res["32"]["loss"], "loss64", res["64"]["loss"],
              "max|out32-out64|", float(np.abs(res["32"]["out_a"] - res["64"]["out_a"]).max()))
    out["meta"] = json.dumps(meta)
    np.savez_compressed(os.path.join(HERE, "train_hardnet.npz"), **out)


if __name__ == "__main__":
    if not os.path.isdir(G.REF):
        sys.exit(f"{G.REF} not found: fixtures can only be regenerated in the survey container")
    torch.set_num_threads(8)
    make_train_hardnet()
