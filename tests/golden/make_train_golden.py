"""Train-mode fixtures from the REFERENCE code (survey container only).

Run from the repo root:  python tests/golden/make_train_golden.py
Writes tests/golden/train_hardnet.npz, train_nas.npz and train_fdl.npz (data only; the reference is
executed, never copied).

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
    return F.summary(g, i)


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


# ---- hardnetNAS --------------------------------------------------------------------------
NAS_TRAIN = {"wang2": None, "cov_b": None}   # a plain arch and one with SE + shuffles in every layer
NAS_PAIRS = 64
SUPER_PAIRS = 32
SUPER_SEED = 5
SUPER_TEMPERATURE = 5.0          # config_for_supernet.py: init_temperature
SUPER_TARGET = 15.0              # config_for_supernet.py: target_latency
SUPER_SAMPLE = 64                # sampled entries per supernet gradient (1,650 tensors)


def _nas_ref():
    sys.path.insert(0, os.path.join(G.REF, "hardnetNAS"))
    from fbnet_building_blocks.fbnet_builder import PRIMITIVES
    from supernet_functions.model_supernet import FBNet_Stochastic_SuperNet, SupernetLoss
    import general_functions.Losses as NL
    return PRIMITIVES, FBNet_Stochastic_SuperNet, SupernetLoss, NL


def _to_super(k, idx):
    if k.startswith("stages."):
        p = k.split(".")
        return ".".join(["stages_to_search", p[1], "ops", str(idx[int(p[1])])] + p[2:])
    return k


def make_train_nas(out, name):
    """One step of the supernet training loop's shape (training_functions_supernet.py:88-103) over a
    SAMPLED net: two calls of the module in train() (X, Y), the hardnetNAS loss_HardNet
    (general_functions/Losses.py:27-51), backward.  The sampled net is the reference supernet with
    each MixedOperation replaced by its arch op (as tests/golden/make_golden.py::make_nas), at the
    golden synthetic weights + calibrated running statistics, BN momentum 0.1."""
    from hardnetnas_amd.model import HardNetNAS
    PRIMITIVES, SuperNet, _, NL = _nas_ref()
    fx = np.load(os.path.join(HERE, f"nas_{name}.npz"), allow_pickle=False)
    ops = json.loads(str(fx["meta"]))["ops"]
    idx = [G.A.CANDIDATE_BLOCKS.index(op) for op in ops]
    ours = HardNetNAS(ops)
    tmpl = {k: tuple(v.shape) for k, v in ours.state_dict().items()}
    w = synth.synth_state_dict(tmpl, G.WEIGHT_SEED)
    a, p = F.train_pairs(NAS_PAIRS, SEED_A + 10, SEED_N + 10)
    res = {}
    for tag, dtype in (("32", torch.float32), ("64", torch.float64)):
        lut = G._StubLUT()
        lut.lookup_table_operations = {op: PRIMITIVES[op] for op in G.A.CANDIDATE_BLOCKS}
        torch.manual_seed(0)
        sup = SuperNet(lut)
        ssd = sup.state_dict()
        for k, v in w.items():
            ssd[_to_super(k, idx)] = torch.from_numpy(fx["bn/" + k] if "running" in k else v)
        sup.load_state_dict(ssd)
        sup = sup.to(dtype).train()

        def fwd(x):  # model_supernet.py:70-85 with the arch ops
            y = sup.first(x)
            for i, j in enumerate(idx):
                y = sup.stages_to_search[i].ops[j](y)
            y = sup.last_stages(y)
            return y / torch.norm(y, p=2, dim=-1, keepdim=True)

        oa = fwd(torch.from_numpy(a).to(dtype))
        op_ = fwd(torch.from_numpy(p).to(dtype))
        loss = NL.loss_HardNet(oa, op_)
        loss.backward()
        ssd = sup.state_dict(keep_vars=True)
        r = {"out_a": oa.detach().numpy(), "out_p": op_.detach().numpy(), "loss": np.float64(loss.item()),
             "stats": {}, "grads": {}}
        for k in tmpl:
            t = ssd[_to_super(k, idx)]
            if "running" in k:
                r["stats"][k] = t.detach().numpy()
            elif not k.endswith("num_batches_tracked"):
                r["grads"][k] = t.grad.numpy()
        res[tag] = r
    pre = f"nas_{name}/"
    for tag in ("32", "64"):
        r = res[tag]
        cast = (lambda v: v.astype(np.float32)) if tag == "32" else (lambda v: v)
        out[f"{pre}out_a_{tag}"], out[f"{pre}out_p_{tag}"] = cast(r["out_a"]), cast(r["out_p"])
        out[f"{pre}loss_{tag}"] = r["loss"]
        for k, v in r["stats"].items():
            out[f"{pre}stat/{k}_{tag}"] = cast(v)
    fp32_err = {}
    for k, g64 in res["64"]["grads"].items():
        for kk, v in F.summary(g64, F.name_seed(k)).items():
            out[f"{pre}g/{k}_{kk}"] = v
        g32 = res["32"]["grads"][k].astype(np.float64)
        n = np.linalg.norm(g64)
        fp32_err[k] = float(np.linalg.norm(g32 - g64) / n) if n > 0 else 0.0
        if n < 1e-9 * max(np.linalg.norm(v) for v in res["64"]["grads"].values()):
            fp32_err[k] = 0.0  # a gradient that is zero in exact arithmetic (nas_grad_check)
    out[f"{pre}grad_names"] = np.array(sorted(fp32_err))
    out[f"{pre}fp32_err"] = np.array([fp32_err[k] for k in sorted(fp32_err)])
    print("nas", name, "loss", res["32"]["loss"], res["64"]["loss"], "worst fp32 grad err",
          max(fp32_err.values()))
    return {"ops": ops, "n_pairs": NAS_PAIRS, "seed_a": SEED_A + 10, "seed_n": SEED_N + 10,
            "momentum": 0.1, "fp32_grad_l2rel_vs_fp64": fp32_err,
            "source": "hardnetNAS FBNet_Stochastic_SuperNet + PRIMITIVES + general_functions/Losses.py:27-51 "
                      "(imported, torch %s CPU)" % torch.__version__}


def make_train_supernet(out):
    """One step of the supernet training loop itself (training_functions_supernet.py:88-103) over the
    reference FBNet_Stochastic_SuperNet: outs_X = model(X, T, lat0) with grad, outs_Y under
    no_grad, SupernetLoss (model_supernet.py:88-110: loss_HardNet + the latency term), backward.
    The Gumbel noise of every gumbel_softmax draw (6 per call) is recorded -- the same draw as
    torch's F.gumbel_softmax: g = -log(Exponential(1)), softmax((thetas + g) / T) -- so the HIP
    path can be fed the identical soft weights.  Synthetic weights (splitmix64 seed 1234), fresh
    BatchNorm buffers, synthetic per-op latencies 1 + 9u."""
    PRIMITIVES, SuperNet, SupernetLoss, NL = _nas_ref()
    import torch.nn.functional as TF
    lat = synth.uniform(77, 6 * 17).reshape(6, 17) * 9.0 + 1.0
    a, p = F.train_pairs(SUPER_PAIRS, SEED_A + 20, SEED_N + 20)
    res = {}
    orig = TF.gumbel_softmax
    for tag, dtype in (("32", torch.float32), ("64", torch.float64)):
        lut = G._StubLUT()
        lut.lookup_table_operations = {op: PRIMITIVES[op] for op in G.A.CANDIDATE_BLOCKS}
        lut.lookup_table_latency = [{op: float(lat[i, j]) for j, op in enumerate(G.A.CANDIDATE_BLOCKS)}
                                    for i in range(6)]
        torch.manual_seed(0)
        sup = SuperNet(lut)
        sd = sup.state_dict()
        tmpl = {k: tuple(v.shape) for k, v in sd.items() if not k.endswith(".thetas")}
        w = synth.synth_state_dict(tmpl, G.WEIGHT_SEED)
        sd.update({k: torch.from_numpy(v) for k, v in w.items()})
        sup.load_state_dict(sd)
        sup = sup.to(dtype).train()
        noise = []

        replay = list(res["32"]["noise"]) if tag == "64" else None  # the fp64 run replays the fp32 draws

        def gumbel(logits, tau=1.0, hard=False, eps=1e-10, dim=-1):
            if replay is None:
                g = -torch.empty_like(logits).exponential_().log()
            else:
                g = torch.from_numpy(replay.pop(0)).to(logits.dtype)
            noise.append(g.detach().numpy().copy())
            return ((logits + g) / tau).softmax(dim)

        TF.gumbel_softmax = gumbel
        # MixedOperation.softnms convolves with an fp32 torch.ones kernel (model_supernet.py:45),
        # which F.conv1d refuses for an fp64 input: the fp64 run casts that kernel (fixture only)
        conv1d = TF.conv1d
        TF.conv1d = lambda inp, weight, *a_, **k_: conv1d(inp, weight.to(inp.dtype), *a_, **k_)
        try:
            torch.manual_seed(SUPER_SEED)
            lat0 = torch.tensor([[0.0]], dtype=dtype, requires_grad=True)
            oX, lacc, soft1, hard1 = sup(torch.from_numpy(a).to(dtype), SUPER_TEMPERATURE, lat0)
            with torch.no_grad():
                oY, _, _, _ = sup(torch.from_numpy(p).to(dtype), SUPER_TEMPERATURE, lacc)
            crit = SupernetLoss()
            crit.weight_criterion_hardnet = NL.loss_HardNet
            loss, ce, latl = crit(oX, oY, lacc, soft1, SUPER_TARGET)
            loss.backward()
        finally:
            TF.gumbel_softmax = orig
            TF.conv1d = conv1d
        sdv = sup.state_dict(keep_vars=True)
        r = {"out_x": oX.detach().numpy(), "out_y": oY.detach().numpy(), "loss": float(loss.item()),
             "ce": float(ce.item()), "lat": float(latl.item()), "noise": np.stack(noise),
             "thetas_grad": np.stack([sup.stages_to_search[i].thetas.grad.numpy() for i in range(6)]),
             "grads": {k: sdv[k].grad.numpy() for k in tmpl if "running" not in k and
                       not k.endswith("num_batches_tracked")},
             "stat_norms": {k: float(np.linalg.norm(sdv[k].detach().numpy().astype(np.float64)))
                            for k in tmpl if "running" in k}}
        res[tag] = r
    pre = "super/"
    out[f"{pre}noise"] = res["32"]["noise"].astype(np.float32)   # [2 calls x 6 layers][17]
    out[f"{pre}latency"] = lat
    for tag in ("32", "64"):
        r = res[tag]
        cast = (lambda v: v.astype(np.float32)) if tag == "32" else (lambda v: v)
        out[f"{pre}out_x_{tag}"], out[f"{pre}out_y_{tag}"] = cast(r["out_x"]), cast(r["out_y"])
        out[f"{pre}thetas_grad_{tag}"] = r["thetas_grad"]
        for kk in ("loss", "ce", "lat"):
            out[f"{pre}{kk}_{tag}"] = np.float64(r[kk])
        out[f"{pre}stat_names"] = np.array(sorted(r["stat_norms"]))
        out[f"{pre}stat_norms_{tag}"] = np.array([r["stat_norms"][k] for k in sorted(r["stat_norms"])])
    names = sorted(res["64"]["grads"])
    out[f"{pre}grad_names"] = np.array(names)
    fp32_err = {}
    for k in names:
        g64 = res["64"]["grads"][k]
        for kk, v in F.summary(g64, F.name_seed(k), SUPER_SAMPLE).items():
            out[f"{pre}g/{k}_{kk}"] = v
        n = np.linalg.norm(g64)
        fp32_err[k] = float(np.linalg.norm(res["32"]["grads"][k].astype(np.float64) - g64) / n) if n > 0 else 0.0
        if n < 1e-9 * max(np.linalg.norm(v) for v in res["64"]["grads"].values()):
            fp32_err[k] = 0.0  # a gradient that is zero in exact arithmetic (nas_grad_check)
    out[f"{pre}fp32_err"] = np.array([fp32_err[k] for k in names])
    print("supernet loss", res["32"]["loss"], res["64"]["loss"], "worst fp32 grad err", max(fp32_err.values()))
    return {"n_pairs": SUPER_PAIRS, "seed_a": SEED_A + 20, "seed_n": SEED_N + 20, "torch_seed": SUPER_SEED,
            "temperature": SUPER_TEMPERATURE, "target_latency": SUPER_TARGET, "sample": SUPER_SAMPLE,
            "momentum": 0.1, "fp32_grad_l2rel_vs_fp64_worst": max(fp32_err.values()),
            "source": "hardnetNAS supernet_functions/model_supernet.py FBNet_Stochastic_SuperNet + SupernetLoss, "
                      "training_functions_supernet.py:88-103 (imported, torch %s CPU)" % torch.__version__}


def _fdl_ref(variant):
    """FDLNet HardNetNeiMask (latency/<variant>/model/des.py), imported with its package root on
    sys.path, as tests/golden/make_golden.py::make_fdl does."""
    for k in [k for k in sys.modules if k.split(".")[0] in ("model", "utils")]:
        del sys.modules[k]
    sys.path.insert(0, os.path.join(G.REF, "FDLNet-master", "latency", variant))
    try:
        from model.des import HardNetNeiMask as RefNet
    finally:
        sys.path.pop(0)
    return RefNet


def make_train_fdl(out, variant):
    """One train step of FDLNet's HardNetNeiMask in the loop shape the other fixtures use (two
    train() calls, the hardnetNAS loss_HardNet, backward; FDLNet's own neighbour-mask loss is out of
    scope), at the golden synthetic weights + calibrated running statistics of
    fdl_<variant>.npz, BN momentum 0.1."""
    from hardnetnas_amd.model import HardNetNeiMask
    _, _, _, NL = _nas_ref()
    RefNet = _fdl_ref(variant)
    tag = variant.replace(".", "")
    fx = np.load(os.path.join(HERE, f"fdl_{tag}.npz"), allow_pickle=False)
    tmpl = {k: tuple(v.shape) for k, v in HardNetNeiMask(variant=variant).state_dict().items()}
    w = synth.synth_state_dict(tmpl, G.WEIGHT_SEED)
    a, p = F.train_pairs(NAS_PAIRS, SEED_A + 20, SEED_N + 20)
    res = {}
    for dt, dtype in (("32", torch.float32), ("64", torch.float64)):
        torch.manual_seed(0)
        model = RefNet(1.0, 1.0)
        sd = model.state_dict()
        assert tmpl == {k: tuple(v.shape) for k, v in sd.items()}, "state_dict layout differs"
        for k, v in w.items():
            sd[k] = torch.from_numpy(fx["bn/" + k] if "running" in k else v)
        model.load_state_dict(sd)
        model = model.to(dtype).train()
        oa = model(torch.from_numpy(a).to(dtype))
        op_ = model(torch.from_numpy(p).to(dtype))
        loss = NL.loss_HardNet(oa, op_)
        loss.backward()
        msd = model.state_dict(keep_vars=True)
        r = {"out_a": oa.detach().numpy(), "out_p": op_.detach().numpy(), "loss": np.float64(loss.item()),
             "stats": {}, "grads": {}}
        for k in tmpl:
            t = msd[k]
            if "running" in k:
                r["stats"][k] = t.detach().numpy()
            elif not k.endswith("num_batches_tracked"):
                r["grads"][k] = t.grad.numpy()
        res[dt] = r
    pre = f"fdl_{tag}/"
    for dt in ("32", "64"):
        r = res[dt]
        cast = (lambda v: v.astype(np.float32)) if dt == "32" else (lambda v: v)
        out[f"{pre}out_a_{dt}"], out[f"{pre}out_p_{dt}"] = cast(r["out_a"]), cast(r["out_p"])
        out[f"{pre}loss_{dt}"] = r["loss"]
        for k, v in r["stats"].items():
            out[f"{pre}stat/{k}_{dt}"] = cast(v)
    fp32_err = {}
    gmax = max(np.linalg.norm(v) for v in res["64"]["grads"].values())
    for k, g64 in res["64"]["grads"].items():
        for kk, v in F.summary(g64, F.name_seed(k)).items():
            out[f"{pre}g/{k}_{kk}"] = v
        g32 = res["32"]["grads"][k].astype(np.float64)
        n = np.linalg.norm(g64)
        fp32_err[k] = float(np.linalg.norm(g32 - g64) / n) if n > 1e-9 * gmax else 0.0
    out[f"{pre}grad_names"] = np.array(sorted(fp32_err))
    out[f"{pre}fp32_err"] = np.array([fp32_err[k] for k in sorted(fp32_err)])
    print("fdl", variant, "loss", res["32"]["loss"], res["64"]["loss"], "worst fp32 grad err",
          max(fp32_err.values()))
    return {"variant": variant, "n_pairs": NAS_PAIRS, "seed_a": SEED_A + 20, "seed_n": SEED_N + 20,
            "momentum": 0.1, "fp32_grad_l2rel_vs_fp64": fp32_err,
            "source": "FDLNet-master/latency/%s/model/des.py HardNetNeiMask + hardnetNAS "
                      "general_functions/Losses.py:27-51 (imported, torch %s CPU)" % (variant, torch.__version__)}


def make_train_fdl_all():
    torch.Tensor.cuda = lambda self, *a, **k: self  # the loss's eye().cuda(): CPU fixture generation
    out, meta = {}, {}
    for v in G.A.FDL_VARIANTS:
        meta[v.replace(".", "")] = make_train_fdl(out, v)
    out["meta"] = json.dumps(meta)
    np.savez_compressed(os.path.join(HERE, "train_fdl.npz"), **out)


def make_train_nas_all():
    torch.Tensor.cuda = lambda self, *a, **k: self  # the losses' eye().cuda(): CPU fixture generation
    out, meta = {}, {}
    for name in NAS_TRAIN:
        meta[name] = make_train_nas(out, name)
    meta["supernet"] = make_train_supernet(out)
    out["meta"] = json.dumps(meta)
    np.savez_compressed(os.path.join(HERE, "train_nas.npz"), **out)


if __name__ == "__main__":
    if not os.path.isdir(G.REF):
        sys.exit(f"{G.REF} not found: fixtures can only be regenerated in the survey container")
    torch.set_num_threads(8)
    if len(sys.argv) < 2 or sys.argv[1] == "hardnet":
        make_train_hardnet()
    if len(sys.argv) < 2 or sys.argv[1] == "nas":
        make_train_nas_all()
    if len(sys.argv) < 2 or sys.argv[1] == "fdl":
        make_train_fdl_all()
