"""ORACLE -- test infrastructure only.

CPU restatement of the reference hot path (eval-mode descriptor forward), used as
the checker for the HIP path.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product path
(``hardnetnas_amd``) never does.

The restatement uses stock ``torch.nn.functional`` ops on CPU in fp32 -- the same
ATen ops the reference modules call -- driven by a plain ``{state_dict key: tensor}``
dict instead of nn.Modules.  ``dtype=torch.float64`` gives an fp64 reference.

Pinning: ``tests/golden/*.npz`` were produced by running the reference's own module
code (AST-extracted ``HardNet``/``L2Norm`` from hardnet/HardNet.py + hardnet/Utils.py,
and ``PRIMITIVES``/``ConvBNRelu`` imported from hardnetNAS/fbnet_building_blocks)
in the survey container (``tests/golden/make_golden.py``);
``tests/test_oracle_golden.py`` checks this restatement against those vectors.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

# ---- shared constants of the reference -----------------------------------------
BN_EPS = 1e-5                 # nn.BatchNorm2d default
HARDNET_INPUT_NORM_EPS = 1e-7  # hardnet/HardNet.py:308
HARDNET_L2_EPS = 1e-10         # hardnet/Utils.py:18

# hardnet/HardNet.py:280-302 : (conv idx, bn idx, stride, pad, relu)
_HARDNET_LAYERS = [(0, 1, 1, 1, True), (3, 4, 1, 1, True), (6, 7, 2, 1, True),
                   (9, 10, 1, 1, True), (12, 13, 2, 1, True), (15, 16, 1, 1, True),
                   (19, 20, 1, 0, False)]

CANDIDATE_BLOCKS = [
    "skip", "ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3", "ir_k5_s4",
    "ir_k3_e1_se", "ir_k3_e3_se", "ir_k3_s4_se", "ir_k5_e1_se", "ir_k5_e3_se",
    "ir_k5_s4_se", "ir_k3_s2", "ir_k5_s2", "ir_k3_s2_se", "ir_k5_s2_se",
]  # lookup_table_builder.py:18-20
SEARCH_SPACE2 = [(32, 32, 2), (32, 32, 1), (32, 64, 2), (64, 64, 1), (64, 128, 2),
                 (128, 128, 1)]  # lookup_table_builder.py:22-45


def _t(p, k, dtype):
    return torch.as_tensor(p[k]).to(dtype)


def input_norm(x: torch.Tensor, eps: float = HARDNET_INPUT_NORM_EPS) -> torch.Tensor:
    """hardnet/HardNet.py:306-310 -- torch.std is unbiased (N-1), eps after sqrt."""
    flat = x.view(x.size(0), -1)
    mp = torch.mean(flat, dim=1)
    sp = torch.std(flat, dim=1) + eps
    return (x - mp.view(-1, 1, 1, 1)) / sp.view(-1, 1, 1, 1)


def l2norm(x: torch.Tensor, eps: float = HARDNET_L2_EPS) -> torch.Tensor:
    """hardnet/Utils.py:15-22."""
    norm = torch.sqrt(torch.sum(x * x, dim=1) + eps)
    return x / norm.unsqueeze(-1)


def _bn(y, p, prefix, dtype, affine):
    """nn.BatchNorm2d eval semantics (running statistics)."""
    w = _t(p, prefix + ".weight", dtype) if affine else None
    b = _t(p, prefix + ".bias", dtype) if affine else None
    return F.batch_norm(y, _t(p, prefix + ".running_mean", dtype),
                        _t(p, prefix + ".running_var", dtype), w, b, False, 0.0, BN_EPS)


def hardnet_forward(p: Dict[str, torch.Tensor], x: torch.Tensor, dtype=torch.float32,
                    return_layers: bool = False, input_norm_eps=HARDNET_INPUT_NORM_EPS,
                    l2_eps=HARDNET_L2_EPS):
    """HardNet.forward, hardnet/HardNet.py:312-315 (eval: Dropout(0.3) is identity)."""
    y = input_norm(x.to(dtype), input_norm_eps)
    acts = [y]
    for ci, bi, s, pad, relu in _HARDNET_LAYERS:
        y = F.conv2d(y, _t(p, f"features.{ci}.weight", dtype), None, s, pad)
        y = _bn(y, p, f"features.{bi}", dtype, affine=False)
        if relu:
            y = F.relu(y)
        acts.append(y)
    out = l2norm(y.reshape(y.size(0), -1), l2_eps)
    return (out, acts) if return_layers else out


def hardnet_train_forward(p: Dict[str, torch.Tensor], x: torch.Tensor, running: Dict[str, torch.Tensor],
                          momentum: float = 0.1, dtype=torch.float32):
    """model.train() forward of HardNet (hardnet/HardNet.py:306-315 under :381): BatchNorm with the
    batch's statistics (biased variance normalises; the running update uses the unbiased one with
    ``momentum``, nn.BatchNorm2d), Dropout at p = 0.  ``running`` maps
    ``features.{i}.running_{mean,var}`` to tensors updated in place.  The weights in ``p`` may
    require grad: the result is differentiable (the training loop's backward, :421-423)."""
    y = input_norm(x.to(dtype))
    for ci, bi, s, pad, relu in _HARDNET_LAYERS:
        w = p[f"features.{ci}.weight"]
        y = F.conv2d(y, w if w.dtype == dtype else w.to(dtype), None, s, pad)
        y = F.batch_norm(y, running[f"features.{bi}.running_mean"], running[f"features.{bi}.running_var"],
                         None, None, True, momentum, BN_EPS)
        if relu:
            y = F.relu(y)
    return l2norm(y.reshape(y.size(0), -1))


# ---- hardnetNAS sampled descriptor ------------------------------------------------
# fbnet_builder.py:36-191 restricted to CANDIDATE_BLOCKS:
#   name -> (expansion, kernel, pw_group, se)   (shuffle iff pw_group > 1)
def _op_spec(name: str):
    if name == "skip":
        return None
    parts = name.split("_")            # ir, k3, e1|s2|s4, [se]
    k = int(parts[1][1:])
    if parts[2][0] == "e":
        e, g = int(parts[2][1:]), 1
    else:                                # s2: e=1,g=2 ; s4: e=4,g=4
        g = int(parts[2][1:])
        e = 1 if g == 2 else 4
    return e, k, g, len(parts) > 3 and parts[3] == "se"


def _cbr(y, p, prefix, dtype, stride, pad, groups, relu):
    """ConvBNRelu, fbnet_builder.py:352-404 (affine BN)."""
    y = F.conv2d(y, _t(p, prefix + ".conv.weight", dtype), None, stride, pad, 1, groups)
    y = _bn(y, p, prefix + ".bn", dtype, affine=True)
    return F.relu(y) if relu else y


def _shuffle(y, g):
    """ChannelShuffle, fbnet_builder.py:332-349."""
    n, c, h, w = y.shape
    return y.view(n, g, c // g, h, w).permute(0, 2, 1, 3, 4).contiguous().view(n, c, h, w)


def nas_layer(y, p, prefix, op, c_in, c_out, stride, dtype):
    spec = _op_spec(op)
    if spec is None:  # Identity, fbnet_builder.py:202-228
        if stride == 2:
            y = F.max_pool2d(y, 3, 2, 1)
        if c_in != c_out:
            sub = prefix + (".conv.1" if stride == 2 else ".conv")
            y = _cbr(y, p, sub, dtype, 1, 0, 1, True)
        return y
    e, k, g, se = spec  # IRFBlock.forward, fbnet_builder.py:559-570
    mid = int(c_in * e)
    x_in = y
    y = _cbr(y, p, prefix + ".pw", dtype, 1, 0, g, True)
    if g > 1:
        y = _shuffle(y, g)
    y = _cbr(y, p, prefix + ".dw", dtype, stride, k // 2, mid, True)
    y = _cbr(y, p, prefix + ".pwl", dtype, 1, 0, g, False)
    if stride == 1 and c_in == c_out:
        y = y + x_in
    if se:  # SEModule, fbnet_builder.py:407-421
        s = F.adaptive_avg_pool2d(y, 1)
        s = F.conv2d(s, _t(p, prefix + ".se4.op.1.weight", dtype),
                     _t(p, prefix + ".se4.op.1.bias", dtype))
        s = F.relu(s)
        s = F.conv2d(s, _t(p, prefix + ".se4.op.3.weight", dtype),
                     _t(p, prefix + ".se4.op.3.bias", dtype))
        y = y * torch.sigmoid(s)
    return y


def nas_forward(p: Dict[str, torch.Tensor], ops: Sequence[str], x: torch.Tensor,
                dtype=torch.float32, layers: Sequence[Tuple[int, int, int]] = SEARCH_SPACE2,
                return_layers: bool = False):
    """Sampled supernet forward (model_supernet.py:70-85 with argmax ops)."""
    y = _cbr(x.to(dtype), p, "first", dtype, 1, 1, 1, True)
    acts: List[torch.Tensor] = [y]
    for i, (op, (ci, co, s)) in enumerate(zip(ops, layers)):
        y = nas_layer(y, p, f"stages.{i}", op, ci, co, s, dtype)
        acts.append(y)
    y = F.conv2d(y, _t(p, "last_stages.conv_k1.weight", dtype))
    y = _bn(y, p, "last_stages.batchnorm", dtype, affine=False)
    y = y.reshape(y.size(0), -1)
    out = y / torch.norm(y, p=2, dim=-1, keepdim=True)   # model_supernet.py:84, no eps
    acts.append(out)
    return (out, acts) if return_layers else out


# ---- FDLNet hand-instantiated NAS descriptors (SURVEY 2 row 16, 8(c) fixture plan) ----
FDL_LAYERS = [(64, 64, 1), (64, 128, 2), (128, 128, 1)]
FDL_OPS = ["ir_k5_e1", "ir_k3_e3", "ir_k5_s2"]
FDL_INPUT_NORM_EPS = 1e-8  # latency/NASNet/model/des.py:40-47


def fdl_forward(p: Dict[str, torch.Tensor], variant: str, x: torch.Tensor, dtype=torch.float32):
    """HardNetNeiMask.forward, FDLNet-master/latency/NASNet/model/des.py:49-53 (variant
    "NASNet": features at des.py:13-36) and latency/NASNet_0.1/model/des.py:17-29
    ("NASNet_0.1").  input_norm with eps 1e-8 after the unbiased std; the stem conv has a
    bias; the IRFBlocks are latency/NASNet/model/operations.py:205-320 (= fbnet_builder's);
    L2 by torch.norm without eps."""
    y = input_norm(x.to(dtype), FDL_INPUT_NORM_EPS)
    y = F.conv2d(y, _t(p, "features.0.weight", dtype), _t(p, "features.0.bias", dtype), 1, 1)
    if variant == "NASNet":
        y = _bn(y, p, "features.1", dtype, affine=False)
        for conv, bn in ((2, 3), (5, 6)):  # Conv 1x1 s2 (no bias) + BN + ReLU
            y = F.conv2d(y, _t(p, f"features.{conv}.weight", dtype), None, 2)
            y = F.relu(_bn(y, p, f"features.{bn}", dtype, affine=True))
        first, head = 8, 11
    elif variant == "NASNet_0.1":
        y = F.max_pool2d(y, 3, 2, 1)
        # Identity(32, 32, 1) is the identity; Identity(32, 64, 2) = ConvBNRelu 1x1 stride 2
        y = _cbr(y, p, "features.3.conv", dtype, 2, 0, 1, True)
        first, head = 4, 7
    else:
        raise ValueError(variant)
    for i, (op, (ci, co, s)) in enumerate(zip(FDL_OPS, FDL_LAYERS)):
        y = nas_layer(y, p, f"features.{first + i}", op, ci, co, s, dtype)
    y = F.conv2d(y, _t(p, f"features.{head}.weight", dtype))
    y = _bn(y, p, f"features.{head + 1}", dtype, affine=False)
    y = y.reshape(y.size(0), -1)
    return y / torch.norm(y, p=2, dim=-1, keepdim=True)


# ---- losses / metrics ----------------------------------------
def distance_matrix_vector(anchor, positive):
    """hardnet/Losses.py:5-13."""
    d1_sq = torch.sum(anchor * anchor, dim=1).unsqueeze(-1)
    d2_sq = torch.sum(positive * positive, dim=1).unsqueeze(-1)
    eps = 1e-6
    return torch.sqrt((d1_sq.repeat(1, positive.size(0)) + torch.t(d2_sq.repeat(1, anchor.size(0)))
                       - 2.0 * torch.mm(anchor, torch.t(positive))) + eps)


def hardest_negative(anchor, positive, anchor_swap=False):
    """The 'min' batch_reduce of loss_HardNet, hardnet/Losses.py:87-110: returns
    (pos, min_neg) per row."""
    eps = 1e-8
    dm = distance_matrix_vector(anchor, positive) + eps
    eye = torch.eye(dm.size(1), dtype=dm.dtype, device=dm.device)
    pos1 = torch.diag(dm)
    d = dm + eye * 10
    mask = (d.ge(0.008).to(d.dtype) - 1.0) * (-1)
    d = d + mask * 10
    min_neg = torch.min(d, 1)[0]
    if anchor_swap:
        min_neg = torch.min(min_neg, torch.min(d, 0)[0])
    return pos1, min_neg


def hardest_negative_rows(anchor, positive, rows, anchor_swap=False):
    """(pos, min_neg) of hardest_negative for the given row indices only (the full matrix is
    never formed: row i needs row i and, with anchor_swap, column i of dm; Losses.py:95-108)."""
    eps = 1e-8
    rows = torch.as_tensor(rows)
    a, p = anchor, positive
    a_sq = torch.sum(a * a, dim=1)
    p_sq = torch.sum(p * p, dim=1)

    def masked(dm, diag_col):
        d = dm.clone()
        idx = torch.arange(d.shape[0])
        d[idx, diag_col] += 10
        return d + (d.ge(0.008).to(d.dtype) - 1.0) * (-1) * 10

    dm_r = torch.sqrt(a_sq[rows, None] + p_sq[None, :] - 2.0 * a[rows] @ p.t() + 1e-6) + eps
    pos = dm_r[torch.arange(len(rows)), rows]
    min_neg = masked(dm_r, rows).min(dim=1)[0]
    if anchor_swap:
        dm_c = torch.sqrt(p_sq[rows, None] + a_sq[None, :] - 2.0 * p[rows] @ a.t() + 1e-6) + eps
        min_neg = torch.minimum(min_neg, masked(dm_c, rows).min(dim=1)[0])
    return pos, min_neg


def loss_hardnet(anchor, positive, anchor_swap=False, margin=1.0, loss_type="triplet_margin"):
    """loss_HardNet with batch_reduce='min', hardnet/Losses.py:87-154."""
    eps = 1e-8
    pos, min_neg = hardest_negative(anchor, positive, anchor_swap)
    if loss_type == "triplet_margin":
        loss = torch.clamp(margin + pos - min_neg, min=0.0)
    elif loss_type == "softmax":
        exp_pos = torch.exp(2.0 - pos)
        exp_den = exp_pos + torch.exp(2.0 - min_neg) + eps
        loss = -torch.log(exp_pos / exp_den)
    elif loss_type == "contrastive":
        loss = torch.clamp(margin - min_neg, min=0.0) + pos
    else:
        raise ValueError(loss_type)
    return torch.mean(loss)


def error_rate_at_95_recall(labels, scores):
    """hardnet/EvalMetrics.py:6-19 (numpy quicksort argsort, as in the reference)."""
    import numpy as np
    distances = 1.0 / (scores + 1e-8)
    recall_point = 0.95
    labels = labels[np.argsort(distances)]
    threshold_index = np.argmax(np.cumsum(labels) >= recall_point * np.sum(labels))
    fp = np.sum(labels[:threshold_index] == 0)
    tn = np.sum(labels[threshold_index:] == 0)
    return float(fp) / float(fp + tn)
