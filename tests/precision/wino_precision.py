"""Precision study (CPU, no GPU): HardNet forward with the stride-1 3x3 convs computed as
Winograd F(2x2,3x3) on bf16x3 split operands, against the fp64 oracle.

Emulation: transforms in fp32 (input / output) and fp64 -> bf16 hi/lo (filter, done once on
the host); products hi*hi + hi*lo + lo*hi accumulated in fp64 (the kernel accumulates in
fp32; that rounding is far below the split error).  Usage:
    python tests/precision/wino_precision.py [layers, e.g. 135] [n_patches]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fixtures import build_module, golden_inputs  # noqa: E402
from oracle import hardnet_oracle as O  # noqa: E402

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


MODE = os.environ.get("WINO_MODE", "bf16x3")  # bf16x3 | f16u1: V fp16 hi/lo, U one fp16


def split(x, dt=torch.bfloat16):
    h = x.to(dt).to(torch.float64)
    lo = (x.to(torch.float64) - h).to(dt).to(torch.float64)
    return h, lo


def conv_direct_x3(y, w, b):
    yh, yl = split(y)
    wh, wl = split(w)
    out = F.conv2d(yh, wh, None, 1, 1) + F.conv2d(yh, wl, None, 1, 1) + F.conv2d(yl, wh, None, 1, 1)
    return out + b.view(1, -1, 1, 1)


def conv_wino_x3(y, w, b):
    """y [P,C,H,H] fp32, w [K,C,3,3] fp64 (BN folded), b [K] -> [P,K,H,H]."""
    P, C, H, _ = y.shape
    T = H // 2
    yp = F.pad(y.to(torch.float32), (1, 1, 1, 1))
    # tiles d[P,C,T,T,4,4]
    d = yp.unfold(2, 4, 2).unfold(3, 4, 2)
    # V = BT d B in fp32
    V = torch.einsum("ab,pcijbd,ed->pcijae", BT.float(), d, BT.float())
    U = torch.einsum("ab,kcbd,ed->kcae", G, w, G)  # fp64
    if MODE == "f16u1":
        Vh, Vl = split(V, torch.float16)
        Uh = U.to(torch.float16).to(torch.float64)
        M = torch.einsum("kcae,pcijae->pkijae", Uh, Vh) + torch.einsum("kcae,pcijae->pkijae", Uh, Vl)
    else:
        Vh, Vl = split(V)
        Uh, Ul = split(U)
        M = (torch.einsum("kcae,pcijae->pkijae", Uh, Vh) + torch.einsum("kcae,pcijae->pkijae", Uh, Vl)
             + torch.einsum("kcae,pcijae->pkijae", Ul, Vh))
    M = M.to(torch.float32)
    Yt = torch.einsum("ra,pkijae,se->pkijrs", AT.float(), M, AT.float())  # [P,K,T,T,2,2]
    Yt = Yt.permute(0, 1, 2, 4, 3, 5).reshape(P, -1, H, H)
    return Yt.to(torch.float64) + b.view(1, -1, 1, 1)


def forward(p, x, wino_layers):
    dt = torch.float64
    y = O.input_norm(x.to(dt))
    for li, (ci, bi, s, pad, relu) in enumerate(O._HARDNET_LAYERS):
        w = torch.as_tensor(p[f"features.{ci}.weight"]).to(dt)
        rm = torch.as_tensor(p[f"features.{bi}.running_mean"]).to(dt)
        rv = torch.as_tensor(p[f"features.{bi}.running_var"]).to(dt)
        r = 1.0 / torch.sqrt(rv + O.BN_EPS)
        wf = w * r.view(-1, 1, 1, 1)
        bf = -rm * r
        if li in wino_layers:
            y = conv_wino_x3(y, wf, bf)
        elif li == 0 or li == 6:
            y = F.conv2d(y, wf, None, s, pad) + bf.view(1, -1, 1, 1)
        else:
            yh, yl = split(y)
            wh, wl = split(wf)
            y = (F.conv2d(yh, wh, None, s, pad) + F.conv2d(yh, wl, None, s, pad)
                 + F.conv2d(yl, wh, None, s, pad)) + bf.view(1, -1, 1, 1)
        if relu:
            y = F.relu(y)
        y = y.to(torch.float32).to(dt)
    return O.l2norm(y.reshape(y.size(0), -1))


def main():
    layers = {int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "35")}
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    m, fx, p = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)[:n])
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    ref = O.hardnet_forward(t, x, dtype=torch.float64)
    base = forward(p, x, set())
    got = forward(p, x, layers)
    print(f"direct bf16x3: max abs {float((base - ref).abs().max()):.3e}")
    print(f"wino layers {sorted(layers)}: max abs {float((got - ref).abs().max()):.3e}")


if __name__ == "__main__":
    main()
