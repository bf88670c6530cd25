"""Precision study (CPU, no GPU): HardNet forward with chosen stride-1 3x3 convs computed as a
1-D Winograd F(m, 3) along x (rows stay direct: the three kernel rows are three GEMMs per
transformed position), on bf16x3 split operands, against the fp64 oracle.

Emulation: input transform V = B^T d in fp32, filter transform U = G w in fp64 -> bf16 hi/lo
(done once on the host), products hi*hi + hi*lo + lo*hi summed in fp64 and rounded to fp32
(the kernel accumulates in fp32), output transform A^T m in fp32.  The matrices come from the
Toom-Cook points (infinity implied) for correlation, B^T solved from the defining identity.
Usage:
    python tests/precision/wino1d_precision.py "1:4 3:2 5:2" [n_patches] [points for m=4]
e.g. "1:4" = conv1 as F(4, 3); "3:2 5:2" = conv3 / conv5 as F(2, 3) (the production form).
"""
from __future__ import annotations

import os
import sys
from fractions import Fraction

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fixtures import build_module, golden_inputs, load  # noqa: E402
from oracle import hardnet_oracle as O  # noqa: E402


def toom_cook(m: int, r: int, pts):
    """(BT [n,n], G [n,r], AT [m,n]) for y_i = sum_k g_k d_{i+k}, points pts + infinity."""
    n = m + r - 1
    assert len(pts) == n - 1
    AT = np.zeros((m, n))
    G = np.zeros((n, r))
    for j, a in enumerate(pts):
        f = np.prod([a - b for k, b in enumerate(pts) if k != j])
        for i in range(m):
            AT[i, j] = a ** i
        for k in range(r):
            G[j, k] = a ** k / f
    AT[m - 1, n - 1] = 1.0
    G[n - 1, r - 1] = 1.0
    # solve BT from AT diag(G e_k) BT = T_k (correlation Toeplitz), k = 0..r-1
    rows, rhs = [], []
    for k in range(r):
        T = np.zeros((m, n))
        for i in range(m):
            T[i, i + k] = 1.0
        Mk = AT * G[:, k][None, :]  # [m, n]
        # (Mk @ BT)[i, c] = sum_j Mk[i, j] BT[j, c]
        for i in range(m):
            for c in range(n):
                row = np.zeros((n, n))
                row[:, c] = Mk[i, :]
                rows.append(row.ravel())
                rhs.append(T[i, c])
    A = np.array(rows)
    bt, res, *_ = np.linalg.lstsq(A, np.array(rhs), rcond=None)
    BT = bt.reshape(n, n)
    err = np.abs(A @ bt - np.array(rhs)).max()
    assert err < 1e-9, f"Toom-Cook solve failed ({err})"
    BT[np.abs(BT) < 1e-12] = 0.0
    return BT, G, AT


def split(x, dt=torch.bfloat16):
    h = x.to(dt).to(torch.float64)
    lo = (x.to(torch.float64) - h).to(dt).to(torch.float64)
    return h, lo


def conv_wino1d_x3(y, w, b, m, pts):
    """y [P,C,H,W] (fp32 values), w [K,C,3,3] fp64 (BN folded), b [K] -> [P,K,H,W]."""
    BT, G, AT = (torch.from_numpy(a) for a in toom_cook(m, 3, pts))
    P, C, H, W = y.shape
    n = m + 2
    yp = F.pad(y.to(torch.float32), (1, 1, 1, 1))
    out = torch.zeros(P, w.shape[0], H, W // m, n, dtype=torch.float64)
    for ky in range(3):
        rows = yp[:, :, ky:ky + H, :]                         # [P,C,H,W+2]
        d = rows.unfold(3, n, m)                              # [P,C,H,T,n]
        V = torch.einsum("ab,pchtb->pchta", BT.float(), d)    # fp32
        U = torch.einsum("ab,kcb->kca", G, w[:, :, ky, :])    # fp64
        Vh, Vl = split(V)
        Uh, Ul = split(U)
        out += (torch.einsum("kca,pchta->pkhta", Uh, Vh) + torch.einsum("kca,pchta->pkhta", Uh, Vl)
                + torch.einsum("kca,pchta->pkhta", Ul, Vh))
    M = out.to(torch.float32)
    Y = torch.einsum("ia,pkhta->pkhti", AT.float(), M).reshape(P, -1, H, W)
    return Y.to(torch.float64) + b.view(1, -1, 1, 1)


def forward(p, x, wino, pts4):
    dt = torch.float64
    y = O.input_norm(x.to(dt))
    for li, (ci, bi, s, pad, relu) in enumerate(O._HARDNET_LAYERS):
        w = torch.as_tensor(p[f"features.{ci}.weight"]).to(dt)
        rm = torch.as_tensor(p[f"features.{bi}.running_mean"]).to(dt)
        rv = torch.as_tensor(p[f"features.{bi}.running_var"]).to(dt)
        r = 1.0 / torch.sqrt(rv + O.BN_EPS)
        wf = w * r.view(-1, 1, 1, 1)
        bf = -rm * r
        if li in wino:
            m = wino[li]
            pts = [0.0, 1.0, -1.0] if m == 2 else pts4
            y = conv_wino1d_x3(y, wf, bf, m, pts)
        elif li == 6:
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
    spec = sys.argv[1] if len(sys.argv) > 1 else "1:4 3:2 5:2"
    wino = {int(a): int(b) for a, b in (t.split(":") for t in spec.split())}
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    pts4 = [float(Fraction(t)) for t in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, -1, 2, -2]
    m, fx, p = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)[:n])
    xe = torch.from_numpy(load("hardnet")["x_edge"])
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    for name, xx in (("random", x), ("edge", xe)):
        ref = O.hardnet_forward(t, xx, dtype=torch.float64)
        base = forward(p, xx, {}, pts4)
        got = forward(p, xx, wino, pts4)
        print(f"{name}: direct bf16x3 max abs {float((base - ref).abs().max()):.3e}; "
              f"wino {spec} pts4 {pts4}: max abs {float((got - ref).abs().max()):.3e}")


if __name__ == "__main__":
    main()
