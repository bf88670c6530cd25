"""Precision study (CPU, no GPU): HardNet forward with the 3x3 convs computed from split
operands, against the fp64 oracle, to price dropping one of the three bf16x3 products.

Modes (products accumulated in fp64; the kernels accumulate in fp32, far below these errors):
    bf16x3   x_hi*w_hi + x_hi*w_lo + x_lo*w_hi, bf16 halves (what the kernels do)
    fp16x2w  x_hi*(w_hi + w_lo): activation rounded once to fp16, weight split in fp16
             (weights pre-scaled by 2^SC so w_lo stays a normal fp16; undone in the epilogue)
    fp16x2x  (x_hi + x_lo)*w_hi: activation split, weight rounded once to fp16
    bf16x2w  x_hi*(w_hi + w_lo) with bf16 halves
Usage:
    python tests/precision/split_precision.py [mode] [layers, e.g. 12345] [n_patches]
"""
from __future__ import annotations

import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fixtures import build_module, golden_inputs  # noqa: E402
from oracle import hardnet_oracle as O  # noqa: E402

SC = 2.0 ** 8


def split(x, dt):
    h = x.to(dt).to(torch.float64)
    lo = (x.to(torch.float64) - h).to(dt).to(torch.float64)
    return h, lo


def conv(mode, y, w, s, pad):
    if mode == "bf16x3":
        yh, yl = split(y, torch.bfloat16)
        wh, wl = split(w, torch.bfloat16)
        return F.conv2d(yh, wh, None, s, pad) + F.conv2d(yh, wl, None, s, pad) + F.conv2d(yl, wh, None, s, pad)
    if mode in ("fp16x2w", "bf16x2w"):
        dt = torch.float16 if mode == "fp16x2w" else torch.bfloat16
        sc = SC if dt == torch.float16 else 1.0
        yh = y.to(dt).to(torch.float64)
        wh, wl = split(w * sc, dt)
        return (F.conv2d(yh, wh, None, s, pad) + F.conv2d(yh, wl, None, s, pad)) / sc
    if mode == "fp16x2x":
        yh, yl = split(y, torch.float16)
        wh = (w * SC).to(torch.float16).to(torch.float64)
        return (F.conv2d(yh, wh, None, s, pad) + F.conv2d(yl, wh, None, s, pad)) / SC
    raise ValueError(mode)


def forward(p, x, mode, layers):
    dt = torch.float64
    y = O.input_norm(x.to(dt))
    for li, (ci, bi, s, pad, relu) in enumerate(O._HARDNET_LAYERS):
        w = torch.as_tensor(p[f"features.{ci}.weight"]).to(dt)
        rm = torch.as_tensor(p[f"features.{bi}.running_mean"]).to(dt)
        rv = torch.as_tensor(p[f"features.{bi}.running_var"]).to(dt)
        r = 1.0 / torch.sqrt(rv + O.BN_EPS)
        wf = w * r.view(-1, 1, 1, 1)
        bf = -rm * r
        y = conv(mode if li in layers else "bf16x3", y, wf, s, pad) + bf.view(1, -1, 1, 1)
        if relu:
            y = F.relu(y)
        y = y.to(torch.float32).to(dt)
    return O.l2norm(y.reshape(y.size(0), -1))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "fp16x2w"
    layers = {int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "0123456")}
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    m, fx, p = build_module("hardnet")
    x = torch.from_numpy(golden_inputs(fx)[:n])
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    ref = O.hardnet_forward(t, x, dtype=torch.float64)
    base = forward(p, x, "bf16x3", set())
    got = forward(p, x, mode, layers)
    print(f"bf16x3 everywhere: max abs {float((base - ref).abs().max()):.3e}")
    print(f"{mode} on layers {sorted(layers)}: max abs {float((got - ref).abs().max()):.3e}")


if __name__ == "__main__":
    main()
