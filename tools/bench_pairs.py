"""BASELINE config 5: HardNet forward of B anchor/positive pairs (2B patches, matching the
reference train step hardnet/HardNet.py:392-393) + the fused distance_matrix_vector +
hardest-negative reduction (hardnet/Losses.py:87-154) without materialising the BxB matrix.
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hardnetnas_amd._native import NativeModel, pairdist_hardneg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=65536)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--warmup", type=int, default=2)
args = ap.parse_args()
dev = torch.device("cuda:0")
b = args.pairs
nm = NativeModel.from_module(bench.build_model("hardnet"), dev)
xa = bench.synth_input_on_device(b, dev, 1)
xp = (xa + 0.3 * torch.randn_like(xa)).contiguous()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]


def step():
    ev[0].record()
    a = nm(xa)
    p = nm(xp)
    ev[1].record()
    pos, mn = pairdist_hardneg(a, p, anchor_swap=True)
    ev[2].record()
    return pos, mn


for _ in range(args.warmup):
    step()
torch.cuda.synchronize()
fwd_ms, pd_ms = 0.0, 0.0
t0 = time.perf_counter()
for _ in range(args.steps):
    pos, mn = step()
    torch.cuda.synchronize()
    fwd_ms += ev[0].elapsed_time(ev[1])
    pd_ms += ev[1].elapsed_time(ev[2])
el = time.perf_counter() - t0
pair_flop = 2.0 * b * b * 128
print(json.dumps({"config": "HardNet forward of %d pairs + fused distance/hardest-negative" % b,
                  "ms_per_step": round(el / args.steps * 1e3, 3),
                  "forward_ms": round(fwd_ms / args.steps, 3),
                  "pairdist_ms": round(pd_ms / args.steps, 3),
                  "pairdist_tflops": round(pair_flop / (pd_ms / args.steps * 1e-3) / 1e12, 2),
                  "mpatches_per_s": round(2 * b / (el / args.steps) / 1e6, 4),
                  "loss_triplet_margin": float(torch.clamp(1.0 + pos - mn, min=0).mean())}))
