"""hn_preprocess throughput on device-resident uint8 64x64 patches.

HBM-bound byte work: 4,096 B read + 4,096 B written per patch (algorithmic).  Reports the
hipEvent-timed kernel rate against the 8 TB/s HBM3E peak.  Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hardnetnas_amd._native import preprocess  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=262144)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
u = torch.randint(0, 256, (args.batch, 64, 64), device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
out = torch.empty((args.batch, 1, 32, 32), device=dev)
res = {"batch": args.batch, "bytes_per_patch": 8192, "peak_GBps": 8000}
for mode in ("cv2", "pil"):
    for _ in range(3):
        preprocess(u, resize=mode, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.steps):
        preprocess(u, resize=mode, out=out)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.steps
    gbps = args.batch * 8192 / (ms * 1e-3) / 1e9
    res[mode] = {"ms": round(ms, 4), "GBps": round(gbps, 1), "frac": round(gbps / 8000, 4),
                 "mpatches_per_s": round(args.batch / ms / 1e3, 1)}
print(json.dumps(res))
