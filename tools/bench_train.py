"""Train step of the stock HardNet: model.train() forward + loss_HardNet
(anchor_swap, triplet margin) + backward + SGD step at the reference's batch of 1024 pairs
(hardnet/HardNet.py:379-441: out_a = model(data_a); out_p = model(data_p), 2 x 1024 patches per step), on the HIP train kernels vs the same
module's torch layers on the same GPU (MIOpen).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hardnetnas_amd.losses import loss_HardNet  # noqa: E402
from hardnetnas_amd.model import HardNet  # noqa: E402

dev = torch.device("cuda:0")
pairs = int(os.environ.get("PAIRS", "1024"))
steps = int(os.environ.get("TRAIN_STEPS", "10"))
legs = os.environ.get("LEGS", "hip,torch_miopen").split(",")  # LEGS=hip: profile the HIP leg alone
res = {"config": f"HardNet train step, {pairs} pairs ({2 * pairs} patches), loss_HardNet + SGD"}
for name, native in (("hip", True), ("torch_miopen", False)):
    if name not in legs:
        continue
    torch.manual_seed(0)
    m = HardNet().to(dev).train()
    m.native_train = native
    opt = torch.optim.SGD(m.features.parameters(), lr=0.1, momentum=0.9, dampening=0.9, weight_decay=1e-4)
    xa = torch.randn(pairs, 1, 32, 32, device=dev)
    xp = xa + 0.5 * torch.randn(pairs, 1, 32, 32, device=dev)

    def step():  # the reference loop's shape: two model calls, HardNet.py:392-393
        out_a = m(xa)
        out_p = m(xp)
        loss = loss_HardNet(out_a, out_p, anchor_swap=True)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    res[name] = {"ms_per_step": round(ms, 2), "patches_per_s": round(2 * pairs / ms * 1e3, 1)}
print(json.dumps(res))
