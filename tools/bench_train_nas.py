"""Train steps of hardnetNAS on MI355X: the sampled descriptor (wang2) and FDLNet's
HardNetNeiMask (both variants) in the supernet
training loop's shape (two train() calls, loss_HardNet with anchor swap, backward, SGD) and the supernet search
step itself (training_functions_supernet.py:88-103: outs_X with grad, outs_Y under no_grad, SupernetLoss,
backward, SGD on the weights), on the HIP kernels (hn_nas_train_*) vs the same modules' torch layers on the same
GPU (MIOpen).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hardnetnas_amd.losses import SupernetLoss, loss_HardNet  # noqa: E402
from hardnetnas_amd.model import HardNetNAS, HardNetNASSupernet, HardNetNeiMask  # noqa: E402

dev = torch.device("cuda:0")
steps = int(os.environ.get("TRAIN_STEPS", "5"))
res = {}
PAIRS = int(os.environ.get("PAIRS", "512"))
for what, pairs in (("wang2", PAIRS), ("supernet", int(os.environ.get("SPAIRS", "128"))), ("fdl_NASNet", PAIRS),
                    ("fdl_NASNet_0.1", PAIRS)):
    res[what] = {"pairs": pairs}
    for name, native in (("hip", True), ("torch_miopen", False)):
        torch.manual_seed(0)
        m = (HardNetNAS("wang2") if what == "wang2" else HardNetNASSupernet() if what == "supernet"
             else HardNetNeiMask(variant=what[4:])).to(dev).train()
        m.native_train = native
        opt = torch.optim.SGD([p for n, p in m.named_parameters() if not n.endswith("thetas")], lr=0.01,
                              momentum=0.9, weight_decay=1e-4)
        xa = torch.randn(pairs, 1, 32, 32, device=dev)
        xp = xa + 0.5 * torch.randn(pairs, 1, 32, 32, device=dev)
        crit = SupernetLoss()

        def step():
            opt.zero_grad()
            if what != "supernet":
                loss = loss_HardNet(m(xa), m(xp), anchor_swap=True)
            else:
                lat0 = torch.zeros(1, 1, device=dev, requires_grad=True)
                ox, lacc, soft, _ = m(xa, 5.0, lat0)
                with torch.no_grad():
                    oy, _, _, _ = m(xp, 5.0, lacc)
                loss = crit(ox, oy, lacc, soft, 15.0)[0]
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
        res[what][name] = {"ms_per_step": round(ms, 2), "patches_per_s": round(2 * pairs / ms * 1e3, 1)}
    res[what]["speedup"] = round(res[what]["torch_miopen"]["ms_per_step"] / res[what]["hip"]["ms_per_step"], 2)
print(json.dumps(res))
