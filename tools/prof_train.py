"""The 512-pair HardNet train step of bench.run_train under a profiler: 3 warmup + 10 timed steps; prints wall and
hipEvent ms per step.  Usage: rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x -- python3
tools/prof_train.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hardnetnas_amd.losses import loss_HardNet  # noqa: E402
from hardnetnas_amd.model import HardNet  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
torch.manual_seed(0)
m = HardNet().to(dev).train()
opt = torch.optim.SGD(m.features.parameters(), lr=1.0, momentum=0.9, dampening=0.9, weight_decay=1e-4)
b = bench.TRAIN_PAIRS
xa = bench.synth_input_on_device(b, dev, seed=31)
xp = xa + 0.3 * bench.synth_input_on_device(b, dev, seed=32)


def step():
    loss = loss_HardNet(m(xa), m(xp), anchor_swap=True)
    opt.zero_grad()
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(10):
    step()
e1.record()
torch.cuda.synchronize()
print("wall ms/step %.3f  event ms/step %.3f" % ((time.perf_counter() - t0) / 10 * 1e3, e0.elapsed_time(e1) / 10))
