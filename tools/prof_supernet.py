"""One supernet search step under a profiler: 2 warmup + 5 timed steps of bench.run_train_supernet's step at the
reference's 128 pairs (no CPU baseline).  Usage: rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3
tools/prof_supernet.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
m, opt, crit, xa, xp = bench._supernet_setup(dev, bench.SUPERNET_PAIRS)
for _ in range(2):
    bench._supernet_step(m, opt, crit, xa, xp, dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    bench._supernet_step(m, opt, crit, xa, xp, dev)
torch.cuda.synchronize()
print("ms/step", (time.perf_counter() - t0) / 5 * 1e3)
