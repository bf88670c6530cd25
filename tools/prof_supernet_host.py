"""Host-side profile of the supernet search step (bench._supernet_step at 128 pairs): cProfile of 5 steps after
warm-up, top functions by cumulative and own time, plus wall and hipEvent ms per step."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
m, opt, crit, xa, xp = bench._supernet_setup(dev, bench.SUPERNET_PAIRS)
for _ in range(3):
    bench._supernet_step(m, opt, crit, xa, xp, dev)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(5):
    bench._supernet_step(m, opt, crit, xa, xp, dev)
e1.record()
torch.cuda.synchronize()
print("wall ms/step %.2f event ms/step %.2f" % ((time.perf_counter() - t0) / 5 * 1e3, e0.elapsed_time(e1) / 5))
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    bench._supernet_step(m, opt, crit, xa, xp, dev)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
