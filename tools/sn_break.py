import os, sys, time, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
m, opt, crit, xa, xp = bench._supernet_setup(dev, 128)
for _ in range(3): bench._supernet_step(m, opt, crit, xa, xp, dev)
torch.cuda.synchronize()
def t(f, n=5):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): r = f()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
import torch.nn.functional as F
sw = torch.stack([F.gumbel_softmax(st.thetas, 5.0) for st in m.stages_to_search]).detach()
lat0 = torch.zeros(1, 1, device=dev)
print("latency terms only", t(lambda: [st.latency_terms(sw[i], lat0) for i, st in enumerate(m.stages_to_search)]))
with torch.no_grad():
    print("no_grad forward (native)", t(lambda: m(xa, 5.0, lat0)))
    print("no_grad forward given soft", t(lambda: m(xa, 5.0, lat0, sw)))
print("step", t(lambda: bench._supernet_step(m, opt, crit, xa, xp, dev)))
def fb():
    ox, l, s, _ = m(xa, 5.0, lat0, sw)
    ox.sum().backward()
print("fwd+bwd given soft", t(fb))
# GPU-only time of a forward via events
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.no_grad():
    e0.record(); m(xa, 5.0, lat0, sw); e1.record(); torch.cuda.synchronize(); print("fwd event ms", e0.elapsed_time(e1))
