"""A/B the conv tiling variants in one process (cdna_hip_programming.md rule 24):
per-stage device ms per 262,144-patch step for each HN_VARIANT setting, interleaved rounds."""
import os
import sys
import json

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hardnetnas_amd._native import NativeModel  # noqa: E402

variants = sys.argv[1].split(";") if len(sys.argv) > 1 else ["000000", "111111"]
rounds = int(os.environ.get("ROUNDS", "3"))
dev = torch.device("cuda:0")
model = bench.build_model("hardnet")
b = 262144
x = bench.synth_input_on_device(b, dev, 5)
out = torch.empty((b, 128), device=dev)
models = {}
for v in variants:
    os.environ["HN_VARIANT"] = v
    models[v] = NativeModel.from_module(model, dev)
ws = torch.empty(max(m.workspace_bytes(b) for m in models.values()), device=dev, dtype=torch.uint8)
ref = None
res = {v: {} for v in variants}
for rnd in range(rounds):
    for v, nm in models.items():
        nm.forward(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        err = (out - ref).abs().max().item()
        nm.stage_times()
        nm.set_profiling(True)
        nm.forward(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        nm.set_profiling(False)
        st = nm.stage_times()
        for k, (ms, n) in st.items():
            res[v].setdefault(k, []).append(ms)
        res[v].setdefault("total", []).append(sum(ms for ms, _ in st.values()))
        res[v]["maxdiff_vs_first"] = err
for v in variants:
    print(v, json.dumps({k: (round(min(x), 3) if isinstance(x, list) else x) for k, x in res[v].items()}))
