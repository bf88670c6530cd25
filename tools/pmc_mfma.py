"""MFMA-busy fraction per kernel from a tools/pmc.sh pass over tools/pmc_groups_mfma.txt.

  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)

(SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD, GRBM_GUI_ACTIVE over the 8 XCDs; both per
dispatch.)  usage: python tools/pmc_mfma.py <pmc_dir> <out.json> [model]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
model = sys.argv[3] if len(sys.argv) > 3 else ""
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k.startswith("void at::") or "rocclr" in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
res = {"model": model, "formula": __doc__.split("\n\n")[1].strip(), "kernels": {}}
for k, c in tot.items():
    mean = {n: v / max(len(disp[k][n]), 1) for n, v in c.items()}
    active = mean.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    busy = mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    res["kernels"][k] = {
        "dispatches": max(len(s) for s in disp[k].values()),
        "gpu_cycles_per_dispatch": round(active),
        "mfma_busy": round(busy / (active * 256 * 4), 4) if active else None,
        "mfma_insts_per_dispatch": round(mean.get("SQ_INSTS_MFMA", 0.0)),
        "valu_insts_per_dispatch": round(mean.get("SQ_INSTS_VALU", 0.0)),
    }
json.dump(res, open(out, "w"), indent=1)
for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["gpu_cycles_per_dispatch"]):
    print(f"{v['mfma_busy']!s:8} {v['gpu_cycles_per_dispatch']:>10} {k[:90]}")
