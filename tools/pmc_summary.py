"""Per-kernel PMC summary from tools/pmc.sh output: mean counter value per dispatch.
usage: python tools/pmc_summary.py [pmc_dir] [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pats = sys.argv[2:]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pats and not any(p in k for p in pats):
            continue
        k = k.replace("(anonymous namespace)::", "").split("(")[0][:70]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(k)
    for c in sorted(tot[k]):
        n = max(len(disp[k][c]), 1)
        print(f"   {c:28s} {tot[k][c] / n:16.4g}   (per dispatch, {n} dispatches)")
