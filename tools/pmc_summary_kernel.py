"""Sum rocprofv3 --pmc counter rows per kernel (tools/pmc_kernels.sh output): python tools/pmc_summary_kernel.py
<dir with p*/run_counter_collection.csv> [kernel-substring ...]; prints each matching kernel's counter totals and the
derived LDS bank-conflict share, VALU / MFMA instructions per dispatch."""
import collections
import csv
import glob
import sys

root, pats = sys.argv[1], sys.argv[2:] or [""]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if any(s in k for s in pats):
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r.get("Dispatch_Id")))
for k, v in tot.items():
    n = max(1, len({d for _, d in disp[k]}))
    print(k[:100])
    for c in sorted(v):
        print(f"  {c:28s} {v[c]:.4g}")
    if v.get("SQ_LDS_IDX_ACTIVE"):
        print(f"  bank-conflict share of LDS cycles: {v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE']:.3f}")
