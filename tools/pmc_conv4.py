"""Summary of tools/pmc_conv4.sh: per configuration and kernel (conv4 = k_conv_ws<64, 128, ...>, plus the others of
the step), the mean dispatch duration (kernel trace), GRBM_GUI_ACTIVE cycles per dispatch and the clock they imply,
and the TLB / TA / L2 counters per dispatch."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_conv4"
SHORT = {"k_c12s": "c12s", "k_conv_w1<64": "conv3", "k_conv_ws<64, 128": "conv4", "k_conv_w1<128": "conv5",
         "k_head4": "head"}


def short(k):
    for s, v in SHORT.items():
        if s in k:
            return v
    return None


for cfg in ("big", "small"):
    dur = collections.defaultdict(list)
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    for p in sorted(glob.glob(f"{root}/{cfg}_p*")):
        for f in glob.glob(f"{p}/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if k:
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
        for f in glob.glob(f"{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if k:
                    cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    ndisp[(k, p)].add(r["Dispatch_Id"])
    print(f"== {cfg}")
    for k in ("c12s", "conv3", "conv4", "conv5", "head"):
        if k not in dur:
            continue
        d = sum(dur[k]) / len(dur[k])
        n = max(len(ndisp[(k, p)]) for p in glob.glob(f"{root}/{cfg}_p*"))
        c = {a: b / n / 2 if a == "GRBM_GUI_ACTIVE" else b / n for a, b in cnt[k].items()}  # GRBM in both passes
        ghz = c.get("GRBM_GUI_ACTIVE", 0) / (d * 1e3) if d else 0
        print(f"  {k:6s} {len(dur[k])} disp, {d:8.1f} us; GRBM_GUI_ACTIVE/disp {c.get('GRBM_GUI_ACTIVE', 0):.4g} -> {ghz:.3f} GHz")
        for a in sorted(c):
            if a != "GRBM_GUI_ACTIVE":
                print(f"      {a:36s} {c[a]:.4g}")
