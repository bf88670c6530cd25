"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh) into HBM bytes per
launch per bench stage -> profiles/pmc_traffic_<model>.json (read by bench.py).

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports exactly half of the bytes
of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
exact for 16-B-per-lane streaming stores: write bytes = WRITE_SIZE * 1024.
usage: python tools/pmc_traffic.py <pmc dir> <model> <patches processed in the profiled run> [out.json]
Output per stage: HBM bytes per patch (read + write, summed over every launch of the stage), so
bench.py can scale it to its own launch size.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

HARDNET = {(32, 32, 32, 1): "stem+conv1", (32, 32, 32, 0): "conv1", (32, 64, 32, 0): "conv2",
           (64, 64, 16, 0): "conv3", (64, 128, 16, 0): "conv4", (128, 128, 8, 0): "conv5"}


def stage_of(name: str):
    m = re.search(r"k_conv(?:3x3|_pipe|_ws)<(\d+), (\d+), (\d+), \d+, \d+, \d+, \d+, \d+, (true|false)", name)
    if m:
        key = (int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(4) == "true"))
        return HARDNET.get(key)
    m = re.search(r"k_conv_w1<(\d+), (\d+), (\d+),", name)  # 1-D Winograd conv3 / conv5 (hn_wino1.hip)
    if m:
        return {(64, 64, 16): "conv3", (128, 128, 8): "conv5"}.get((int(m.group(1)), int(m.group(2)), int(m.group(3))))
    if "k_c12h<" in name or "k_c12w<" in name or "k_c12s<" in name:
        return "stem+conv1+conv2"
    for k, st in (("k_c12<", "stem+conv1+conv2"), ("k_front<", "front"), ("k_irf<", "irf"),
                  ("k_head<", "head"), ("k_head2<", "head"), ("k_head3<", "head"), ("k_head4<", "head")):
        if k in name:
            return st
    if "k_stem<" in name:
        return "stem"
    for k, st in (("k_pw_tiled<", "pw"), ("k_pw(", "pw"), ("k_dw<", "dw"),
                  ("k_maxpool(", "maxpool"), ("k_se(", "se"), ("k_l2rows(", "head")):
        if k in name:
            return st
    return None


def main():
    d, model, patches = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join("profiles", f"pmc_traffic_{model}.json")
    tot = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            st = stage_of(r["Kernel_Name"])
            if st is None:
                continue
            c = r["Counter_Name"]
            tot[st][c] += float(r["Counter_Value"])
            cnt[st][c].add(r["Dispatch_Id"])
    res = {"patches_profiled": patches}
    for st, cs in tot.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            rd = 2 * cs["FETCH_SIZE"] * 1024
            wr = cs["WRITE_SIZE"] * 1024
            res[st] = {"bytes_per_patch": round((rd + wr) / patches, 1),
                       "read_bytes_per_patch": round(rd / patches, 1),
                       "write_bytes_per_patch": round(wr / patches, 1),
                       "dispatches": len(cnt[st]["FETCH_SIZE"]), "fetch_correction": 2.0}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
