"""Per-stage PMC summary of a tools/pmc.sh run over tools/pmc_groups_stage.txt ->
profiles/pmc_<model>.json, which bench.py reads for the roofline's `traffic` and the NAS roofs.

Per bench stage (the names hn_stage_times reports), per patch (per launch for config 5's pair kernel):
  bytes      HBM read + write: read = 2 * FETCH_SIZE * 1024 (gfx950: FETCH_SIZE counts half of the
             bytes of a wide coalesced streaming read, MI355X_MICROARCH.md HBM section), write =
             WRITE_SIZE * 1024; separate --pmc passes (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
  valu / mfma instructions  SQ_INSTS_VALU (MFMAs included) / SQ_INSTS_MFMA, wave-instructions
  mfma_busy  SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1,024 SIMDs)
  valu_busy  SQ_ACTIVE_INST_VALU * 4 (quad-cycles) / (GRBM_GUI_ACTIVE / 8 * 1,024 SIMDs)
usage: python tools/pmc_stage.py <pmc dir> <model|c5> <patches (or pairs for c5) per profiled run> [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import stage_of  # noqa: E402


def stage(name: str):
    if "k_pairdist_rows<" in name or "k_pairdist_ring<" in name:
        return "pairdist"
    if "k_irf3<" in name:
        return "irf3"
    if "k_irf2<" in name:
        return "irf2"
    if "k_irf_skip<" in name:
        return "irf+skip"
    if "k_mpfront_irf<" in name:
        return "front+irf"
    if "k_head_fin<" in name:
        return "head"
    if "k_skip_s2<" in name or "k_skip_s2(" in name:
        return "skip"
    if "k_fdl_front" in name:
        return "front"
    return stage_of(name)


def main():
    d, model, units = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join("profiles", f"pmc_{model}.json")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    kernels = defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            st = stage(r["Kernel_Name"])
            if st is None:
                continue
            c = r["Counter_Name"]
            tot[st][c] += float(r["Counter_Value"])
            disp[st][c].add(r["Dispatch_Id"])
            kernels[st].add(r["Kernel_Name"].split("(")[0].replace("void ", ""))
    res = {"model": model, "units_profiled": units, "unit": "pair" if model == "c5" else "patch",
           "formula": __doc__.split("\n\n")[1].strip(), "stages": {}}
    per = "pair" if model == "c5" else "patch"
    for st, cs in tot.items():
        e = {"kernels": sorted(kernels[st]), "dispatches": max(len(v) for v in disp[st].values())}
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            rd, wr = 2 * cs["FETCH_SIZE"] * 1024, cs["WRITE_SIZE"] * 1024
            e.update({f"bytes_per_{per}": round((rd + wr) / units, 2), f"read_bytes_per_{per}": round(rd / units, 2),
                      f"write_bytes_per_{per}": round(wr / units, 2), "fetch_correction": 2.0})
        if "SQ_INSTS_VALU" in cs:
            e[f"valu_insts_per_{per}"] = round(cs["SQ_INSTS_VALU"] / units, 3)
            e[f"mfma_insts_per_{per}"] = round(cs.get("SQ_INSTS_MFMA", 0.0) / units, 3)
        g = cs.get("GRBM_GUI_ACTIVE", 0.0)
        if g:
            simd_cycles = g / 8.0 * 1024
            e["mfma_busy"] = round(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles, 4)
            e["valu_busy"] = round(4 * cs.get("SQ_ACTIVE_INST_VALU", 0.0) / simd_cycles, 4)
            e["gpu_cycles_per_dispatch"] = round(g / 8.0 / max(len(disp[st]["GRBM_GUI_ACTIVE"]), 1))
        res["stages"][st] = e
    if model == "c5":  # one pair-kernel launch per profiled step: bytes per launch at this batch
        pd = res["stages"].get("pairdist")
        if pd and "bytes_per_pair" in pd:
            n = pd["dispatches"]
            res["pairs"] = units // max(n, 1)
            res["pairdist"] = {"bytes_per_launch": round(pd["bytes_per_pair"] * units / max(n, 1))}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
