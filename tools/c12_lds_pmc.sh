#!/bin/bash
# k_c12s LDS bank conflicts per phase ablation: one rocprofv3 --pmc pass (LDS counters only) per HN_C12_ABL
# value of the experiments library (ABLS, default "64 72 80 88 84"), summarised by tools/pmc_summary-like
# parsing into gpurun_out/c12_lds_pmc.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export HN_LIB=abl/libhardnet_mi355x.so HN_C12_CFG=15
: > gpurun_out/c12_lds_pmc.txt
for a in ${ABLS:-64 72 80 88 84}; do
  rm -rf gpurun_out/c12lds_$a
  HN_C12_ABL=$a timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace \
    -d gpurun_out/c12lds_$a -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 --batch 65536 \
    > gpurun_out/c12lds_$a.log 2>&1 || { tail -5 gpurun_out/c12lds_$a.log; exit 1; }
  python3 - "$a" >> gpurun_out/c12_lds_pmc.txt <<'PY'
import csv, glob, sys, collections
a = sys.argv[1]
f = glob.glob(f"gpurun_out/c12lds_{a}/**/run_counter_collection.csv", recursive=True)[0]
v = collections.defaultdict(float); d = set()
for r in csv.DictReader(open(f)):
    if "k_c12s" in r["Kernel_Name"]:
        v[r["Counter_Name"]] += float(r["Counter_Value"]); d.add(r["Dispatch_Id"])
n = max(1, len(d))
print(f"abl {a}: dispatches {len(d)} conflict {v['SQ_LDS_BANK_CONFLICT']/n:.3e} idx {v['SQ_LDS_IDX_ACTIVE']/n:.3e} "
      f"insts {v['SQ_INSTS_LDS']/n:.3e} conflict/idx {v['SQ_LDS_BANK_CONFLICT']/max(1,v['SQ_LDS_IDX_ACTIVE']):.3f} "
      f"gui {v['GRBM_GUI_ACTIVE']/n:.3e}")
PY
done
cat gpurun_out/c12_lds_pmc.txt
