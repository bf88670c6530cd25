#!/bin/bash
# k_c12 phase ablations (HN_C12_ABL bits: 1 = no stem MFMA, 2 = no conv1 MFMA, 4 = no conv2 MFMA)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for a in ${ABLS:-0 1 2 4 6 7}; do
  HN_LIB=abl/libhardnet_mi355x.so   HN_C12_CFG=${CFG:-0} HN_C12_ABL=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abl_$a.log 2>&1 || exit 1
  echo "abl=$a $(tail -1 gpurun_out/abl_$a.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["stages_ms_per_step"]["stem+conv1+conv2"])')"
done
