#!/bin/bash
# conv3/conv4/conv5 timing ablations through HN_VARIANT on the experiments library (results wrong by design)
# env: VARS (space-separated HN_VARIANT strings; default: conv4 production f and the ablation digits 8 9 4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export HN_LIB=$PWD/abl/libhardnet_mi355x.so
for r in 1 2; do
  for v in ${VARS:-605gfg 605g8g 605g9g 605g4g}; do
    HN_VARIANT=$v timeout -k 10 150 python bench.py --no-cpu-baseline --no-extra-configs --steps 5 --warmup 2 > gpurun_out/cabl_$v.log 2>&1 || { tail -5 gpurun_out/cabl_$v.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/cabl_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline"]["stages_ms_per_step"]; print(s)')"
  done
done
