#!/bin/bash
# Same-box A/B of HN_TRAIN_* settings on the 512-pair train step (tools/bench_train.py, HIP leg): ENVS as tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${ENVS:--}"
for r in $(seq ${REPS:-2}); do
  for i in "${!SETS[@]}"; do
    e="${SETS[$i]}"; [ "$e" = "-" ] && e=""
    env $e PAIRS=${PAIRS:-512} LEGS=hip TRAIN_STEPS=20 timeout -k 10 200 python tools/bench_train.py > gpurun_out/abtr_$i.log 2>&1 || { tail -5 gpurun_out/abtr_$i.log; exit 1; }
    echo "[$e] $(tail -1 gpurun_out/abtr_$i.log | cut -c1-200)"
  done
done
