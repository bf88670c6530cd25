#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for HardNet and wang2 -> gpurun_out/pmc_{hardnet,wang2}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for M in hardnet wang2; do
  mkdir -p gpurun_out/pmc_$M
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_$M/p$i -o run --output-format csv -- \
      python bench.py --no-cpu-baseline --steps 1 --warmup 1 --batch 32768 --model $M > gpurun_out/pmc_$M/p$i.log 2>&1 || exit $?
  done
done
