#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 pass, --kernel-trace only) for each
# model -> gpurun_out/pmc_<model>; then tools/pmc_traffic.py <dir> <model> 65536 (batch 32,768
# x (1 warmup + 1 timed step)) writes gpurun_out/pmc_traffic_<model>.json (copy it to profiles/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for M in ${MODELS:-hardnet wang2 wang3 wang4}; do
  rm -rf gpurun_out/pmc_$M; mkdir -p gpurun_out/pmc_$M
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_$M/p$i -o run --output-format csv -- \
      python bench.py --no-cpu-baseline --steps 1 --warmup 1 --batch 32768 --model $M > gpurun_out/pmc_$M/p$i.log 2>&1 || exit $?
  done
  python tools/pmc_traffic.py gpurun_out/pmc_$M $M 65536 gpurun_out/pmc_traffic_$M.json || exit $?
done
