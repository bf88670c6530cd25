#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per counter group; --kernel-trace only, no
# sys/runtime tracing) over a small bench workload.  Output: gpurun_out/pmc/<tag>/...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
MODEL=${MODEL:-hardnet}
ARGS="--no-cpu-baseline --steps 1 --warmup 1 --batch ${PMC_BATCH:-32768} --model $MODEL ${PMC_EXTRA:-}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
while IFS= read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "== pass $i: $group"
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done < "${PMC_GROUPS:-tools/pmc_groups.txt}"
