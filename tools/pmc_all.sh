#!/bin/bash
# Per-stage PMC passes (tools/pmc_groups_stage.txt: FETCH_SIZE, WRITE_SIZE, then the SQ instruction
# / busy counters; one rocprofv3 --pmc pass each, --kernel-trace only) for each model, then
# tools/pmc_stage.py -> gpurun_out/pmc_<model>.json (copy to profiles/ for bench.py's roofline).
# hardnet / NAS: batch 65,536 (k_head4 runs) x (1 warmup + 1 timed step) = 131,072 patches; c5: the config-5 pair
# step at 65,536 pairs x 2 launches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for M in ${MODELS:-hardnet wang2 wang3 wang4 c5}; do
  rm -rf gpurun_out/pmc_$M; mkdir -p gpurun_out/pmc_$M
  if [ "$M" = c5 ]; then ARGS="--config 5 --batch 65536"; UNITS=131072; else ARGS="--model $M --batch 65536"; UNITS=131072; fi
  i=0
  while IFS= read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    echo "== $M pass $i: $group"
    timeout -k 10 150 rocprofv3 --pmc $group --kernel-trace -d gpurun_out/pmc_$M/p$i -o run --output-format csv -- \
      python bench.py --no-cpu-baseline --steps 1 --warmup 1 $ARGS > gpurun_out/pmc_$M/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_$M/p$i.log; exit 1; }
  done < tools/pmc_groups_stage.txt
  python tools/pmc_stage.py gpurun_out/pmc_$M $M $UNITS gpurun_out/pmc_$M.json > /dev/null || exit 1
done
