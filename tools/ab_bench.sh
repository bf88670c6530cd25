#!/bin/bash
# Same-box A/B of environment settings over bench.py lines: ENVS (';'-separated "VAR=val ..." sets, "-" =
# defaults), REPS alternations, BENCH_ARGS for bench.py.  Prints value, ms/step and the stage times (or the
# pair step) of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${ENVS:--}"
for r in $(seq ${REPS:-1}); do
  for i in "${!SETS[@]}"; do
    e="${SETS[$i]}"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra-configs ${BENCH_ARGS:-} > gpurun_out/ab_bench_$i.log 2>&1 || { tail -5 gpurun_out/ab_bench_$i.log; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab_bench_$i.log').read().strip().splitlines()[-1]);r=d['roofline']
print('[$e]', d['config']['model'], d['value'], d['ms_per_step'], d.get('pair_step_ms', ''), r.get('stages_ms_per_step', r.get('forward_stages_ms_per_step')))"
  done
done
