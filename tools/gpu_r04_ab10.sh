#!/bin/bash
# Same-box A/B of scratch libraries (LIBS, '-' = the tree's) per model (MODELS), REPS alternations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in $(seq ${REPS:-2}); do
  for m in ${MODELS:-wang2 wang3 wang4}; do
    for lib in ${LIBS:--}; do
      e=""; [ "$lib" != "-" ] && e="HN_LIB=$lib"
      env $e timeout -k 10 200 python bench.py --no-cpu-baseline --model $m > gpurun_out/ab10_$m.log 2>&1 || { tail -5 gpurun_out/ab10_$m.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/ab10_$m.log').read().strip().splitlines()[-1]);print('$m [$e]',d['value'],d['roofline']['stages_ms_per_step'])"
    done
  done
done
