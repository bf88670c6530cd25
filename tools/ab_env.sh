#!/bin/bash
# Same-box A/B of environment settings (ENVS: ';'-separated list of "VAR=val VAR2=val" sets;
# "-" = defaults), after a parity subset (PYK, optional).  REPS alternations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -n "${PYK:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYK" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
IFS=';' read -ra SETS <<< "${ENVS:--}"
for r in $(seq ${REPS:-1}); do
  for i in "${!SETS[@]}"; do
    e="${SETS[$i]}"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --model ${MODEL:-hardnet} ${BENCH_ARGS:-} > gpurun_out/ab_env_$i.log 2>&1 || { tail -5 gpurun_out/ab_env_$i.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_env_$i.log').read().strip().splitlines()[-1]);print('[$e]',d['value'],d['roofline']['stages_ms_per_step'])"
  done
done
