# Same-box A/B of the in-tree library against abl/base.so (HN_LIB), after a parity subset.
# env: PYK (pytest -k filter), MODELS (bench models), REPS (alternations)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -n "${PYK:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYK" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
for r in $(seq ${REPS:-2}); do
  for m in ${MODELS:-hardnet}; do
    for lib in base new; do
      if [ $lib = base ]; then export HN_LIB=$PWD/abl/base.so; else unset HN_LIB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --model $m > gpurun_out/ab_${m}_$lib.log 2>&1 || { tail -5 gpurun_out/ab_${m}_$lib.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/ab_${m}_$lib.log').read().strip().splitlines()[-1]);print('$m','$lib',d['value'],d['roofline']['stages_ms_per_step'])"
    done
  done
done
