# Same-box A/B of the in-tree library against other builds (HN_LIB), after a parity subset.
# env: PYK (pytest -k filter), MODELS (bench models), REPS (alternations),
#      LIBS (space-separated .so paths relative to the repo, "new" = in-tree; default "abl/base.so new")
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -n "${PYK:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYK" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
for r in $(seq ${REPS:-2}); do
  for m in ${MODELS:-hardnet}; do
    for lib in ${LIBS:-abl/base.so new}; do
      if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/$lib; fi
      tag=$(basename $lib .so)
      timeout -k 10 200 python bench.py --no-cpu-baseline --model $m ${BENCH_ARGS:-} > gpurun_out/ab_${m}_$tag.log 2>&1 || { tail -5 gpurun_out/ab_${m}_$tag.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/ab_${m}_$tag.log').read().strip().splitlines()[-1]);print('$m','$tag',d['value'],d['roofline']['stages_ms_per_step'])"
    done
  done
done
