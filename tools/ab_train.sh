cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
[ -n "${NOTEST:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abt_pytest.log 2>&1 || { tail -30 gpurun_out/abt_pytest.log; exit 1; }
tail -1 gpurun_out/abt_pytest.log
for r in 1 2 3; do
  for lib in ${LIBS:-abl/base.so new}; do
    if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/$lib; fi
    LEGS=hip timeout -k 10 200 python tools/bench_train.py > gpurun_out/abt_${r}_$(basename $lib .so).log 2>&1 || { tail -5 gpurun_out/abt_${r}_$(basename $lib .so).log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/abt_${r}_$(basename $lib .so).log)"
  done
done
