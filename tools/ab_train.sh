cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1; tail -3 gpurun_out/t3.log
for r in 1 2; do for lib in ab/head.so new; do
  if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/$lib; fi
  PAIRS=512 LEGS=hip TRAIN_STEPS=20 timeout -k 10 200 python tools/bench_train.py > gpurun_out/tr_$r_$(basename $lib).log 2>&1 || { tail -5 gpurun_out/tr_$r_$(basename $lib).log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/tr_$r_$(basename $lib).log | cut -c1-300)"
done; done
