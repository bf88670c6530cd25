#!/bin/bash
# One GPU session on the gpurun box: tests, smoke, bench, rocprof kernel stats, PMC passes.
# Each GPU step has its own time limit; a crash/abort/timeout (exit not 0 or 1) stops the
# session, test failures (exit 1) do not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
[[ $STEPS == *pytest* ]] && run pytest_gpu 500 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *smoke* ]] && run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 300 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
[[ $STEPS == *prof* ]] && run rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 20 --warmup 5}
[[ $STEPS == *pmc* ]] && run pmc 900 bash tools/pmc_all.sh
[[ $STEPS == *pre* ]] && run bench_pre 200 python tools/bench_preprocess.py
[[ $STEPS == *pairs* ]] && run bench_pairs 200 python tools/bench_pairs.py
[[ $STEPS == *train* ]] && run bench_train 200 python tools/bench_train.py
exit 0
