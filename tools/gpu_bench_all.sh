#!/bin/bash
# bench lines for every model / config on one box (each step time-limited; stops on a crash)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
run() {  # name, seconds, args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python bench.py "$@" > "gpurun_out/bench_${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/bench_${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for m in ${MODELS:-hardnet c5 wang2 wang3 wang4 fdl_NASNet fdl_NASNet_01}; do
  if [ "$m" = c5 ]; then run c5 300 --config 5 ${ARGS:-}; else run $m 300 --model $m ${ARGS:-}; fi
done
