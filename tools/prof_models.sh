#!/bin/bash
# rocprofv3 kernel stats of bench.py for MODELS (default wang2 wang4): top kernels by total time
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODELS:-wang2 wang4}; do
  rm -rf gpurun_out/prof_$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-extra-configs --model $m ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/prof_$m.log 2>&1 || { tail -5 gpurun_out/prof_$m.log; exit 1; }
done
for m in ${MODELS:-wang2 wang4}; do
  f=$(find gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1)
  echo "== $m"
  python tools/top_kernels.py "$f"
done
